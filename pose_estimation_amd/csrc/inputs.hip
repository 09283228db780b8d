// On-GPU input construction of the KRRN eval path, replacing the numpy
// per-sample work of PoseDataset._load_data (dataset/linemod/batchdataset.py:603-771) for a
// batch of crops of one square size S (the host snaps the boxes, get_square_bbox :890-961):
//
//   krrn_crop_inputs_u8   img_croped = Normalize(img[rmin:rmax, cmin:cmax] / 255.) (:722, 744;
//                         ImageNet mean / std, :70) as NCHW f32, and the crop's point mask =
//                         mask_label * mask_depth (* mask_obj when given) (:662-666)
//   krrn_choose_points    choose = the mask pixels in row-major order (:667), a uniformly random
//                         order-preserving subset of N when there are more (:668-673), wrap-padded
//                         to N when fewer (:675-679); then x/y_map_choosed (full-frame column / row,
//                         :712-715) and the back-projected cloud (:714-721)
//
// One workgroup per crop for choose: block-wide ballot scans keep the row-major order, and the
// random subset is the N smallest of per-rank 32-bit hash keys found by a 4-pass radix select
// (ties broken by rank), so no sort and no workspace. The reference draws the subset with
// numpy's global RNG (np.random.shuffle); this one is a counter hash of (seed, crop, rank):
// the same distribution, not the same draw.
#include "krrn_common.h"

namespace {

constexpr int kChooseThreads = 1024;
constexpr int kChooseWaves = kChooseThreads / 64;

__device__ __forceinline__ unsigned mix32(unsigned long long x) {
  // splitmix64 finaliser, high half
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (unsigned)(x >> 32);
}

__global__ __launch_bounds__(256) void crop_inputs_kernel(const unsigned char* __restrict__ rgb,
                                                          const float* __restrict__ depth,
                                                          const unsigned char* __restrict__ mlabel,
                                                          const unsigned char* __restrict__ mobj, int H, int W,
                                                          const int* __restrict__ frame, const int* __restrict__ rc,
                                                          int S, float* __restrict__ img,
                                                          unsigned char* __restrict__ mask) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= S * S) return;
  const int r = p / S, c = p - (p / S) * S;
  const int row = rc[2 * b] + r, col = rc[2 * b + 1] + c;
  const size_t f = (size_t)frame[b];
  const size_t fp = (f * H + row) * W + col;
  // torchvision Normalize on float32(u8 / 255.) (the division in f64, as numpy does it)
  const float mean[3] = {0.485f, 0.456f, 0.406f};
  const float stdv[3] = {0.229f, 0.224f, 0.225f};
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float x = (float)((double)rgb[fp * 3 + ch] / 255.0);
    img[((size_t)b * 3 + ch) * S * S + p] = (x - mean[ch]) / stdv[ch];
  }
  const bool m = mlabel[fp] != 0 && depth[fp] != 0.f && (!mobj || mobj[fp] != 0);
  mask[(size_t)b * S * S + p] = m ? 1 : 0;
}

// exclusive prefix of a 0/1 flag over the block (thread order), and the block total
__device__ __forceinline__ int block_excl_scan(bool flag, int* wsum, int& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long bal = __ballot(flag);
  const int in_wave = __popcll(bal & ((1ull << lane) - 1ull));
  __syncthreads();
  if (lane == 0) wsum[wave] = __popcll(bal);
  __syncthreads();
  int before = 0;
  total = 0;
  for (int w = 0; w < kChooseWaves; ++w) {
    const int v = wsum[w];
    before += (w < wave) ? v : 0;
    total += v;
  }
  return before + in_wave;
}

__global__ __launch_bounds__(kChooseThreads) void choose_points_kernel(
    const unsigned char* __restrict__ mask, int S, int N, const float* __restrict__ depth, int H, int W,
    const int* __restrict__ frame, const int* __restrict__ rc, const float* __restrict__ K4, float depth_scale,
    const long long* __restrict__ seed, int stream_id, long long* __restrict__ choose, float* __restrict__ cloud,
    float* __restrict__ xmap, float* __restrict__ ymap, int* __restrict__ count_out) {
  __shared__ int wsum[kChooseWaves];
  __shared__ int hist[256];
  __shared__ int sel_state[2];  // threshold key, ties to take
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int SS = S * S;
  const unsigned char* mb = mask + (size_t)b * SS;
  const unsigned long long base = ((unsigned long long)seed[0] * 0x9E3779B97F4A7C15ull) ^
                                  ((unsigned long long)(stream_id + 1) << 48) ^ ((unsigned long long)b << 24);

  // pass A: number of mask pixels
  int count = 0;
  for (int p0 = 0; p0 < SS; p0 += kChooseThreads) {
    const int p = p0 + tid;
    int tot;
    block_excl_scan(p < SS && mb[p] != 0, wsum, tot);
    count += tot;
  }
  if (tid == 0) count_out[b] = count;
  if (count == 0) {  // the reference drops such a sample (choose error, :679-681); zeros here
    for (int j = tid; j < N; j += kChooseThreads) {
      choose[(size_t)b * N + j] = 0;
      xmap[(size_t)b * N + j] = 0.f;
      ymap[(size_t)b * N + j] = 0.f;
      cloud[((size_t)b * N + j) * 3 + 0] = 0.f;
      cloud[((size_t)b * N + j) * 3 + 1] = 0.f;
      cloud[((size_t)b * N + j) * 3 + 2] = 0.f;
    }
    return;
  }

  // radix select: the N-th smallest key over ranks [0, count)
  unsigned thr = 0xFFFFFFFFu;
  int need = N;
  const bool subset = count > N;
  if (subset) {
    unsigned prefix = 0, pmask = 0;
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = 24 - 8 * pass;
      for (int i = tid; i < 256; i += kChooseThreads) hist[i] = 0;
      __syncthreads();
      for (int i = tid; i < count; i += kChooseThreads) {
        const unsigned k = mix32(base + (unsigned long long)i);
        if ((k & pmask) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1);
      }
      __syncthreads();
      if (tid == 0) {
        int acc = 0, d = 0;
        for (; d < 256; ++d) {
          if (acc + hist[d] >= need) break;
          acc += hist[d];
        }
        sel_state[0] = d;
        sel_state[1] = need - acc;
      }
      __syncthreads();
      prefix |= (unsigned)sel_state[0] << shift;
      pmask |= 255u << shift;
      need = sel_state[1];
      __syncthreads();
    }
    thr = prefix;  // keys < thr all taken, plus the first `need` ranks with key == thr
  }

  // pass B: selected mask pixels in row-major order
  int rank0 = 0, tie0 = 0, out0 = 0;
  long long* cb = choose + (size_t)b * N;
  for (int p0 = 0; p0 < SS; p0 += kChooseThreads) {
    const int p = p0 + tid;
    const bool m = p < SS && mb[p] != 0;
    int tot;
    const int r = rank0 + block_excl_scan(m, wsum, tot);
    rank0 += tot;
    bool take = m, tie = false;
    unsigned k = 0;
    if (subset && m) {
      k = mix32(base + (unsigned long long)r);
      take = k < thr;
      tie = k == thr;
    }
    int ttot;
    const int tr = tie0 + block_excl_scan(tie, wsum, ttot);
    tie0 += ttot;
    take = take || (tie && tr < need);
    int stot;
    const int slot = out0 + block_excl_scan(take, wsum, stot);
    out0 += stot;
    if (take && slot < N) cb[slot] = p;
  }
  __syncthreads();
  // wrap padding (np.pad(..., 'wrap')): slot j >= count repeats slot j % count
  for (int j = count + tid; j < N; j += kChooseThreads) cb[j] = cb[j % count];
  __syncthreads();

  // chosen pixels -> full-frame maps and the back-projected cloud, float32 arithmetic in the
  // reference's order: pt2 = depth / scale; pt0 = (x - cx) * pt2 / fx; pt1 = (y - cy) * pt2 / fy
  const float fx = K4[4 * b + 0], fy = K4[4 * b + 1], cx = K4[4 * b + 2], cy = K4[4 * b + 3];
  const size_t f = (size_t)frame[b];
  for (int j = tid; j < N; j += kChooseThreads) {
    const int p = (int)cb[j];
    const int row = rc[2 * b] + p / S, col = rc[2 * b + 1] + p % S;
    const float xm = (float)col, ym = (float)row;
    const float pt2 = depth[(f * H + row) * W + col] / depth_scale;
    xmap[(size_t)b * N + j] = xm;
    ymap[(size_t)b * N + j] = ym;
    float* o = cloud + ((size_t)b * N + j) * 3;
    o[0] = (xm - cx) * pt2 / fx;
    o[1] = (ym - cy) * pt2 / fy;
    o[2] = pt2;
  }
}

}  // namespace

KRRN_API int krrn_crop_inputs_u8(const unsigned char* rgb, const float* depth, const unsigned char* mask_label,
                                 const unsigned char* obj_mask, int F, int H, int W, const int* frame, const int* rc,
                                 int B, int S, float* img, unsigned char* mask, void* stream) {
  if (!rgb || !depth || !mask_label || !frame || !rc || !img || !mask) return KRRN_EARG;
  if (F < 1 || H < 1 || W < 1 || B < 1 || S < 1 || S > H || S > W || B > 65535) return KRRN_ESHAPE;
  hipLaunchKernelGGL(crop_inputs_kernel, dim3(krrn_cdiv(S * S, 256), B), dim3(256), 0, (hipStream_t)stream, rgb,
                     depth, mask_label, obj_mask, H, W, frame, rc, S, img, mask);
  return krrn_launch_status();
}

KRRN_API int krrn_choose_points(const unsigned char* mask, int B, int S, int N, const float* depth, int H, int W,
                                const int* frame, const int* rc, const float* K4, float depth_scale,
                                const long long* seed, int stream_id, long long* choose, float* cloud, float* xmap,
                                float* ymap, int* count, void* stream) {
  if (!mask || !depth || !frame || !rc || !K4 || !seed || !choose || !cloud || !xmap || !ymap || !count)
    return KRRN_EARG;
  if (B < 1 || S < 1 || N < 1 || H < 1 || W < 1 || S > H || S > W || depth_scale == 0.f) return KRRN_ESHAPE;
  hipLaunchKernelGGL(choose_points_kernel, dim3(B), dim3(kChooseThreads), 0, (hipStream_t)stream, mask, S, N, depth,
                     H, W, frame, rc, K4, depth_scale, seed, stream_id, choose, cloud, xmap, ymap, count);
  return krrn_launch_status();
}
