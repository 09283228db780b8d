/*
 * krrn_hip.h — C ABI of libkrrn_hip.so, the MI355X (gfx950) kernels of the KRRN dense-fusion
 * inference path of yaomy533/pose_estimation (lib/network/krrn.py + tools/trainer.py:383-438).
 *
 * The reference has no FFI (pure Python/PyTorch); each entry point below names
 * the reference function(s) whose arithmetic it replaces. The Python host side
 * (pose_estimation_amd/) keeps the reference's model/loader/get_pose API and binds these
 * symbols with ctypes (INTEGRATION.md shows the binding).
 *
 * Contract shared by every entry point
 *   - Ownership: the caller allocates every input, output and workspace buffer (device
 *     memory); the library never allocates, keeps no global state and is reentrant.
 *   - Streams: all work is enqueued on `stream` (a hipStream_t); no host synchronisation, so
 *     every call can be captured into a hipGraph.
 *   - Errors: 0 = launched; KRRN_EARG (-1) null pointer / bad enum, KRRN_ESHAPE (-2) size out
 *     of range, KRRN_EALIGN (-3) 16-byte / channel-multiple-of-4 violation — all detected on
 *     the host before any launch; a positive value is the hipError_t of the launch.
 *   - Layouts: activations are NHWC f32 with a channel stride `*_cs` and channel offset
 *     `*_co` (so a buffer can be a slice of a concat); point sets are [B][n][stride] f32 with a
 *     batch stride `*_bs` (floats); indices produced by the library are int32.
 */
#ifndef KRRN_HIP_H
#define KRRN_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KRRN_OK 0
#define KRRN_EARG (-1)
#define KRRN_ESHAPE (-2)
#define KRRN_EALIGN (-3)
#define KRRN_EUNSUPPORTED (-4) /* hipBLASLt rejected the problem, or a form the kernel does not offer */

/* Implicit-GEMM convolution / GEMM on the f32 matrix cores, BN folded into scale/bias.
 * Replaces nn.Conv2d + BatchNorm2d (+ residual add) (+ ReLU) of BasicBlock / Bottleneck /
 * transitions / fuse layers / last_layer (lib/network/hrnet/myhrnet.py:34-103, 177-221,
 * 328-381), the XYZNet / NMLNet convs and 1x1 heads (lib/network/krrn.py:46-84),
 * ConvTranspose2d (myhrnet.py:314-326, krrn.py:47) as 4 parity-class launches, the GCN
 * `feature_map @ weights + bias` (lib/network/point/gcn3d.py:151, 203) and the TBase Conv1d
 * chain (lib/network/pose/posenet.py:58-77).
 *   out[m, n] = act(scale[n] * sum_k A[m,k] W[n,k] + bias[n] + bias2[m / b2_div, n] + res[m, n])
 *   m = (b, gy, gx) on a B x Hg x Wg grid; k = (tap, c), A = in[b, gy*in_s + tap_dy, gx*in_s + tap_dx, c]
 *   output pixel (gy*osy + ooy, gx*osx + oox) of a Ho x Wo map; wt is [N][ntaps*cin] row-major.
 *   N = computed channels (multiple of 4), n_store <= N stored; out_nchw = 1 writes
 *   out[b][out_co + n][oy][ox] with out_cs = total channels. tile (BMxBNxBK): 0 auto,
 *   1 = 128x128x16, 2 = 128x64x16, 3 = 64x64x16, 4 = 128x128x32, 5 = 256x32x16,
 *   6 = 128x32x32, 7 = 128x64x32, 8 = 64x64x32; out_nchw supports tiles 0-3 only.
 *   splits > 1 (NHWC only; N, n_store multiples of 4): split-K for small-M / deep-K layers
 *   (the 4x4 and 8x8 HRNet branches): each of `splits` slices of the k-tiles writes raw
 *   partial sums to workspace [splits][M][N] f32, then a second kernel sums them in slice
 *   order and applies the epilogue (deterministic). The slice count actually used is
 *   cdiv(nkt, cdiv(nkt, splits)) <= splits. splits = 1: workspace unused (may be NULL). */
int krrn_conv2d_f32(const float* in, int in_cs, int in_co, int B, int Hi, int Wi, int cin, int Hg, int Wg,
                    int in_s, int ntaps, const int* tap_dy, const int* tap_dx, const float* wt, int N,
                    int n_store, const float* scale, const float* bias, const float* bias2, int b2_div,
                    const float* res, int res_cs, int res_co, float* out, int out_cs, int out_co, int Ho,
                    int Wo, int osy, int osx, int ooy, int oox, int relu, int out_nchw, int tile, int splits,
                    float* workspace, void* stream);

/* One problem of a grouped convolution launch: the arguments of krrn_conv2d_f32 as a struct
 * (NHWC output only; tap_dy/tap_dx hold the first ntaps entries). */
typedef struct krrn_conv_desc {
  const float* in;
  int in_cs, in_co, B, Hi, Wi, cin, Hg, Wg, in_s, ntaps;
  int tap_dy[9];
  int tap_dx[9];
  const float* wt;
  int N, n_store;
  const float* scale;
  const float* bias;
  const float* bias2;
  int b2_div;
  const float* res;
  int res_cs, res_co;
  float* out;
  int out_cs, out_co, Ho, Wo, osy, osx, ooy, oox, relu, out_nchw, splits;
  float* workspace;
  /* k order of wt: 0 = tap-major (k = tap*cin + c); Q > 0 (Q % 4 == 0, Q | cin) = channel-chunk
   * major, k = ((c / Q)*ntaps + tap)*Q + c % Q: a block walks every tap of a Q-channel slice of
   * its input pixels back to back, so the taps' overlapping reads hit L1 / L2 instead of re-fetching
   * a whole tap's slab (the transposed convs' parity classes). Grouped launches only. */
  int k_chunk;
} krrn_conv_desc;

/* Up to 4 independent convolutions in ONE launch with a shared tile shape (tile 1 = 128x128x16,
 * 6 = 128x32x32 or 8 = 64x64x32), each with its own split-K factor: the j-th conv of every HRNet branch of a
 * HighResolutionModule (myhrnet.py:177-225: branch i is a chain of BasicBlocks on its own
 * resolution, so the branches are independent until the fuse layer). Each problem computes
 * exactly what krrn_conv2d_f32 would with the same descriptor. */
int krrn_conv2d_group_f32(const krrn_conv_desc* descs, int n, int tile, void* stream);

/* krrn_conv2d_f32 / krrn_conv2d_group_f32 on the bf16 matrix cores at f32 accuracy (NHWC output,
 * every tile of the menu / tiles 1, 6, 8): the activations are split while staged, the weights beforehand, into
 * three bf16 terms each (x = x_h + x_m + x_l, round-to-nearest, exact); every product is summed
 * over the six term pairs hh, hm, mh, hl, lh, mm (the dropped ones are below 2^-23 |a b|) and
 * accumulated in f32. wt3 (or each desc's wt) holds the split weights, bf16 [N][K / 4][16]: per 4 k
 * the terms m0..m3 h0..h3 l0..l3 then 4 zeros (ops.conv_weights_x3); 16-byte aligned. */
int krrn_conv2d_x3_f32(const float* in, int in_cs, int in_co, int B, int Hi, int Wi, int cin, int Hg, int Wg,
                       int in_s, int ntaps, const int* tap_dy, const int* tap_dx, const void* wt3, int N, int n_store,
                       const float* scale, const float* bias, const float* bias2, int b2_div, const float* res,
                       int res_cs, int res_co, float* out, int out_cs, int out_co, int Ho, int Wo, int osy, int osx,
                       int ooy, int oox, int relu, int tile, int splits, float* workspace, void* stream);
int krrn_conv2d_group_x3_f32(const krrn_conv_desc* descs, int n, int tile, void* stream);
/* Stride-2 ConvTranspose2d (kernel <= 4, padding 1; myhrnet.py:314-326's deconv, krrn.py:47-49's
 * XYZNet layer) as its four output parity classes in ONE block per 4 x 32 region of the input grid, on
 * split-bf16 operands at f32 accuracy (convt.hip): out[2a + py][2b + px][n] (NHWC, channels out_co ..
 * out_co + N - 1 of pixel rows of out_cs floats, Ho x Wo <= 2 Hi x 2 Wi) = act(scale[n] *
 * sum over the class's taps t and channels k of in[a + dy_t][b + dx_t][k] W[k][n] + bias[n]).
 * cls_taps (host memory, read at the call): for class c = 2 py + px, cls_taps[5c] = its tap count
 * (1..4) and cls_taps[5c + 1 + t] = (dy_t + 1) * 3 + (dx_t + 1). U3 = ops.convT_weights_x3: plane
 * U_mh [cin/8][16][N][2][8] bf16 (element class * 4 + tap; m0..m3 h0..h3 of channels 4 half ..
 * 4 half + 3) then plane U_l [cin/8][16][N][2][4]; 16-byte aligned. N = 128; cin a multiple of 8;
 * in 16-byte aligned with in_cs, in_co multiples of 4. relu != 0 applies ReLU. Replaces the grouped
 * krrn_conv2d_group_x3_f32 launch of the four classes (lib/network/krrn.py:47-49). */
int krrn_convT_s2_x3_f32(const float* in, int in_cs, int in_co, int B, int Hi, int Wi, int cin, const int* cls_taps,
                         const void* U3, int N, const float* scale, const float* bias, int relu, float* out,
                         int out_cs, int out_co, int Ho, int Wo, void* stream);

/* Plain f32 GEMM on hipBLASLt (library-shaped GEMMs of the fusion / TBase, see blas.hip):
 *   out[m*ldo + n] = act(sum_k A[m*lda + k] W[n*K + k] + bias[n] + res[m*ldr + n]),  0 <= n < N
 * in `batch` strided groups of M rows (A / out / res advance a_grp / o_grp / r_grp floats per
 * group, W [N][K] shared). create: heuristic query once, the plan is caller-owned (destroy frees
 * it); *ws_bytes = the workspace run() needs (<= max_ws). run: one hipblasLtMatmul on `stream`
 * (graph-capturable); bias / res must be given iff the plan was created with them.
 * KRRN_EUNSUPPORTED when hipBLASLt has no algorithm or fails. */
typedef struct krrn_blas_gemm krrn_blas_gemm;
int krrn_blas_gemm_create(int M, int N, int K, int lda, int ldo, int batch, long long a_grp, long long o_grp,
                          int has_bias, int relu, int has_res, int ldr, long long r_grp, long long max_ws,
                          krrn_blas_gemm** out_plan, long long* ws_bytes);
int krrn_blas_gemm_run(const krrn_blas_gemm* g, const float* a, const float* w, const float* bias, const float* res,
                       float* out, void* workspace, long long ws_bytes, void* stream);
int krrn_blas_gemm_destroy(krrn_blas_gemm* g);

/* The same GEMM on the bf16 matrix cores at f32 accuracy (gemm_x3.hip: split-bf16 operands,
 * six term products per f32 product): the GCN `feature_map @ weights` of G6/G7
 * (lib/network/point/gcn3d.py:125-127, 184-186) and TBase's Conv1d chain (posenet.py:51-96).
 *   out[m*ldo + n] = act(sum_k A[m*lda + k] W[n][k] + bias[n] + res[m*ldr + n])
 * in `batch` strided groups of M rows (a_grp / o_grp / r_grp floats per group); ldr = 0 adds one
 * res row per group (res[g*r_grp + n], a per-crop bias). w3f holds W split
 * into per-wave MFMA fragments (ops.gemm_weights_x3: [N/32][K/8][2][64 lanes][4] u32).
 * K % 32 == 0, N % 128 == 0, lda / ldo / ldr % 4 == 0, 16-byte aligned A / W / out / res. */
int krrn_gemm_x3_f32(const float* a, int lda, int M, int K, int N, const void* w3f, const float* bias,
                     const float* res, int ldr, float* out, int ldo, int relu, int batch, long long a_grp,
                     long long o_grp, long long r_grp, void* stream);

/* TBase conv2 on a gathered operand (gemm_x3.hip, GA form): conv1 runs by linearity on the fusion's
 * level rows (posenet.py:51-96 with the concat of lib/network/point/fusion.py:234-238 and the
 * one-hot channels of lib/network/krrn.py:132-138 folded into two per-crop row tables), and conv2
 * reads h1 = ReLU(A[b, ia[b, i]] + A2[b, ib[b, i]]) row by row while staging its operand, so h1 is
 * never materialised (it replaces krrn_gather2_add_f32 + krrn_gemm_x3_f32 on h1):
 *   out[(b*npts + i)*ldo + n] = act(sum_k h1[b, i, k] W[n][k] + bias[n])
 * A [B][a_bs floats], rows a_st apart; A2 likewise; ia / ib int32 [B][npts] row indices into the
 * crop's table. w3f as for krrn_gemm_x3_f32. K % 32 == 0, N % 128 == 0, strides % 4 == 0,
 * 16-byte aligned tables / W / out, B * a_bs and B * a2_bs < 2^29 floats. */
int krrn_gemm_x3_gather_f32(const int* ia, const float* A, long long a_bs, int a_st, const int* ib, const float* A2,
                            long long a2_bs, int a2_st, int npts, int B, int K, int N, const void* w3f,
                            const float* bias, float* out, int ldo, int relu, void* stream);

/* Short-K GEMM streaming its output (gemm_panel.hip): the fusion's level-0 / level-1 GCN
 * `feature_map @ weights + bias` of Conv_layer (lib/network/point/gcn3d.py:136-164, K = 128,
 * N = 8 * 128) and layer1's 64 -> 256 1x1 convs (myhrnet.py:65-103, K = 64):
 *   out[m*ldo + n] = act(sum_k A[m*lda + k] W[n][k] + bias[n] + res[m*ldr + n]),  0 <= n < N
 * Split-bf16 operands at f32 accuracy; each wave keeps its 32 activation rows in registers, the
 * 4 waves of a block walk 32-column tiles whose weights are copied once per block into LDS. wpf
 * holds W split into bf16 terms (ops.gemm_weights_panel: [N/32][K/8][384] u32, per 8-k group 64 lanes
 * x [m0..m3 h0..h3] then 64 lanes x [l0..l3]).
 * K = 64 or 128, N % 32 == 0, N <= 2048, lda % 4 == 0, A / wpf 16-byte
 * aligned; `csplit` column ranges per row panel (grid = ceil(M / 128) x csplit). K = 128 with a
 * residual: KRRN_EUNSUPPORTED. */
int krrn_gemm_panel_x3_f32(const float* a, int lda, int M, int K, int N, const void* wpf, const float* bias,
                           const float* res, int ldr, float* out, int ldo, int relu, int csplit, void* stream);

/* 1x1 conv with NCHW output (the heads' final xyz / normal convs, lib/network/krrn.py:97-98,
 * 80-84): out[b][out_co + n][p] = scale[n] * sum_c in[(b * HW + p) * in_cs + in_co + c] wt[n][c]
 * + bias[n] for n < n_store, p < HW; out has out_cs channels per image. cin <= 256 (multiple of 4),
 * N <= 80 weight rows (wt [N][cin]); in / wt 16-byte aligned. */
int krrn_conv1x1_nchw_f32(const float* in, int in_cs, int in_co, int B, int HW, int cin, const float* wt, int N,
                          int n_store, const float* scale, const float* bias, float* out, int out_cs, int out_co,
                          void* stream);

/* krrn_conv1x1_nchw_f32 on split-bf16 operands (f32 accuracy; the same output): cin = 128 and w3
 * the split weight planes of ops.quad_weights_x3(wt, N, 128) (16-byte aligned); 32 < N <= 80. */
int krrn_conv1x1_nchw_x3_f32(const float* in, int in_cs, int in_co, int B, int HW, int cin, const void* w3, int N,
                             int n_store, const float* scale, const float* bias, float* out, int out_cs, int out_co,
                             void* stream);

/* 3x3 stride-1 pad-1 convolution by fused Winograd F(2x2, 3x3) (the head / last_layer /
 * deconv-BasicBlock convs: krrn.py:46-84, myhrnet.py:324-346; cuDNN / MIOpen use the same
 * algorithm for these f32 convs). U = G g G^T are the transformed weights, f32 in chunk-major
 * order [ceil(cin/8)][16][N][8] (element xi = 4u + v of the 4x4 transform; input channels
 * padded to a multiple of 8 with zeros), computed once per plan; epilogue as
 * krrn_conv2d_f32: out = act(scale[n] * conv + bias[n] (+ res)). NHWC in/out with channel
 * stride / offset; cin multiple of 4, U 16-byte aligned. */
int krrn_conv3x3_wino_f32(const float* in, int in_cs, int in_co, int B, int H, int W, int cin, const float* U,
                          int N, int n_store, const float* scale, const float* bias, const float* res, int res_cs,
                          int res_co, float* out, int out_cs, int out_co, int relu, void* stream);
/* krrn_conv3x3_wino_f32 on the bf16 matrix cores at f32 accuracy: every operand split into
 * three bf16 terms (x = x_h + x_m + x_l, round-to-nearest, exact), each product summed over the
 * six term pairs hh, hm, mh, hl, lh, mm (the dropped ones are below 2^-23 |a b|), accumulated in
 * f32. U3 is wino_weights' U split on the host (wino_weights_x3): plane U_mh
 * [ceil(cin/8)][16][N][2][8] bf16 (m0..m3 h0..h3 of channels 4 half .. 4 half + 3) followed by
 * plane U_l [ceil(cin/8)][16][N][2][4] bf16; U3 16-byte aligned. Other arguments as
 * krrn_conv3x3_wino_f32. */
int krrn_conv3x3_wino_x3_f32(const float* in, int in_cs, int in_co, int B, int H, int W, int cin, const void* U3,
                             int N, int n_store, const float* scale, const float* bias, const float* res, int res_cs,
                             int res_co, float* out, int out_cs, int out_co, int relu, void* stream);
/* The same conv by Winograd F(4x4, 3x3) (points 0, +-1, +-2; 2.25 products per output instead of
 * 4) on split-bf16 operands, for the heads' wide 128 -> 128 convs (krrn.py:52-63, 74-81). U3 is
 * wino4_weights' U = G g G^T ([cin/8][36][N][8] f32, element xi = 6u + v) split on the host
 * (wino_weights_x3): plane U_mh [cin/8][36][N][2][8] bf16 then plane U_l [cin/8][36][N][2][4]
 * bf16. cin a multiple of 8; in 16-byte aligned with in_cs, in_co multiples of 4; other arguments
 * as krrn_conv3x3_wino_x3_f32 (any out / res channel alignment). */
int krrn_conv3x3_wino4_x3_f32(const float* in, int in_cs, int in_co, int B, int H, int W, int cin, const void* U3,
                              int N, int n_store, const float* scale, const float* bias, const float* res, int res_cs,
                              int res_co, float* out, int out_cs, int out_co, int relu, void* stream);
/* krrn_conv3x3_wino_x3_head_f32 on the F(4x4, 3x3) kernel (U3 as krrn_conv3x3_wino4_x3_f32; cin a
 * multiple of 8, in 16-byte aligned with in_cs, in_co multiples of 4). */
int krrn_conv3x3_wino4_x3_head_f32(const float* in, int in_cs, int in_co, int B, int H, int W, int cin,
                                   const void* U3, int N, const float* scale, const float* bias, const float* res,
                                   int res_cs, int res_co, int relu, const float* w1, const float* b1, int p1,
                                   float* part, float* out, int out_c, void* stream);
/* A head's last 3x3 conv fused with its final 1x1 conv (nml_final, krrn.py:80-84 / 98, when it has
 * at most 4 output channels): h = act(scale[n] * conv3x3 + bias[n] (+ res)) as
 * krrn_conv3x3_wino_x3_f32 with n_store = N, then out[b][o][y][x] = sum_n w1[o][n] h[n] + b1[o]
 * for o < p1 (NCHW, out_c channels per image). The N-channel map h is never written: each
 * 64-channel block of the Winograd grid writes its 4 partial dot products per pixel to part
 * (ceil(N / 64) * B * H * W * 4 floats, 16-byte aligned), and a second launch adds them in block
 * order plus b1 (deterministic). w1 [4][N] f32 (rows >= p1 zero), 16-byte aligned; N % 4 == 0,
 * 1 <= p1 <= 4; b1 may be NULL. */
int krrn_conv3x3_wino_x3_head_f32(const float* in, int in_cs, int in_co, int B, int H, int W, int cin,
                                  const void* U3, int N, const float* scale, const float* bias, const float* res,
                                  int res_cs, int res_co, int relu, const float* w1, const float* b1, int p1,
                                  float* part, float* out, int out_c, void* stream);

/* Direct conv for narrow layers: 3x3 / pad 1 / stride 1 or 2, or 1x1 / stride 1 (the HRNet
 * branches' BasicBlock convs, lib/network/hrnet/myhrnet.py:34-63, and the fuse layers' stride-2
 * downsamples / 1x1 projections, :177-225). NHWC in (in_cs / in_co, H x W input, cin physical
 * channels, multiple of 4), weights wt [N][ksize^2 * cin] (k = tap * cin + c, tap = ky * ksize + kx),
 * out (Ho x Wo = the conv's output size) = act(scale[n] * conv + bias[n] (+ res)) for n < n_store.
 * A block stages the input rows of its 64 / ks output pixels (all channels) in LDS once;
 * 16x16x4 f32 MFMAs; nw = 16-channel output tiles per wave (1..3), ks = waves splitting the
 * reduction of one tile (1, 2, 4; partials summed in LDS in order). */
int krrn_conv_small_f32(const float* in, int in_cs, int in_co, int B, int H, int W, int cin, const float* wt, int N,
                        int n_store, const float* scale, const float* bias, const float* res, int res_cs, int res_co,
                        float* out, int out_cs, int out_co, int relu, int ksize, int stride, int nw, int ks,
                        void* stream);


/* k nearest neighbours without the [n, n] distance matrix.
 * Replaces gcn3d.get_neighbor_index (gcn3d.py:15-26; mode 0, drop_first = 1: topk(k+1)[1:])
 * and gcn3d.get_nearest_index (gcn3d.py:29-38; mode 1, k = 1, drop_first = 0).
 * Queries: q + b*q_bs + qi*q_st (qi = qidx[t] if qidx else t, t < nq; qidx shared by the
 * batch: the Pool_layer randperm rows, gcn3d.py:239); candidates c + b*c_bs + j*c_st, j < nc;
 * d = 3 or 9. Exact f32 expression order (no FMA):
 *   mode 0: ((-2 <q,c>) + |c|^2) + |q|^2      mode 1: (|c|^2 + |q|^2) - 2 <q,c>
 * with <.,.> and |.|^2 summed sequentially over d; ties -> lower index.
 * out: int32 [B][nq][k]. k + drop_first <= 16. */
int krrn_knn_f32(const float* q, long long q_bs, int q_st, int nq, const int* qidx, const float* c,
                 long long c_bs, int c_st, int nc, int d, int k, int drop_first, int mode, int B, int* out,
                 void* stream);

/* 3D-GCN neighbourhood reduction, fused with the BN1d + ReLU FusionNetLite applies.
 * Y == NULL: Conv_surface (gcn3d.py:88-112):  out[i,c] = sum_s max_j relu(dir_ij . dn[:, sC+c])
 * Y != NULL: Conv_layer / Conv_fuse_layer (gcn3d.py:136-216):
 *   out[i,c] = Y[i,c] + sum_s max_j relu(dir_ij . dn[:, sC+c]) * Y[idx[i,j], C + sC + c]
 * then out = out*bn_scale + bn_bias (if given), relu (if set) (fusion.py:183-213).
 * dir_ij = F.normalize(v[idx[i,j]] - v[i]) over d = 3 or 9 coords (v stride v_st);
 * dn = F.normalize(directions, dim=0) [d][S*C]; Y [B][n][(S+1)*C]; idx int32 [B][n][k], k <= 16;
 * out + b*o_bs + i*o_st + c. */
int krrn_gcn_conv_f32(const int* idx, int n, int k, const float* v, long long v_bs, int v_st, int d,
                      const float* dn, int S, int C, const float* Y, const float* bn_scale, const float* bn_bias,
                      int relu, float* out, long long o_bs, int o_st, int B, void* stream);

/* Pool_layer max (gcn3d.py:233-236) at the sampled rows only: out[b,t,:] = max_j F[b, nbr[b,t,j], :].
 * C, strides multiple of 4 (float4). */
int krrn_pool_max_f32(const int* nbr, int nq, int kk, const float* F, long long f_bs, int f_st, int C, float* out,
                      long long o_bs, int o_st, int B, void* stream);

/* Bilinear resize NHWC (F.interpolate(mode='bilinear'), myhrnet.py:242-245 / 511-516 with
 * align_corners = 0; nn.UpsamplingBilinear2d, krrn.py:56/78, with align_corners = 1), optionally
 * out = add + resize(in) and ReLU: the HRNet fuse-layer "y = y + interpolate(...)" step. */
int krrn_resize_bilinear_f32(const float* in, int B, int Hi, int Wi, int in_cs, int in_co, int C, float* out,
                             int Ho, int Wo, int out_cs, int out_co, const float* add, int add_cs, int add_co,
                             int align_corners, int relu, void* stream);

/* out = relu?(a + b) on NHWC channel slices (HRNet fuse identity term, myhrnet.py:237-238;
 * b == NULL copies a, the concat of myhrnet.py:516). */
int krrn_add_relu_f32(const float* a, int a_cs, int a_co, const float* b, int b_cs, int b_co, float* out,
                      int o_cs, int o_co, long long npix, int C, int relu, void* stream);

/* NCHW [B][C][H][W] -> NHWC channel slice (the API boundary of KRRN.forward's x). */
int krrn_nchw_to_nhwc_f32(const float* in, int B, int C, int H, int W, float* out, int o_cs, int o_co,
                          void* stream);

/* Per-crop class selection of the xyz / normal maps + F.normalize(p=2, dim=1, eps=1e-12)
 * (krrn.py:105-108). fx: xyz_final output NCHW [B][Cx][H][W] (xyz block at channel xyz_off),
 * fn: nml_final output [B][Cn][H][W]; cls int64 [B]. */
int krrn_heads_select_f32(const float* fx, int Cx, int xyz_off, const float* fn, int Cn, const long long* cls,
                          float* xyz_out, float* nml_out, int B, int H, int W, void* stream);

/* The `choose` gather (krrn.py:121-122) packed as P9 [B][N][9] = [cloud | xyz_emb | nml_emb]
 * (the feat_feature layout of fusion.py:194). choose int64 [B][N]. */
int krrn_points_gather_f32(const float* cloud, const float* xyz, const float* nml, const long long* choose, int B,
                           int N, int H, int W, float* p9, void* stream);

/* Row gather dst[b, r, 0:width] = src[b, idx[b*idx_bs + r], 0:width] (int32 or int64 idx;
 * idx_bs = 0 shares one index list across the batch): Pool_layer sampling (gcn3d.py:240-241),
 * indexing_neighbor by the nearest indices into the 1280-wide concat (fusion.py:234-238),
 * the one-hot column of TBase conv1 (krrn.py:132-138). */
int krrn_gather_rows_f32(const void* idx, int idx64, long long idx_bs, int nrows, const float* src, long long src_bs,
                         int src_st, float* dst, long long dst_bs, int dst_st, int width, int B, void* stream);

/* TBase conv1 over the fusion concat by linearity (krrn.py:132-141 with fusion.py:234-238):
 * out[b][i] = act(scale * (A[b][ia[b][i]] + B[b][ib[b][i]]) + bias + bias2[b]) over C channels,
 * with A = fm_5 W1[:, 0:512]^T (level-2 rows, ia = nearest_pool_2) and B = feat_1 W1[:, 512:896]^T +
 * feat_2 W1[:, 896:1280]^T (level-1 rows, ib = nearest_pool_1); ia / ib int32 [B][n]; bias2
 * [B][C] optional (the one-hot class column, pre-scaled). C, strides multiple of 4, 16-B aligned. */
int krrn_gather2_add_f32(const int* ia, const float* A, long long a_bs, int a_st, const int* ib, const float* B_,
                         long long b_bs, int b_st, int n, int C, const float* scale, const float* bias,
                         const float* bias2, int relu, float* out, long long o_bs, int o_st, int B, void* stream);

/* TBase conv4 (first 3 outputs, posenet.py:76-80) + pred_t = mean_N(cloud + t_res) (krrn.py:153).
 * h [B][n][C]; w4 [3][C]; b4 [3]; cloud [B][n][3]; pred_t [B][3]; t_res optional [B][n][3].
 * C multiple of 4, h and w4 16-byte aligned (KRRN_EALIGN otherwise). */
int krrn_tbase_tail_f32(const float* h, int B, int n, int C, const float* w4, const float* b4, const float* cloud,
                        float* pred_t, float* t_res, void* stream);

/* Batched PnP-RANSAC: Trainer.get_pose (tools/trainer.py:383-438), cv2.solvePnPRansac(EPNP,
 * reprojectionError = thr, confidence = conf (0.9999 there), iterationsCount = H) restated.
 * xyz [B][3][HW] (normalised model coords), choose int64 [B][N], sel int32 [B][P] (the
 * randperm(N)[:P] subset), x/ymap [B][N] full-frame pixels, K4 [B][4] = fx fy cx cy,
 * extent / lfborder f64 [B][3], subsets int32 [B][H][5] (hypothesis h's sample); workspace:
 * B*H*13 floats (per-hypothesis pose + inlier count). Hypotheses are scored in parallel; the
 * selection is ptsetreg.cpp's loop over them in order with its adaptive iteration count
 * (niters <- RANSACUpdateNumIters(conf, outlier ratio, 5, niters) on every new best). Outputs R
 * [B][9] row-major, t [B][3], inlier count [B] (0 = RANSAC failed -> R = I, t = 0), inlier_mask
 * [B][P] (optional). Two launches: one 16-lane group per hypothesis, then one wave per crop for
 * the selection + EPnP on all inliers. */
int krrn_pnp_ransac_f32(const float* xyz, int HW, const long long* choose, int N, const int* sel, int P,
                        const float* xmap, const float* ymap, const float* K4, const double* extent,
                        const double* lfborder, const int* subsets, int H, float thr, double conf, float* workspace,
                        float* R, float* t, int* inliers, unsigned char* inlier_mask, int B, void* stream);

/* torch.randperm(n)[:k] per row (gcn3d.py:239, trainer.py:407) from a counter-based generator
 * seeded by *seed_ptr (device memory) and `stream_id`; n <= 4096. out int32 [rows][k]. */
int krrn_randperm_i32(const unsigned long long* seed_ptr, unsigned int stream_id, int n, int k, int rows, int* out,
                      void* stream);

/* Up to 8 independent single-row draws of krrn_randperm_i32 in ONE launch (the five Pool_layer
 * permutations of a forward, gcn3d.py:239): draw q is torch.randperm(n[q])[:k[q]] for stream id
 * stream_id[q] into out[q], bit-identical to krrn_randperm_i32(seed_ptr, stream_id[q], n[q], k[q],
 * 1, out[q]); the draws run side by side (one block each) instead of back to back. */
int krrn_randperm_multi_i32(const unsigned long long* seed_ptr, int count, const unsigned int* stream_id, const int* n,
                            const int* k, int* const* out, void* stream);

/* RANSAC subsets: 5 distinct indices in [0, P) per (crop, hypothesis); out int32 [B][H][5]. */
int krrn_ransac_subsets(const unsigned long long* seed_ptr, unsigned int stream_id, int B, int H, int P, int* out,
                        void* stream);

/* *seed_ptr += 1 (last node of a replayed step). */
int krrn_rng_advance(unsigned long long* seed_ptr, void* stream);

/* Eval-time KRRNLoss map terms (lib/network/loss.py:57-65 over loss_utils.py:8-70), SURVEY §8f f1.
 * NCHW maps of B crops with HW pixels: xyz / xyz_gt [B][3][HW] (l1), nml / nml_gt [B][3][HW]
 * (1 - cosine, CosineSimilarity eps 1e-6), region [B][R][HW] + region_gt int64 [B][HW] and mask
 * [B][M][HW] + mask_gt int64 [B][HW] (-log(softmax + 1e-6) at the label). Pixels whose target is
 * all zero (label 0) are excluded; each term = sum / valid count. Any term may be skipped by
 * passing NULL maps. out f64 [8]: losses xyz, normal, region, mask, then the four valid counts.
 * ws: f64 workspace of krrn_map_losses_ws(B, HW) doubles. Deterministic (fixed-order sums). */
int krrn_map_losses_ws(int B, int HW, long long* n_doubles);
int krrn_map_losses_f32(const float* xyz, const float* xyz_gt, const float* nml, const float* nml_gt,
                        const float* region, int R, const long long* region_gt, const float* mask, int M,
                        const long long* mask_gt, int B, int HW, double* ws, double* out, void* stream);
/* Per-crop form, read from the ws a preceding krrn_map_losses_f32(B, HW) filled (same stream):
 * out_crop f64 [B][8] = crop b's four losses then its four valid counts. The reference's test
 * loop runs batch size 1 and adds each crop's own losses to its object (tools/trainer.py:180-182). */
int krrn_map_losses_crop_f32(const double* ws, int B, int HW, double* out_crop, void* stream);

/* PoseLoss (lib/network/loss.py:19-42) with the GT rotation and the predicted translation as
 * KRRNLoss calls it (:66-67): pred = model_points [B][P][3] @ target_r[b]^T + pred_t[b]; for
 * crops whose cls_id is in sym[0..nsym) each predicted point takes its nearest target point
 * (squared distance, ties -> lower index; the KeOps argkmin of train.py:126); out f64 [1] =
 * mean over crops of mean_P |pred - target|. ws: krrn_pose_loss_ws(B, P) doubles. */
int krrn_pose_loss_ws(int B, int P, long long* n_doubles);
int krrn_pose_loss_f32(const float* target_r, const float* pred_t, const float* target, const float* model_points,
                       const long long* cls_id, const int* sym, int nsym, int B, int P, double* ws, double* out,
                       void* stream);

/* ADD(-S) per crop (Metric.cal_adds_cuda, lib/utils/metric.py:17-35, called by Trainer.cal_dis,
 * tools/trainer.py:370-381): pred = model_points [B][P][3] @ pred_r[b]^T + pred_t[b]; out f64 [B]
 * = mean_i |pred_i - target_i| (ADD), or for cls_id[b] in sym[0..nsym) mean over targets i of
 * min over preds j |pred_j - target_i| (ADD-S, exact direct-difference norms). ws: the same
 * size as krrn_pose_loss_ws(B, P). Deterministic. */
int krrn_add_metric_f32(const float* pred_r, const float* pred_t, const float* model_points, const float* target,
                        const long long* cls_id, const int* sym, int nsym, int B, int P, double* ws, double* out,
                        void* stream);

/* On-GPU input construction, replacing PoseDataset._load_data's per-sample numpy
 * work (dataset/linemod/batchdataset.py:603-771) for B crops of one snapped square size S.
 * Frames: rgb u8 [F][H][W][3], depth f32 [F][H][W], mask_label u8 [F][H][W], optional obj_mask u8
 * [F][H][W] (the reference's mask_obj from the GT coordinate map, :662; NULL = all ones); crop b
 * reads frame frame[b] at rows rc[2b] .. +S, cols rc[2b+1] .. +S.
 * krrn_crop_inputs_u8: img f32 [B][3][S][S] = (float(u8 / 255.) - mean) / std (ImageNet, :70, 722,
 * 744); mask u8 [B][S*S] = mask_label != 0 && depth != 0 (&& obj_mask != 0) (:662-666). */
int krrn_crop_inputs_u8(const unsigned char* rgb, const float* depth, const unsigned char* mask_label,
                        const unsigned char* obj_mask, int F, int H, int W, const int* frame, const int* rc, int B,
                        int S, float* img, unsigned char* mask, void* stream);

/* choose (:667-679): the crop's mask pixels in row-major order; more than N -> a uniformly random
 * order-preserving N-subset (the N smallest of counter-hash keys of (seed, stream_id, crop, rank),
 * radix-selected; the reference draws it with np.random.shuffle), fewer -> wrap-padded to N.
 * Then x_map / y_map = full-frame column / row (:712-715) and cloud [B][N][3] = ((x - cx) * z / fx,
 * (y - cy) * z / fy, z) with z = depth / depth_scale, f32 arithmetic in the reference's order
 * (:718-721); K4 [B][4] = fx, fy, cx, cy. count [B] = mask pixels (0 -> zeros everywhere: the
 * reference drops such a sample). choose int64 [B][N] (crop-local r*S + c). */
int krrn_choose_points(const unsigned char* mask, int B, int S, int N, const float* depth, int H, int W,
                       const int* frame, const int* rc, const float* K4, float depth_scale, const long long* seed,
                       int stream_id, long long* choose, float* cloud, float* xmap, float* ymap, int* count,
                       void* stream);

/* Farthest point sampling (tools/script/sample_model.py:35-48): per set b of
 * pts [B][n][3], out_idx int32 [B][n_samples] = start at 0, then repeatedly the argmax (lowest
 * index on ties) of the running min distance to the selected set; distances as numpy computes
 * them (f32, sqrt(((dx*dx + dy*dy) + dz*dz)), no FMA). n <= 16384. */
int krrn_fps_f32(const float* pts, int B, int n, int n_samples, int* out_idx, void* stream);

/* BPnP forward (lib/network/dnn/BPnP.py:43-44, cv2.solvePnP(SOLVEPNP_ITERATIVE,
 * useExtrinsicGuess=True)): Levenberg-Marquardt on sum_i ||pi(z_i; y) - x_i||^2 per crop, f64,
 * from y_init. pts2d [B][n][2] pixels; pts3d [n][3] shared (z_per_crop = 0) or [B][n][3];
 * K [3][3] row-major; y_init / y_out [B][6] = angle-axis (kornia convention) then t; R_init
 * [B][9] (optional): a rotation matrix replacing y_init's angle-axis (log map), e.g. the
 * krrn_pnp_ransac_f32 result as cv2.solvePnPRansac's rvec0 (BPnP.py:36-38); cost_out [B] final
 * squared error (optional). At most `iters` accepted steps (stops earlier once a step is below
 * 1e-13 relative). n >= 3. */
int krrn_bpnp_solve_f32(const float* pts2d, const float* pts3d, int z_per_crop, const float* K, const float* y_init,
                        const float* R_init, int B, int n, int iters, float* y_out, float* cost_out, void* stream);

/* BPnP backward (lib/network/dnn/BPnP.py:53-117): implicit-function gradients of the pose P6
 * [B][6] given grad_out [B][6]. grad_x [B][n][2]; grad_z [n][3] summed over crops (shared
 * points) or [B][n][3] (z_per_crop); grad_K [3][3] summed over crops. workspace:
 * B*(3n + 9) f64. Deterministic (crop-ordered sums). A singular J_fy gives NaN gradients for
 * that crop (the reference's torch.inverse raises). */
int krrn_bpnp_backward_f32(const float* pts2d, const float* P6, const float* pts3d, int z_per_crop, const float* K,
                           const float* grad_out, int B, int n, float* grad_x, float* grad_z, float* grad_K,
                           double* workspace, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* KRRN_HIP_H */
