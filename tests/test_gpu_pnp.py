"""Batched PnP-RANSAC kernel vs the C oracle (identical subsets) and known-answer recovery."""
import numpy as np
import pytest
import torch

from oracle import pnp as opnp
from pose_estimation_amd import pose

pytestmark = pytest.mark.gpu

K4 = np.array([572.4114, 573.57043, 325.2611, 242.04899], np.float32)


def _scene(B, N, S, seed, outlier_frac=0.1, noise_px=0.0):
    """xyz maps whose chosen pixels hold exact normalised model coordinates of a known pose."""
    rng = np.random.default_rng(seed)
    ext = np.array([0.067, 0.1276, 0.1175])
    lfb = np.array([-0.0335, -0.0638, -0.0587])
    xyz = np.zeros((B, 3, S, S), np.float32)
    choose = np.zeros((B, 1, N), np.int64)
    xm = np.zeros((B, N, 1), np.float32)
    ym = np.zeros((B, N, 1), np.float32)
    Rs, ts = [], []
    for b in range(B):
        R = opnp.rotation_from_axis_angle(rng.normal(size=3))
        t = np.array([rng.uniform(-0.1, 0.1), rng.uniform(-0.1, 0.1), rng.uniform(0.7, 1.1)])
        pix = rng.choice(S * S, N, replace=False)
        u = rng.random((N, 3))
        pw = (u * ext + lfb)
        # store the f32 normalised coordinate the network would predict
        u32 = u.astype(np.float32)
        pw = u32.astype(np.float64) * ext + lfb
        pc = pw @ R.T + t
        img = np.stack([K4[0] * pc[:, 0] / pc[:, 2] + K4[2], K4[1] * pc[:, 1] / pc[:, 2] + K4[3]], 1)
        img += rng.normal(scale=noise_px, size=img.shape) if noise_px else 0
        out = rng.random(N) < outlier_frac
        img[out] += rng.uniform(-20, 20, size=(out.sum(), 2))
        flat = xyz[b].reshape(3, -1)
        flat[:, pix] = u32.T
        choose[b, 0] = pix
        xm[b, :, 0] = img[:, 0]
        ym[b, :, 0] = img[:, 1]
        Rs.append(R)
        ts.append(t)
    data = {"choose": torch.from_numpy(choose), "x_map_choosed": torch.from_numpy(xm),
            "y_map_choosed": torch.from_numpy(ym), "intrinsic": torch.from_numpy(np.tile(K4, (B, 1))),
            "extent": torch.from_numpy(np.tile(ext, (B, 1))), "lfborder": torch.from_numpy(np.tile(lfb, (B, 1)))}
    return torch.from_numpy(xyz), data, np.stack(Rs), np.stack(ts)


def _update_niters(conf, ep, model_points, max_iters):
    """cv::RANSACUpdateNumIters (ptsetreg.cpp)."""
    conf, ep = min(max(conf, 0.0), 1.0), min(max(ep, 0.0), 1.0)
    num = max(1.0 - conf, np.finfo(np.float64).tiny)
    denom = 1.0 - (1.0 - ep) ** model_points
    if denom < np.finfo(np.float64).tiny:
        return 0
    num, denom = np.log(num), np.log(denom)
    return max_iters if (denom >= 0 or -num >= max_iters * (-denom)) else int(np.rint(num / denom))


def _cv2_select(cnts, P, conf=np.float32(0.9999)):
    """ptsetreg.cpp's RANSAC loop over already-scored hypotheses: the selected index."""
    best, best_cnt, niters, h = -1, 0, len(cnts), 0
    while h < niters:
        c = int(cnts[h])
        if c > max(best_cnt, 4):
            best, best_cnt = h, c
            niters = _update_niters(float(conf), (P - c) / P, 5, niters)
        h += 1
    return best


def test_known_pose_recovery(dev):
    B, N, S = 8, 1000, 120
    xyz, data, Rgt, tgt = _scene(B, N, S, 0)
    R, t, info = pose.get_pose({"xyz": xyz.to(dev)}, data, return_info=True)
    torch.cuda.synchronize()
    R, t = R.cpu().numpy(), t.cpu().numpy()
    assert np.abs(R - Rgt).max() < 1e-3, np.abs(R - Rgt).max()
    assert np.abs(t - tgt).max() < 1e-3
    assert (info["inliers"].cpu().numpy() >= 200).all()


@pytest.mark.parametrize("noise_px,cnt_tol,pose_tol", [(0.0, 0, 1e-4), (0.4, 0, 1e-4)])
def test_matches_oracle_same_subsets(dev, noise_px, cnt_tol, pose_tol):
    """RANSAC vs the C oracle on identical subsets: the oracle run on the GPU's selected subset
    reproduces its inlier count exactly and its refined pose within 1e-4 (north_star's R bound),
    noiseless and with 0.4 px noise; and the GPU's RANSAC over all subsets is as good as the
    oracle's over the batch. (The full hypothesis-by-hypothesis comparison is
    test_full_ransac_matches_oracle.)"""
    B, N, S = 16, 1000, 100
    xyz, data, _, _ = _scene(B, N, S, 1, outlier_frac=0.3, noise_px=noise_px)
    R, t, info = pose.get_pose({"xyz": xyz.to(dev)}, data, return_info=True)
    torch.cuda.synchronize()
    sel = info["sel"].cpu().long()
    subs = info["subsets"].cpu()
    H = subs.shape[1]
    hcnt = info["workspace"].cpu()[B * H * 12:].view(torch.int32)[:B * H].view(B, H).numpy()
    tot_gpu = tot_cpu = 0
    for b in range(B):
        s = sel[b]
        pix = data["choose"][b, 0, s]
        obj = (xyz[b].reshape(3, -1)[:, pix].double().t() * data["extent"][b] + data["lfborder"][b]).float().numpy()
        img = np.stack([data["x_map_choosed"][b, s, 0].numpy(), data["y_map_choosed"][b, s, 0].numpy()], 1)
        best_h = _cv2_select(hcnt[b], len(s))  # cv2's loop with its adaptive iteration count
        Ro, to, cnt, mask, _ = opnp.pnp_ransac(obj, img, K4, subs[b, best_h:best_h + 1].numpy(), 1.0)
        gcnt = int(info["inliers"][b])
        assert gcnt == int(hcnt[b][best_h]), (b, gcnt, hcnt[b][best_h])
        assert abs(gcnt - cnt) <= cnt_tol, (b, gcnt, cnt)
        assert np.abs(R[b].cpu().numpy() - Ro).max() < pose_tol
        assert np.abs(t[b].cpu().numpy() - to).max() < pose_tol
        _, _, cnt_all, _, _ = opnp.pnp_ransac(obj, img, K4, subs[b].numpy(), 1.0)
        tot_gpu += gcnt
        tot_cpu += cnt_all
    assert tot_gpu >= 0.99 * tot_cpu, (tot_gpu, tot_cpu)


def test_ransac_failure_identity(dev):
    # pure noise correspondences: no hypothesis reaches 5 inliers -> R = I, t = 0 (cv2 failure)
    B, N, S = 2, 300, 40
    xyz, data, _, _ = _scene(B, N, S, 2, outlier_frac=1.0)
    data["x_map_choosed"] = torch.rand(B, N, 1) * 640
    data["y_map_choosed"] = torch.rand(B, N, 1) * 480
    R, t, info = pose.get_pose({"xyz": xyz.to(dev)}, data, return_info=True)
    torch.cuda.synchronize()
    for b in range(B):
        if int(info["inliers"][b]) == 0:
            assert torch.allclose(R[b].cpu(), torch.eye(3))
            assert torch.all(t[b].cpu() == 0)


def test_device_rng(dev):
    from pose_estimation_amd import _lib
    from pose_estimation_amd.runtime import ptr, P
    seed = torch.tensor([123], dtype=torch.int64, device=dev)
    out = torch.empty((4, 250), dtype=torch.int32, device=dev)
    st = P(torch.cuda.current_stream().cuda_stream)
    _lib.check(_lib.lib().krrn_randperm_i32(ptr(seed), 0, 1000, 250, 4, ptr(out), st), "randperm")
    subs = torch.empty((3, 100, 5), dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().krrn_ransac_subsets(ptr(seed), 1, 3, 100, 256, ptr(subs), st), "subsets")
    torch.cuda.synchronize()
    o = out.cpu()
    for r in range(4):
        assert len(set(o[r].tolist())) == 250 and o[r].min() >= 0 and o[r].max() < 1000
    assert not torch.equal(o[0], o[1])
    s = subs.cpu().reshape(-1, 5)
    assert all(len(set(row.tolist())) == 5 for row in s)
    assert s.min() >= 0 and s.max() < 256



def test_device_rng_multi_matches_single(dev):
    """krrn_randperm_multi_i32 (the five pool permutations in one launch) equals the five
    krrn_randperm_i32 single-row launches draw for draw."""
    import ctypes
    from pose_estimation_amd import _lib
    from pose_estimation_amd.runtime import ptr, P
    seed = torch.tensor([987654321], dtype=torch.int64, device=dev)
    st = P(torch.cuda.current_stream().cuda_stream)
    draws = [(0, 1000, 250), (1, 1000, 250), (2, 1000, 250), (3, 1000, 250), (4, 250, 62), (7, 4096, 1)]
    singles = []
    for sid, n, k in draws:
        o = torch.empty(k, dtype=torch.int32, device=dev)
        _lib.check(_lib.lib().krrn_randperm_i32(ptr(seed), sid, n, k, 1, ptr(o), st), "randperm")
        singles.append(o)
    multi = [torch.full((k,), -1, dtype=torch.int32, device=dev) for _, _, k in draws]
    c = len(draws)
    sids = (ctypes.c_uint * c)(*[d[0] for d in draws])
    ns = (ctypes.c_int * c)(*[d[1] for d in draws])
    ks = (ctypes.c_int * c)(*[d[2] for d in draws])
    outs = (ctypes.c_void_p * c)(*[m.data_ptr() for m in multi])
    _lib.check(_lib.lib().krrn_randperm_multi_i32(ptr(seed), c, sids, ns, ks, outs, st), "randperm multi")
    torch.cuda.synchronize()
    for a, b in zip(singles, multi):
        assert torch.equal(a, b)
    bad = (ctypes.c_int * c)(*([5000] * c))
    assert _lib.lib().krrn_randperm_multi_i32(ptr(seed), c, sids, bad, ks, outs, st) < 0
    assert _lib.lib().krrn_randperm_multi_i32(ptr(seed), 9, sids, ns, ks, outs, st) < 0


@pytest.mark.parametrize("noise_px,outliers", [(0.0, 0.3), (0.4, 0.3), (1.0, 0.5)])
def test_full_ransac_matches_oracle(dev, noise_px, outliers):
    """Every one of the H = 100 hypotheses, the RANSAC selection and the refined pose vs the C oracle
    on identical subsets. oracle/pnp_ref.c restates the kernel's f64 expression order: the 5-point
    EPnP of a hypothesis sums its points in order (HypSum), the all-inlier refinement in the wave's
    order (WaveSum: 64 lane partials + butterfly; M^T M rows by lane group), the normal equations
    solved by Cholesky, the 12 x 12 eigen-solve by the same parallel Jacobi schedule -- so the
    hypothesis inlier counts are equal count for count, the selected hypothesis is the same, and
    R / t agree to 1e-6 (north_star: 1e-4 on R). cv2.solvePnPRansac itself is not installable
    here: parity to OpenCV is unpinned (oracle/pnp_ref.c header)."""
    B, N, S = 16, 1000, 100
    xyz, data, _, _ = _scene(B, N, S, 7, outlier_frac=outliers, noise_px=noise_px)
    R, t, info = pose.get_pose({"xyz": xyz.to(dev)}, data, return_info=True)
    torch.cuda.synchronize()
    sel = info["sel"].cpu().long()
    subs = info["subsets"].cpu()
    H = subs.shape[1]
    hcnt = info["workspace"].cpu()[B * H * 12:].view(torch.int32)[:B * H].view(B, H).numpy()
    worst = 0.0
    for b in range(B):
        s = sel[b]
        pix = data["choose"][b, 0, s]
        obj = (xyz[b].reshape(3, -1)[:, pix].double().t() * data["extent"][b] + data["lfborder"][b]).float().numpy()
        img = np.stack([data["x_map_choosed"][b, s, 0].numpy(), data["y_map_choosed"][b, s, 0].numpy()], 1)
        _, _, ocnt = opnp.pnp_hypotheses(obj, img, K4, subs[b].numpy(), 1.0)
        assert np.array_equal(ocnt, hcnt[b]), (b, np.nonzero(ocnt != hcnt[b])[0][:8])
        Ro, to, cnt, mask, best = opnp.pnp_ransac(obj, img, K4, subs[b].numpy(), 1.0)
        assert int(info["inliers"][b]) == cnt, (b, int(info["inliers"][b]), cnt)
        assert np.array_equal(info["mask"][b].cpu().numpy().astype(bool), mask), b
        worst = max(worst, float(np.abs(R[b].cpu().numpy() - Ro).max()), float(np.abs(t[b].cpu().numpy() - to).max()))
    print(f"noise {noise_px} px, {outliers:.0%} outliers: max |dR|, |dt| vs oracle {worst:.2e}")
    assert worst < 1e-6, worst


@pytest.mark.parametrize("noise_px", [0.0, 0.4])
def test_ransac_matches_opencv_semantics_oracle(dev, noise_px):
    """Against oracle_pnp_ransac_cv, the restatement that follows OpenCV's epnp.cpp numerics instead
    of the kernel's (cyclic 12 x 12 Jacobi, SVD beta solves, QR Gauss-Newton, R = U V^T of the SVD
    with the third row negated when det < 0, sequential sums, xc / zc in the inlier test), on the
    same subsets, both ways.

    Why the counts can differ at all (tests/pnp_divergence.py): a 5-point M is
    10 x 12, so M^T M has a 2-D exact null space (its two smallest eigenvalues are rounding, ~1e-17
    of the largest) and the basis an eigen-solver returns for it is decided by its rounding. EPnP's
    beta approximations 1 and 3 depend on that basis, so Gauss-Newton lands in different minima for
    ~40 % of noisy hypotheses. Swapping single ingredients of the OpenCV-semantics path for the
    kernel's shows it is the only cause: with the kernel's null-space basis every hypothesis count
    agrees (2 of 160 000 differ by rounding at the threshold); the solves (SVD vs Cholesky, QR vs
    Cholesky) change nothing. cv2's own basis comes from its JacobiSVD's rounding (unpinned here).

    1. Exact, two-sided: with the kernel's null-space basis in the OpenCV-semantics oracle, the GPU's
       per-hypothesis counts equal it (<= 0.2 % of hypotheses off by <= 2 at the threshold), the
       selected count is equal in every crop and R / t agree to 1e-4.
    2. Statistical, two-sided, pure OpenCV numerics: noiseless, every count within 8 and R / t within
       1e-4; with 0.4 px noise the selected count differs in <= 25 % of crops (CPU study: 10 %), by at
       most 24 either way (CPU study over 3200 crops: +-22), with |mean gap| <= 2 (no bias: -0.01);
       R / t within 1e-2 where the selected counts agree."""
    import ctypes

    B, N, S, H = 64, 1000, 100, 100
    xyz, data, _, _ = _scene(B, N, S, 9, outlier_frac=0.3, noise_px=noise_px)
    # the 256-point selection and the hypothesis subsets from a local generator: the test does not
    # depend on how far earlier tests moved the global CPU / device RNG streams
    g = torch.Generator().manual_seed(2024)
    sel0 = torch.stack([torch.randperm(N, generator=g)[:256] for _ in range(B)]).to(torch.int32)
    subs0 = torch.stack([torch.stack([torch.randperm(256, generator=g)[:5] for _ in range(H)])
                         for _ in range(B)]).to(torch.int32)
    R, t, info = pose.get_pose({"xyz": xyz.to(dev)}, data, sel=sel0, subsets=subs0, return_info=True)
    torch.cuda.synchronize()
    sel = info["sel"].cpu().long()
    subs = info["subsets"].cpu()
    hcnt = info["workspace"].cpu()[B * H * 12:].view(torch.int32)[:B * H].view(B, H).numpy()
    lib = opnp._load()
    hyp_off = worst_basis = worst = 0.0
    gaps = []
    for b in range(B):
        s = sel[b]
        pix = data["choose"][b, 0, s]
        obj = (xyz[b].reshape(3, -1)[:, pix].double().t() * data["extent"][b] + data["lfborder"][b]).float().numpy()
        img = np.stack([data["x_map_choosed"][b, s, 0].numpy(), data["y_map_choosed"][b, s, 0].numpy()], 1)
        gcnt = int(info["inliers"][b])
        Rg, tg = R[b].cpu().numpy(), t[b].cpu().numpy()
        lib.oracle_set_cv_variant(ctypes.c_int(1))  # the kernel's null-space basis, OpenCV's numerics otherwise
        try:
            cc = _cv_hypothesis_counts(obj, img, subs[b].numpy())
            Rb, tb, cb, _ = opnp.pnp_ransac_cv(obj, img, K4, subs[b].numpy(), 1.0)
        finally:
            lib.oracle_set_cv_variant(ctypes.c_int(0))
        d = np.abs(cc.astype(int) - hcnt[b])
        assert d.max() <= 2, (b, d.max())
        hyp_off += int((d > 0).sum())
        assert gcnt == cb, (b, gcnt, cb)
        worst_basis = max(worst_basis, float(np.abs(Rg - Rb).max()), float(np.abs(tg - tb).max()))
        Ro, to, cnt, _ = opnp.pnp_ransac_cv(obj, img, K4, subs[b].numpy(), 1.0)
        gaps.append(gcnt - cnt)
        if noise_px == 0:
            assert abs(gcnt - cnt) <= 8, (b, gcnt, cnt)
        if gcnt == cnt:
            worst = max(worst, float(np.abs(Rg - Ro).max()), float(np.abs(tg - to).max()))
    gaps = np.array(gaps)
    print(f"noise {noise_px} px: kernel-basis oracle: {hyp_off} of {B * H} hypothesis counts off, max |dR|, |dt| "
          f"{worst_basis:.2e}; OpenCV numerics: selected count differs in {(gaps != 0).sum()} of {B} crops "
          f"(gaps {gaps[gaps != 0].tolist()}), max |dR|, |dt| where equal {worst:.2e}")
    assert hyp_off <= 0.002 * B * H, hyp_off
    assert worst_basis < 1e-4, worst_basis
    assert (gaps != 0).sum() <= 0.25 * B, gaps
    assert np.abs(gaps).max() <= 24, gaps
    assert abs(gaps.mean()) <= 2.0, gaps.mean()
    assert worst < (1e-4 if noise_px == 0 else 1e-2), worst


def _cv_hypothesis_counts(obj, img, subsets, thr=1.0):
    """Inlier count of every hypothesis under the OpenCV-semantics EPnP (oracle_pnp_hypotheses_diag)."""
    import ctypes
    lib = opnp._load()
    f = lib.oracle_pnp_hypotheses_diag
    f.restype = None
    H = len(subsets)
    R = np.zeros((H, 9), np.float32)
    t = np.zeros((H, 3), np.float32)
    cnt = np.zeros(H, np.int32)
    diag = np.zeros(H, np.int32)
    sub = np.ascontiguousarray(subsets, np.int32)
    f(opnp._p(np.ascontiguousarray(obj, np.float32)), opnp._p(np.ascontiguousarray(img, np.float32)),
      ctypes.c_int(len(obj)), opnp._p(K4), opnp._p(sub), ctypes.c_int(H), ctypes.c_float(thr), ctypes.c_int(1),
      opnp._p(R), opnp._p(t), opnp._p(cnt), opnp._p(diag))
    return cnt
