"""BPnP (lib/network/dnn/BPnP.py): the oracle's implicit-function gradients pinned
by finite differences of the re-solved pose on CPU; the HIP kernels (forward LM refinement,
backward) against the oracle on the GPU."""
import numpy as np
import pytest
import torch

from oracle import bpnp_oracle as bo

K_LM = np.array([[572.4114, 0, 325.2611], [0, 573.57043, 242.04899], [0, 0, 1]])


def scene(rng, n, noise=0.0):
    """Object points of a LineMOD-sized model, a random pose ~0.8 m in front of the camera."""
    z = (rng.random((n, 3)) - 0.5) * 0.15
    w = rng.normal(size=3)
    w *= rng.uniform(0.3, 2.5) / np.linalg.norm(w)
    y = np.concatenate([w, [rng.uniform(-0.1, 0.1), rng.uniform(-0.1, 0.1), rng.uniform(0.6, 1.1)]])
    x = bo._residual(y, np.zeros((n, 2)), z, K_LM).reshape(n, 2) + noise * rng.normal(size=(n, 2))
    return x, z, y


def depths(y, z, K):
    return ((z @ bo._rodrigues_np(y[:3]).T + y[3:]) @ K.T)[:, 2]


def test_oracle_gradients_match_finite_differences():
    """Zero-residual scene: the reference's stationarity f = 0 is the depth-weighted least-squares
    condition (weights s_i = depth), so its implicit gradients must equal central differences of
    the re-solved weighted problem w.r.t. x, z and K."""
    rng = np.random.default_rng(0)
    n = 10
    x, z, y = scene(rng, n)
    s = depths(y, z, K_LM)
    g = rng.normal(size=(1, 6))
    gx, gz, gK = bo.bpnp_backward(x[None], y[None], z, K_LM, g, dtype=torch.float64)

    def dy(xx, zz, KK):
        return bo.lm_refine(xx, zz, KK, y, weights=s)

    h = 1e-6
    for (i, k) in [(0, 0), (3, 1), (9, 0)]:
        xp, xm = x.copy(), x.copy()
        xp[i, k] += h
        xm[i, k] -= h
        fd = g[0] @ (dy(xp, z, K_LM) - dy(xm, z, K_LM)) / (2 * h)
        assert abs(fd - gx[0, i, k].item()) < 1e-5 * max(1.0, abs(fd)), (i, k, fd, gx[0, i, k].item())
    h = 1e-7
    for (i, m) in [(1, 0), (5, 2)]:
        zp, zm = z.copy(), z.copy()
        zp[i, m] += h
        zm[i, m] -= h
        fd = g[0] @ (dy(x, zp, K_LM) - dy(x, zm, K_LM)) / (2 * h)
        assert abs(fd - gz[i, m].item()) < 1e-4 * max(1.0, abs(fd)), (i, m, fd, gz[i, m].item())
    for (a, b) in [(0, 0), (1, 2)]:
        hk = 1e-4
        Kp, Km = K_LM.copy(), K_LM.copy()
        Kp[a, b] += hk
        Km[a, b] -= hk
        fd = g[0] @ (dy(x, z, Kp) - dy(x, z, Km)) / (2 * hk)
        assert abs(fd - gK[a, b].item()) < 1e-4 * max(1e-3, abs(fd)), (a, b, fd, gK[a, b].item())


def test_oracle_lm_recovers_pose():
    rng = np.random.default_rng(1)
    x, z, y = scene(rng, 30)
    y0 = y + np.concatenate([rng.normal(size=3) * 0.05, rng.normal(size=3) * 0.01])
    yr = bo.lm_refine(x, z, K_LM, y0)
    assert np.abs(yr - y).max() < 1e-9


def _gpu_case(dev, rng, bs, n, noise, per_crop=False):
    xs, zs, ys = zip(*[scene(rng, n, noise) for _ in range(bs)])
    z = np.stack(zs) if per_crop else zs[0]
    if not per_crop:  # one shared point set: re-project it under each crop's pose
        xs = [bo._residual(y, np.zeros((n, 2)), z, K_LM).reshape(n, 2) + noise * rng.normal(size=(n, 2)) for y in ys]
    x = np.stack(xs)
    return x, z, np.stack(ys)


@pytest.mark.gpu
@pytest.mark.parametrize("bs,n,per_crop", [(4, 40, False), (3, 200, True), (2, 7, False)])
def test_bpnp_backward_matches_oracle(dev, bs, n, per_crop):
    """krrn_bpnp_backward_f32 (f64 inside) vs the oracle's autograd in f64 at a noisy (non-zero
    residual) LM solution: relative 1e-5 of each gradient's max."""
    from pose_estimation_amd import bpnp
    rng = np.random.default_rng(10 + n)
    x, z, y = _gpu_case(dev, rng, bs, n, noise=0.8, per_crop=per_crop)
    y = np.stack([bo.lm_refine(x[b], z[b] if per_crop else z, K_LM, y[b]) for b in range(bs)]).astype(np.float32)
    g = rng.normal(size=(bs, 6)).astype(np.float32)
    f = lambda a: torch.tensor(np.asarray(a, np.float32), device=dev)  # noqa: E731
    gx, gz, gK = bpnp.backward(f(x), f(y), f(z), f(K_LM), f(g))
    rx, rz, rK = bo.bpnp_backward(x.astype(np.float32), y, z.astype(np.float32), K_LM.astype(np.float32), g,
                                  dtype=torch.float64)
    for got, ref in ((gx, rx), (gz, rz), (gK, rK)):
        got, ref = got.cpu().double(), ref.double()
        assert got.shape == ref.shape
        err = (got - ref).abs().max().item() / ref.abs().max().item()
        assert err < 1e-5, err


@pytest.mark.gpu
@pytest.mark.parametrize("noise", [0.0, 0.5])
def test_bpnp_solve_matches_oracle_lm(dev, noise):
    """krrn_bpnp_solve_f32 from a perturbed guess reaches the oracle LM minimum (noise-free:
    the true pose)."""
    from pose_estimation_amd import bpnp
    rng = np.random.default_rng(3)
    bs, n = 5, 60
    x, z, y = _gpu_case(dev, rng, bs, n, noise)
    y0 = y + np.concatenate([rng.normal(size=(bs, 3)) * 0.05, rng.normal(size=(bs, 3)) * 0.01], axis=1)
    f = lambda a: torch.tensor(np.asarray(a, np.float32), device=dev)  # noqa: E731
    got, cost = bpnp.solve(f(x), f(z), f(K_LM), ini_pose=f(y0), return_cost=True)
    got = got.cpu().double().numpy()
    for b in range(bs):
        ref = bo.lm_refine(x[b].astype(np.float32), z.astype(np.float32), K_LM.astype(np.float32),
                           y0[b].astype(np.float32))
        assert np.abs(got[b] - ref).max() < 2e-6, (b, got[b], ref)
        if noise == 0.0:
            assert np.abs(got[b] - y[b]).max() < 2e-6


@pytest.mark.gpu
def test_bpnp_autograd_function_end_to_end(dev):
    """BPnP.apply without ini_pose (EPnP-RANSAC init + LM) recovers the poses of outlier-free
    correspondences, and .backward() fills pts2d / pts3d / K grads with the kernel's values."""
    from pose_estimation_amd.bpnp import BPnP, BPnPModle, backward
    rng = np.random.default_rng(5)
    bs, n = 6, 100
    x, z, y = _gpu_case(dev, rng, bs, n, noise=0.3)
    f = lambda a: torch.tensor(np.asarray(a, np.float32), device=dev)  # noqa: E731
    x_t, z_t, K_t = f(x).requires_grad_(), f(z).requires_grad_(), f(K_LM).requires_grad_()
    P6 = BPnPModle()(x_t, z_t, K_t)
    assert np.abs(P6.detach().cpu().numpy()[:, 3:] - y[:, 3:]).max() < 5e-3
    w = torch.arange(1, 7, dtype=torch.float32, device=dev)
    (P6 * w).sum().backward()
    gx, gz, gK = backward(x_t, P6.detach(), z_t, K_t, w.expand(bs, 6).contiguous())
    assert torch.equal(x_t.grad, gx) and torch.equal(z_t.grad, gz) and torch.equal(K_t.grad, gK)
    assert torch.isfinite(x_t.grad).all()
