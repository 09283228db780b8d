"""CPU oracle for BPnP: TEST INFRASTRUCTURE ONLY — imported by tests/
as the checker for the HIP kernels in pose_estimation_amd/csrc/bpnp.hip, never by the product
path.

Restates, in PyTorch-CPU autograd (f32 like the reference, or f64):
  * BPnP.backward       lib/network/dnn/BPnP.py:53-117 — implicit-function gradients of the PnP
    pose y = (angle-axis, t) w.r.t. the 2-D points x, the 3-D points z and K. Per crop and per
    pose parameter j the reference builds f_j = sum_i sum_k c_ikj * r_ik with
      r_i = x_i * s_i - q_i[0:2],  q_i = K [R(y) | t] [z_i; 1],  s_i = q_i[2]       (:85-96)
      c_ikj = -2 d(q_i[k] / s_i) / d y_j, kept differentiable (create_graph=True)  (:97-99, 128-141)
    and J_f* = d f / d(y, x, z, K) by autograd (:100-105); then J_y* = -J_fy^-1 J_f* (:107-111),
    grad_x[b] = g_b J_yx, grad_z = sum_b g_b J_yz, grad_K = sum_b g_b J_yK (:113-115).
  * batch_project / get_coefs                                  BPnP.py:128-159
  * kornia.geometry.conversions.angle_axis_to_rotation_matrix  (third-party, version unpinned;
    the published formula: Rodrigues with w / (theta + 1e-6), first-order I + [w]x where
    theta^2 <= 1e-6, the two branches blended by a 0/1 mask)
  * the forward's cv2.solvePnP(SOLVEPNP_ITERATIVE, useExtrinsicGuess=True) (BPnP.py:43-44):
    Levenberg-Marquardt on the summed squared reprojection error, restated in f64 numpy.
Parity: cv2 and kornia are absent, so the gradient formula is pinned on its own
math instead: at zero-residual correspondences the reference's stationarity condition f = 0 and
the least-squares one coincide, and the oracle's J_yx / J_yz match finite differences of the
re-solved pose (tests/test_bpnp.py).
"""
from __future__ import annotations

import numpy as np
import torch

KORNIA_EPS = 1e-6


def angle_axis_to_rotation_matrix(aa: torch.Tensor) -> torch.Tensor:
    """[B, 3] -> [B, 3, 3] (kornia's published formula, see the module docstring)."""
    theta2 = (aa * aa).sum(-1, keepdim=True)
    theta = torch.sqrt(theta2)
    w = aa / (theta + KORNIA_EPS)
    wx, wy, wz = w[:, 0:1], w[:, 1:2], w[:, 2:3]
    c, s = torch.cos(theta), torch.sin(theta)
    oc = 1.0 - c
    normal = torch.cat([c + wx * wx * oc, wx * wy * oc - wz * s, wy * s + wx * wz * oc,
                        wz * s + wx * wy * oc, c + wy * wy * oc, -wx * s + wy * wz * oc,
                        -wy * s + wx * wz * oc, wx * s + wy * wz * oc, c + wz * wz * oc], dim=1)
    rx, ry, rz = aa[:, 0:1], aa[:, 1:2], aa[:, 2:3]
    one = torch.ones_like(rx)
    taylor = torch.cat([one, -rz, ry, rz, one, -rx, -ry, rx, one], dim=1)
    mask = (theta2 > KORNIA_EPS).to(aa.dtype)
    return (mask * normal + (1.0 - mask) * taylor).view(-1, 3, 3)


def batch_project(P6: torch.Tensor, z: torch.Tensor, K: torch.Tensor) -> torch.Tensor:
    """BPnP.py:144-159: poses [bs, 6], points [n, 3], K [3, 3] -> pixels [bs, n, 2]."""
    bs, n = P6.shape[0], z.shape[0]
    zh = torch.cat([z, torch.ones(n, 1, dtype=z.dtype)], dim=-1)
    PM = torch.cat([angle_axis_to_rotation_matrix(P6[:, 0:3]), P6[:, 3:6].reshape(bs, 3, 1)], dim=-1)
    q = zh.matmul(PM.transpose(-2, -1)).matmul(K.t())
    return q[:, :, 0:2] / q[:, :, 2:3]


def _f(x: torch.Tensor, y: torch.Tensor, z: torch.Tensor, K: torch.Tensor) -> torch.Tensor:
    """The six stationarity functions f_j of one crop (BPnP.py:85-100) as one vector; x, z, K
    flattened."""
    n = x.numel() // 2
    R = angle_axis_to_rotation_matrix(y[0:3].view(1, 3))[0]
    P = torch.cat([R, y[3:6].view(3, 1)], dim=-1)
    q = K.view(3, 3).mm(P).mm(torch.cat([z.view(n, 3), torch.ones(n, 1, dtype=z.dtype)], dim=-1).t())  # [3, n]
    r = x.view(n, 2).t() * q[2:3] - q[0:2]                                                                 # [2, n]
    # coefficients c[i, k, j] = -2 d pi_k(z_i) / d y_j with their graph kept (get_coefs)
    yr = y.view(1, 6).repeat(n, 1)
    proj = batch_project(yr, z.view(n, 3), K.view(3, 3))                                                  # [n, n, 2]
    eye = torch.eye(n, dtype=z.dtype)
    coefs = torch.stack([-2 * torch.autograd.grad(proj[:, :, k], yr, eye, create_graph=True)[0] for k in range(2)],
                        dim=1)                                                                             # [n, 2, 6]
    return torch.stack([(coefs[:, :, j].t() * r).sum() for j in range(6)])


def bpnp_backward(pts2d, P6, pts3d, K, grad_out, dtype=torch.float32):
    """BPnP.backward: returns (grad_x [bs, n, 2], grad_z [n, 3], grad_K [3, 3]). pts3d may also be
    [bs, n, 3] (one set per crop; grad_z then [bs, n, 3])."""
    cv = lambda a: torch.as_tensor(np.asarray(a), dtype=dtype)  # noqa: E731
    x_all, y_all, z_all, K, g_all = cv(pts2d), cv(P6), cv(pts3d), cv(K), cv(grad_out)
    bs, n = x_all.shape[0], x_all.shape[1]
    per_crop = z_all.dim() == 3
    gx = torch.zeros(bs, n, 2, dtype=dtype)
    gz = torch.zeros_like(z_all)
    gK = torch.zeros(3, 3, dtype=dtype)
    for b in range(bs):
        z = z_all[b] if per_crop else z_all
        args = (x_all[b].reshape(-1), y_all[b].clone(), z.reshape(-1), K.reshape(-1))
        with torch.enable_grad():
            J = torch.autograd.functional.jacobian(_f, args)  # d f / d (x, y, z, K)
        J_fx, J_fy, J_fz, J_fK = (j.reshape(6, -1) for j in J)
        v = -(g_all[b].view(1, 6).mm(torch.inverse(J_fy)))  # -g J_fy^-1
        gx[b] = v.mm(J_fx).view(n, 2)
        if per_crop:
            gz[b] = v.mm(J_fz).view(n, 3)
        else:
            gz += v.mm(J_fz).view(n, 3)
        gK += v.mm(J_fK).view(3, 3)
    return gx, gz, gK


# ---- forward: Levenberg-Marquardt refinement (cv2.solvePnP ITERATIVE with a guess) ----------
def _rodrigues_np(w):
    return angle_axis_to_rotation_matrix(torch.as_tensor(np.asarray(w, np.float64)).view(1, 3))[0].numpy()


def _residual(y, x, z, K, sw=None):
    p = z @ _rodrigues_np(y[:3]).T + y[3:]
    q = p @ K.T
    e = q[:, :2] / q[:, 2:3] - x
    return (e if sw is None else e * sw[:, None]).reshape(-1)


def lm_refine(x, z, K, y0, iters: int = 100, weights=None):
    """Minimise sum_i w_i ||pi(z_i; y) - x_i||^2 (w = 1 by default) from y0 (f64, numerical
    Jacobian by central differences, multiplicative damping). Returns y [6]."""
    x, z, K = (np.asarray(a, np.float64) for a in (x, z, K))
    sw = None if weights is None else np.sqrt(np.asarray(weights, np.float64))
    y = np.asarray(y0, np.float64).copy()
    lam = 1e-3
    e = _residual(y, x, z, K, sw)
    cost = e @ e
    for _ in range(iters):
        J = np.empty((e.size, 6))
        for j in range(6):
            h = 1e-7 * max(1.0, abs(y[j]))
            d = np.zeros(6)
            d[j] = h
            J[:, j] = (_residual(y + d, x, z, K, sw) - _residual(y - d, x, z, K, sw)) / (2 * h)
        A, gvec = J.T @ J, J.T @ e
        improved = False
        for _ in range(30):
            step = np.linalg.solve(A + lam * np.diag(np.diag(A)), -gvec)
            yn = y + step
            en = _residual(yn, x, z, K, sw)
            cn = en @ en
            if cn <= cost:
                y, e, cost, lam, improved = yn, en, cn, max(lam * 0.1, 1e-12), True
                break
            lam *= 10.0
        if not improved or np.abs(step).max() < 1e-13 * max(1.0, np.abs(y).max()):
            break
    return y
