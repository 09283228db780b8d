"""Shared parity helpers of the GPU tests (no GPU needed to import)."""
import torch


def knn_flips_at_ties(hip_idx, ref_idx, hv, rv, q_rows, name):
    """kNN decisions made on *predicted* coordinates: the HIP lists (on its vertices hv) may differ
    from the oracle's (on rv) only where two candidates are tied within (1) the coordinate
    perturbation between the runs — every point moved by at most delta (max-norm) moves each
    distance by <= 2 sqrt(d) delta — and (2) the rounding of the kNN's own f32 distance expression
    ((-2 <q,c> + |c|^2) + |q|^2, gcn3d.py:15-26): a few ulps of |q|^2 + |c|^2, which also lets a
    near-duplicate point sort ahead of the query's exact 0 and change which one drop-first drops.
    Checked in squared distances on the HIP vertices. Returns (mismatches, mismatches at ties)."""
    hv, rv = hv.double().cpu(), rv.double().cpu()
    hip_idx, ref_idx = hip_idx.long().cpu(), ref_idx.long().cpu()
    B, _, dim = hv.shape
    delta = float((hv - rv).abs().max())
    q = hv if q_rows is None else hv[:, q_rows.long().cpu()]
    bi = torch.arange(B)[:, None, None]
    ca, cb = hv[bi, hip_idx], hv[bi, ref_idx]
    da, db = (ca - q[:, :, None]).norm(dim=-1), (cb - q[:, :, None]).norm(dim=-1)
    mag = (q * q).sum(-1)[:, :, None] + (ca * ca).sum(-1) + (cb * cb).sum(-1)
    pert = 4 * dim ** 0.5 * delta
    tol2 = 16 * 2.0 ** -24 * mag + pert * (da + db + pert)
    bad = hip_idx != ref_idx
    tie = (da * da - db * db).abs() <= tol2
    n_bad, n_tie = int(bad.sum()), int((bad & tie).sum())
    print(f"  kNN({name}): {n_bad} of {bad.numel()} entries differ, {n_tie} at ties (delta {delta:.1e})")
    for b, t, j in (bad & ~tie).nonzero().tolist()[:5]:
        print(f"    b{b} q{t} rank{j}: hip {hip_idx[b, t].tolist()} {da[b, t].tolist()} ref {ref_idx[b, t].tolist()} "
              f"{db[b, t].tolist()} tol2 {float(tol2[b, t, j]):.2e}")
    return n_bad, n_tie
