"""Farthest point sampling: oracle known answers on CPU; the HIP kernel bit-exact
(indices) against the oracle, ties included."""
import numpy as np
import pytest
import torch

from oracle.fps_oracle import farthest_point_sampling as fps_ref


def test_oracle_line_known_answer():
    pts = np.array([[0, 0, 0], [1, 0, 0], [2, 0, 0], [3, 0, 0], [4, 0, 0]], np.float32)
    assert fps_ref(pts, 4).tolist() == [0, 4, 2, 1]


@pytest.mark.gpu
@pytest.mark.parametrize("n,ns,kind", [(2600, 64, "rand"), (1000, 300, "lattice"), (16384, 32, "rand"),
                                       (5, 8, "rand")])
def test_fps_gpu_matches_oracle(dev, n, ns, kind):
    from pose_estimation_amd.fps import farthest_point_sampling
    rng = np.random.default_rng(n + ns)
    if kind == "lattice":  # many exact distance ties -> lowest index wins
        g = np.stack(np.meshgrid(np.arange(10), np.arange(10), np.arange(10), indexing="ij"), -1).reshape(-1, 3)
        pts = (g[rng.permutation(len(g))][:n] * 0.01).astype(np.float32)
    else:
        pts = (rng.random((n, 3)) * np.array([0.1, 0.08, 0.05])).astype(np.float32)
    B = 2
    batch = np.stack([pts, pts[::-1].copy()])
    got = farthest_point_sampling(torch.from_numpy(batch).to(dev), ns).cpu().numpy()
    for b in range(B):
        if n > 4096:  # the oracle's n x n matrix: check a prefix via the running-min restatement
            sel, d = [0], np.full(n, np.inf, np.float32)
            for _ in range(ns - 1):
                diff = batch[b] - batch[b][sel[-1]]
                d = np.minimum(d, np.sqrt(diff[:, 0] ** 2 + diff[:, 1] ** 2 + diff[:, 2] ** 2).astype(np.float32))
                sel.append(int(np.argmax(d)))
            ref = np.array(sel)
        else:
            ref = fps_ref(batch[b], ns)
        assert np.array_equal(got[b], ref), (b, np.nonzero(got[b] != ref)[0][:5])
