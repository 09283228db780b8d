"""ORACLE (test infrastructure only). Restatement of farthest_point_sampling and
pairwise_distance of tools/script/sample_model.py:35-63 (numpy, f32 points)."""
import numpy as np


def pairwise_distance(A, B):
    diff = A[:, :, None] - B[:, :, None].T
    return np.sqrt(np.sum(diff ** 2, axis=1))


def farthest_point_sampling(points, n_samples):
    selected = np.zeros((n_samples,), dtype=int)
    dist_mat = pairwise_distance(points, points)
    pt_idx = 0
    dist_to_set = dist_mat[:, pt_idx]
    for i in range(n_samples):
        selected[i] = pt_idx
        dist_to_set = np.minimum(dist_to_set, dist_mat[:, pt_idx])
        pt_idx = np.argmax(dist_to_set)
    return selected
