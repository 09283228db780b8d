"""Loader / batcher host logic (SURVEY §8b loader API, §8f f2/f3) on CPU: the square-box snap
pinned by the reference's own detection fixture, and the size-bucketed batcher."""
import os

import numpy as np

from oracle import inputs_oracle as io
from pose_estimation_amd.dataset import LM_CROP_HIST, BucketBatcher, get_square_bbox

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_square_bbox_matches_reference_histogram():
    """All 13,425 YOLOv3 test boxes of the reference (dataset_config/test_bboxes/bbox_yolov3_all.json,
    fixture made by tests/golden/make_bbox_fixture.py) snap to exactly the crop-size histogram
    SURVEY.md §8d computed with the reference's get_square_bbox."""
    d = np.load(os.path.join(GOLDEN, "lm_test_bboxes_yolov3.npz"))
    hist = {}
    for bb in d["bbox"].astype(np.float64):
        rmin, rmax, cmin, cmax = get_square_bbox(list(bb))
        assert rmax - rmin == cmax - cmin
        assert 0 <= rmin and rmax <= 480 and 0 <= cmin and cmax <= 640
        hist[rmax - rmin] = hist.get(rmax - rmin, 0) + 1
    assert hist == LM_CROP_HIST


def test_square_bbox_edges():
    assert get_square_bbox([0.0, 0.0, 30.0, 50.0]) == (0, 80, 0, 80)
    r0, r1, c0, c1 = get_square_bbox([620.0, 460.0, 30.0, 30.0])
    assert (r1, c1) == (480, 640) and r1 - r0 == 40 and c1 - c0 == 40


def test_oracle_wrap_known_answer():
    m = np.zeros((4, 4), bool)
    m[1, 1] = m[2, 3] = m[3, 0] = True
    assert io.choose_wrap(m, 7).tolist() == [5, 11, 12, 5, 11, 12, 5]


class _FakeDS:
    def __init__(self, sizes):
        self.sizes = sizes

    def __len__(self):
        return len(self.sizes)

    def crop_size(self, i):
        return self.sizes[i]


def test_bucket_batcher_covers_every_crop_once():
    rng = np.random.default_rng(0)
    sizes = list(rng.choice([40, 80, 120, 160], size=203))
    bb = BucketBatcher(_FakeDS(sizes), bs=16, shuffle_buckets=True)
    seen = []
    for S, idx in bb:
        assert 1 <= len(idx) <= 16
        assert all(sizes[i] == S for i in idx)
        seen += idx
    assert sorted(seen) == list(range(len(sizes)))
    assert len(bb) == len(list(bb))
