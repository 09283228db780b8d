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


def test_linemod_tree_index_and_frames(tmp_path):
    """PoseDataset(root=...) on a LineMOD-layout tree: the split lists, gt.yml poses (benchvise's
    obj_id-2 entry), boxes snapped by get_square_bbox, frames decoded as the reference reads them
    (rgb[:, :, :3], depth / 1000 in f64 -> f32, mask channel 0 == 255; 'eval' reads segnet labels)
    and 2600 model points from the ascii PLY (/ 1000)."""
    import numpy as np
    from linemod_tree import write_tree
    from pose_estimation_amd.dataset import PoseDataset, get_square_bbox, ply_vtx

    from pose_estimation_amd.config import LM_OBJLIST
    w = write_tree(str(tmp_path), objs=LM_OBJLIST, per_obj=2)
    for mode in ("test", "eval"):
        ds = PoseDataset(mode, 500, False, str(tmp_path), 0.0, 8, cls_type="all")
        assert len(ds) == 26 and ds.sym_obj == [7, 8]
        assert ds.boxes == [get_square_bbox(it["bbox"]) for it in ds.tree.items]
        for i, it in enumerate(ds.tree.items):
            ref = w[(it["obj"], it["im"])]
            np.testing.assert_allclose(it["R"], ref["R"].astype(np.float64), atol=1e-7)
            np.testing.assert_allclose(it["t"], ref["t"].astype(np.float64), atol=1e-7)
            assert it["bbox"] == [float(v) for v in ref["bbox"]]
            rgb, depth, ml = ds.tree.read(i)
            assert np.array_equal(rgb, ref["rgb"])
            assert np.array_equal(depth, (ref["depth_mm"].astype(np.float64) / 1000.0).astype(np.float32))
            assert np.array_equal(ml, (ref["mask"] == 255).astype(np.uint8))
            assert ds.crop_size(i) in (80, 120)
        mp = ds.tree.model_points[6]
        assert mp.shape == (2600, 3) and np.abs(mp).max() <= 0.05
    v = ply_vtx(str(tmp_path / "models" / "obj_06.ply"))
    assert v.shape == (3000, 3) and v.dtype == np.float32


def test_linemod_tree_cat_only(tmp_path):
    from linemod_tree import write_tree
    from pose_estimation_amd.dataset import BucketBatcher, PoseDataset
    write_tree(str(tmp_path), objs=(6,), per_obj=4, sizes=(80, 120))
    ds = PoseDataset("test", 500, False, str(tmp_path), 0.0, 8, cls_type="cat")
    assert ds.objlist == [6] and len(ds) == 4
    batches = list(BucketBatcher(ds, 8))
    assert sorted(S for S, _ in batches) == [80, 120]
    assert sorted(i for _, idx in batches for i in idx) == [0, 1, 2, 3]
