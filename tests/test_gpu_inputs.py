"""On-GPU input construction (krrn_crop_inputs_u8, krrn_choose_points) vs the numpy oracle of
PoseDataset._load_data on identical frames: normalised crop and point mask bit-exact, `choose`
exact when the mask is small (wrap padding), an order-preserving uniform N-subset of the mask
pixels when it is large, and cloud / x_map / y_map bit-exact for the chosen pixels."""
import numpy as np
import pytest
import torch

from oracle import inputs_oracle as io
from pose_estimation_amd.dataset import PoseDataset, build_inputs, get_square_bbox, synthetic_frames
from pose_estimation_amd.synthetic import LM_K

pytestmark = pytest.mark.gpu

K4 = [LM_K[0, 0], LM_K[1, 1], LM_K[0, 2], LM_K[1, 2]]


def _frames(dev, F, sizes, seed):
    fr = synthetic_frames(F, seed=seed, sizes=sizes)
    fd = {k: torch.from_numpy(fr[k]).to(dev) for k in ("rgb", "depth", "mask_label")}
    boxes = [get_square_bbox([float(v) for v in bb]) for bb in fr["bbox"]]
    return fr, fd, boxes


@pytest.mark.parametrize("S,N", [(40, 2000), (120, 1000), (80, 4096)])
def test_inputs_match_oracle(dev, S, N):
    F = 5
    fr, fd, boxes = _frames(dev, F, [S], seed=S)
    seed = torch.tensor([1234], dtype=torch.int64, device=dev)
    k4 = torch.tensor([K4] * F, dtype=torch.float32)
    out = build_inputs(fd, list(range(F)), boxes, N, k4, seed, stream_id=3)
    torch.cuda.synchronize()
    k4f = k4[0].numpy()
    for b in range(F):
        rmin, rmax, cmin, cmax = boxes[b]
        assert rmax - rmin == S
        img, m = io.crop_inputs(fr["rgb"][b], fr["depth"][b], fr["mask_label"][b], rmin, cmin, S)
        assert np.array_equal(out["img_croped"][b].cpu().numpy(), img)
        assert np.array_equal(out["point_mask"][b, 0].cpu().numpy().astype(bool), m)
        cnt = int(m.sum())
        assert int(out["mask_count"][b]) == cnt
        ch = out["choose"][b, 0].cpu().numpy()
        if cnt <= N:
            assert np.array_equal(ch, io.choose_wrap(m, N))
        else:
            cand = m.flatten().nonzero()[0]
            assert len(ch) == N and np.all(np.diff(ch) > 0) and np.isin(ch, cand).all()
        cloud, xm, ym = io.points(ch, fr["depth"][b], rmin, cmin, S, k4f)
        assert np.array_equal(out["cloud"][b].cpu().numpy(), cloud)
        assert np.array_equal(out["x_map_choosed"][b, :, 0].cpu().numpy(), xm)
        assert np.array_equal(out["y_map_choosed"][b, :, 0].cpu().numpy(), ym)


def test_subset_is_uniform(dev):
    """Every mask pixel enters the N-subset with probability N / count (np.random.shuffle's
    distribution): inclusion counts over 200 draws stay within 6 sigma of the mean."""
    fr, fd, boxes = _frames(dev, 1, [120], seed=4)
    N, draws = 1000, 200
    seed = torch.tensor([99], dtype=torch.int64, device=dev)
    k4 = torch.tensor([K4], dtype=torch.float32)
    hits = None
    for d in range(draws):
        out = build_inputs(fd, [0], boxes, N, k4, seed, stream_id=d)
        ch = out["choose"][0, 0]
        cnt = int(out["mask_count"][0])
        h = torch.zeros(120 * 120, device=dev)
        h[ch] = 1
        hits = h if hits is None else hits + h
    _, m = io.crop_inputs(fr["rgb"][0], fr["depth"][0], fr["mask_label"][0], boxes[0][0], boxes[0][2], 120)
    hm = hits.cpu().numpy()[m.flatten()]
    p = N / cnt
    assert cnt > N
    sigma = np.sqrt(draws * p * (1 - p))
    assert abs(hm.mean() - draws * p) < 0.05 * draws * p
    assert np.abs(hm - draws * p).max() < 6 * sigma


def test_pose_dataset_batch(dev):
    ds = PoseDataset("test", 1000, False, None, 0.0, 8, cls_type="all", num_frames=12, sizes=[80, 120])
    assert len(ds.objlist) == 13 and ds.sym_obj == [7, 8]
    idx = [i for i in range(len(ds)) if ds.crop_size(i) == 80]
    data = ds.batch(idx, dev)
    B = len(idx)
    assert data["img_croped"].shape == (B, 3, 80, 80) and data["choose"].shape == (B, 1, 1000)
    assert data["cloud"].shape == (B, 1000, 3) and data["cls_id"].shape == (B, 1)
    item = ds[idx[0]]
    assert item["cloud"].shape == (1000, 3)
