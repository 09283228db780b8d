"""The forward plan's cross-stream scheduling is bit-neutral.

Six plan-build switches move launches between streams or split them, with the same kernels on the
same values, so DESIGN.md section 4 claims bit-identical results for each:
  hrnet.FUSE_EARLY      fuse terms that read one branch start on that branch's stream
  hrnet.MODULE_STREAMS  consecutive HRNet modules keep each branch on its stream (no barrier)
  hrnet.STAGE_STREAMS   HRNet stages chain per branch stream (transitions on their branch's stream)
  hrnet.FUSE_EDGES      each fuse output waits for its branches through capture edges (no module barrier)
  krrn.FUSION_EARLY     the fusion's cloud-only part runs beside the HRNet phase (stream 7)
  fusion.FUSION_CHUNK   the level-0 GCN GEMM + gather-conv in crop chunks
A missing dependency in any of them would let a consumer on one stream read a buffer before its
producer on another stream wrote it: in the tolerance-based parity tests that shows up only as an
intermittent mismatch. Here one plan is built with all seven off (one stream per module, no chunks)
and one with the shipped defaults, and every output of the serial run, the captured graph and a
replay must be EQUAL (torch.equal), as well as the fusion's level buffers.
"""
import pytest
import torch

from pose_estimation_amd import KRRN, fusion, hrnet, krrn, make_config
from pose_estimation_amd.fusion import level_sizes
from pose_estimation_amd.synthetic import init_weights, make_batch

pytestmark = pytest.mark.gpu

B, S, N = 20, 64, 256  # B = 20 > the 16-crop chunk: a 16-crop and a 4-crop chunk


def _run(dev, sd, args, perms):
    m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
    m.load_state_dict(sd)
    m = m.to(dev).eval()
    outs = []
    for _ in range(3):  # serial warm-up, capture (side streams as graph branches), replay
        outs.append({k: v.clone() for k, v in m(*args, perms=perms).items() if v is not None})
    torch.cuda.synchronize()
    plan = m.get_plan(B, S, N, True)
    bufs = {k: v.clone() for k, v in plan.fusion_bufs.items() if torch.is_tensor(v)}
    del m, plan
    torch.cuda.empty_cache()
    return outs, bufs


def test_scheduling_switches_are_bit_neutral(dev, monkeypatch):
    m0 = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
    sd = init_weights(m0, 0)
    d = make_batch(B, S, N, seed=11)
    args = (d["img_croped"].to(dev), d["cloud"].to(dev), d["choose"].to(dev), d["cls_id"].to(dev))
    g = torch.Generator().manual_seed(5)
    N1, N2, _, _ = level_sizes(N, 10)
    perms = [torch.randperm(N, generator=g)[:N1] for _ in range(4)] + [torch.randperm(N1, generator=g)[:N2]]
    perms = [p.to(dev) for p in perms]
    assert fusion.FUSION_CHUNK and fusion.FUSION_CHUNK < B
    base_outs, base_bufs = _run(dev, sd, args, perms)
    for name, mod in (("FUSE_EARLY", hrnet), ("MODULE_STREAMS", hrnet), ("STAGE_STREAMS", hrnet),
                      ("FUSE_EDGES", hrnet), ("FUSION_EARLY", krrn)):
        assert getattr(mod, name), name  # the shipped default is on
        monkeypatch.setattr(mod, name, False)
    monkeypatch.setattr(fusion, "FUSION_CHUNK", 0)
    flat_outs, flat_bufs = _run(dev, sd, args, perms)
    for r in range(3):
        for k in base_outs[0]:
            assert torch.equal(base_outs[r][k], base_outs[0][k]), (r, k)
            assert torch.equal(flat_outs[r][k], base_outs[0][k]), (r, k)
    assert set(base_bufs) == set(flat_bufs)
    for k in base_bufs:
        assert torch.equal(base_bufs[k], flat_bufs[k]), k
