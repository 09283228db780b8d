"""BatchPipeline (bench.py's step): forward + get_pose as one graph-capturable plan, with the
pose step on its own stream beside fusion + TBase. The step must equal the public API path
(KRRN.forward + get_pose) fed the same device-drawn permutations / subsets, and a hipGraph
replay must equal an eager run bit for bit."""
import pytest
import torch

from pose_estimation_amd import KRRN, get_pose, make_config
from pose_estimation_amd.pipeline import BatchPipeline
from pose_estimation_amd.synthetic import init_weights, make_batch

pytestmark = pytest.mark.gpu


def _snap(pl):
    r = pl.results()
    return {k: v.clone() for k, v in r.items()}


@pytest.mark.parametrize("parts", [1, 2])
def test_pipeline_matches_api_and_graph(dev, parts):
    B, S, N = 4, 64, 256
    m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
    init_weights(m, 0)
    m = m.to(dev).eval()
    d = make_batch(B, S, N, seed=21)
    pl = BatchPipeline(m, B, S, N, dev, parts=parts, seed=3)
    pl.load(d)
    seeds0 = [pt.kp.seed.clone() for pt in pl.parts]
    pl.run()
    torch.cuda.synchronize()
    eager = _snap(pl)
    assert torch.isfinite(eager["R"]).all() and torch.isfinite(eager["pred_t"]).all()

    # the public API on the same inputs and the pipeline's own device draws
    for pt in pl.parts:
        sl = slice(pt.lo, pt.hi)
        perms = [pt.kp.perms[k].clone() for k, _, _ in pt.kp.perm_sizes]
        sub = {k: v[sl] for k, v in d.items() if torch.is_tensor(v) and v.shape[:1] == (B,)}
        out = m(sub["img_croped"].to(dev), sub["cloud"].to(dev), sub["choose"].to(dev), sub["cls_id"].to(dev),
                perms=perms)
        R, t = get_pose(out, sub, sel=pt.aux["sel"].clone(), subsets=pt.aux["subsets"].clone())
        torch.cuda.synchronize()
        assert torch.equal(out["pred_t"], eager["pred_t"][sl])
        assert torch.equal(R, eager["R"][sl])
        assert torch.equal(t, eager["t"][sl])

    # graph replay from the same RNG state == the eager step
    pl.capture()
    for pt, s0 in zip(pl.parts, seeds0):
        pt.kp.seed.copy_(s0)
    pl.step()
    torch.cuda.synchronize()
    replay = _snap(pl)
    for k in eager:
        assert torch.equal(replay[k], eager[k]), k


@pytest.mark.parametrize("split", ["backbone", "heads", "pose"])
def test_pipelined_matches_plain(dev, split):
    """Two-stage pipeline: the batch a half-step completes equals the plain step on the same
    slot (same seed, same kernels), eager and graph-replayed."""
    from pose_estimation_amd.pipeline import PipelinedPipeline
    B, S, N = 4, 64, 256
    m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
    init_weights(m, 0)
    m = m.to(dev).eval()
    d = make_batch(B, S, N, seed=22)
    plain = [BatchPipeline(m, B, S, N, dev, parts=1, seed=s) for s in (0, 1)]
    ref = []
    for p in plain:
        p.load(d)
        p.run()
        torch.cuda.synchronize()
        ref.append(_snap(p))
    pp = PipelinedPipeline(m, B, S, N, dev, seed=0, split=split)
    pp.load(d)
    s0 = [sl.parts[0].kp.seed.clone() for sl in pp.slots]
    pp.run()  # B of slot 0 (+ A of slot 1)
    torch.cuda.synchronize()
    got0 = {k: v.clone() for k, v in pp.results().items()}
    pp.run()  # B of slot 1 (+ A of slot 0)
    torch.cuda.synchronize()
    got1 = {k: v.clone() for k, v in pp.results().items()}
    for k in ref[0]:
        assert torch.equal(got0[k], ref[0][k]), k
        assert torch.equal(got1[k], ref[1][k]), k
    pp.capture()
    for sl, s in zip(pp.slots, s0):
        sl.parts[0].kp.seed.copy_(s)
    pp.reset()  # stage A again from the reset RNG state (split='pose': A draws the pool perms)
    pp.step()
    torch.cuda.synchronize()
    g0 = {k: v.clone() for k, v in pp.results().items()}
    for k in ref[0]:
        assert torch.equal(g0[k], ref[0][k]), k


def _history(dev):
    """Build, run and free launch plans of other shapes first: the allocator and stream-pool history
    under which the round-2 pipelined/plain mismatch showed (tests/test_gpu_krrn.py and
    tests/test_gpu_golden.py running earlier in the same process)."""
    for (B, S, N, parts) in ((2, 80, 256, 1), (3, 64, 300, 1), (4, 64, 256, 2), (1, 120, 1000, 1)):
        m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
        init_weights(m, 1)
        m = m.to(dev).eval()
        pl = BatchPipeline(m, B * parts, S, N, dev, parts=parts, seed=9)
        pl.load(make_batch(B * parts, S, N, seed=5))
        pl.run()
        torch.cuda.synchronize()
        del pl, m
    torch.cuda.synchronize()


@pytest.mark.parametrize("split", ["heads", "backbone"])
def test_pipelined_matches_plain_after_history(dev, split):
    """Regression for the round-2 race: after the history above, the eager pipelined half-steps and
    10 replays of the captured pipelined graphs (stage A of one slot beside stage B of the other)
    equal the plain step bit for bit."""
    from pose_estimation_amd.pipeline import PipelinedPipeline
    _history(dev)
    B, S, N = 4, 64, 256
    m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
    init_weights(m, 0)
    m = m.to(dev).eval()
    d = make_batch(B, S, N, seed=22)
    ref = []
    for s in (0, 1):
        p = BatchPipeline(m, B, S, N, dev, parts=1, seed=s)
        p.load(d)
        p.run()
        torch.cuda.synchronize()
        ref.append(_snap(p))
    pp = PipelinedPipeline(m, B, S, N, dev, seed=0, split=split)
    pp.load(d)
    s0 = [sl.parts[0].kp.seed.clone() for sl in pp.slots]
    for h in range(2):
        pp.run()
        torch.cuda.synchronize()
        got = _snap(pp)
        for k in ref[h]:
            assert torch.equal(got[k], ref[h][k]), (h, k)
    pp.capture()
    for rep in range(10):
        for sl, s in zip(pp.slots, s0):
            sl.parts[0].kp.seed.copy_(s)
        pp.reset()
        for h in range(2):
            pp.step()
            torch.cuda.synchronize()
            got = _snap(pp)
            for k in ref[h]:
                assert torch.equal(got[k], ref[h][k]), (rep, h, k)


def test_pipelined_graph_benched_shape(dev):
    """The bench's exact step (config 2: B = 64, S = 120, N = 1000, PipelinedPipeline(split='heads'),
    hipGraph replay, device-drawn permutations / subsets) equals the plain step of the same slot,
    and the plain step equals the public API (KRRN.forward + get_pose) fed the same device draws."""
    from pose_estimation_amd.pipeline import PipelinedPipeline
    B, S, N = 64, 120, 1000
    m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
    init_weights(m, 0)
    m = m.to(dev).eval()
    d = make_batch(B, S, N, seed=1)
    plain = BatchPipeline(m, B, S, N, dev, parts=1, seed=0)
    plain.load(d)
    plain.run()
    torch.cuda.synchronize()
    ref = _snap(plain)
    pt = plain.parts[0]
    perms = [pt.kp.perms[k].clone() for k, _, _ in pt.kp.perm_sizes]
    out = m(d["img_croped"].to(dev), d["cloud"].to(dev), d["choose"].to(dev), d["cls_id"].to(dev), perms=perms)
    R, t = get_pose(out, d, sel=pt.aux["sel"].clone(), subsets=pt.aux["subsets"].clone())
    torch.cuda.synchronize()
    assert torch.equal(out["pred_t"], ref["pred_t"])
    assert torch.equal(R, ref["R"]) and torch.equal(t, ref["t"])
    del out, plain
    pp = PipelinedPipeline(m, B, S, N, dev, seed=0, split="heads")
    pp.load(d)
    s0 = [sl.parts[0].kp.seed.clone() for sl in pp.slots]
    pp.run()
    torch.cuda.synchronize()
    pp.capture()
    for rep in range(5):
        for sl, s in zip(pp.slots, s0):
            sl.parts[0].kp.seed.copy_(s)
        pp.reset()
        pp.step()
        torch.cuda.synchronize()
        got = _snap(pp)
        for k in ref:
            assert torch.equal(got[k], ref[k]), (rep, k)


def test_benched_step_graph_after_history(dev):
    """bench.py's step as benched (config 2: one hipGraph of the whole path, the plan's branches as
    graph branches) after the allocation history above: graph replays alternating
    between two RNG states each equal the eager serial step of that state bit for bit (a replay that
    read a buffer before this step wrote it would see the other state's values)."""
    _history(dev)
    B, S, N = 64, 120, 1000
    m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
    init_weights(m, 0)
    m = m.to(dev).eval()
    pl = BatchPipeline(m, B, S, N, dev, parts=1, seed=0)
    pl.load(make_batch(B, S, N, seed=1))
    seeds = [pl.parts[0].kp.seed.clone(), pl.parts[0].kp.seed.clone() + 12345]
    refs = []
    for sd in seeds:
        pl.parts[0].kp.seed.copy_(sd)
        pl.run()
        torch.cuda.synchronize()
        refs.append(_snap(pl))
    pl.capture()
    for rep in range(4):
        pl.parts[0].kp.seed.copy_(seeds[rep % 2])
        pl.step()
        torch.cuda.synchronize()
        got = _snap(pl)
        for k in refs[rep % 2]:
            assert torch.equal(got[k], refs[rep % 2][k]), (rep, k)
