"""Write-set audit of the two-slot pipeline's launch lists (tests/write_audit.py): every C-ABI call
of both slots' plans, run alone and in order, may change only the buffers it was given a writable
pointer into. This is the deterministic form of the round-3 cross-graph mismatch hunt:
a stray store from one slot's kernel into the other slot's live buffers would corrupt a consumer only
under overlap, but it changes the other slot's buffer here, at the call that makes it."""
import pytest
import torch

from pose_estimation_amd import KRRN, make_config
from pose_estimation_amd.pipeline import PipelinedPipeline
from pose_estimation_amd.synthetic import init_weights, make_batch

from test_gpu_pipeline import _history
from write_audit import audit, header_pointer_params

def _names(pp):
    out = {}
    for si, sl in enumerate(pp.slots):
        kp = sl.parts[0].kp
        for k, v in dict(p9=kp.p9, xyz=kp.xyz, normal=kp.normal, fx=kp.fx, fn=kp.fn, pred_t=kp.pred_t,
                         **{k: v for k, v in kp.fusion_bufs.items()}).items():
            if isinstance(v, torch.Tensor):
                out[f"slot{si}.{k}"] = v
            elif isinstance(v, (list, tuple)):
                for j, x in enumerate(v):
                    out[f"slot{si}.{k}[{j}]"] = x
    return out


def _audit_pipeline(dev, B, S, N):
    m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
    init_weights(m, 0)
    m = m.to(dev).eval()
    pp = PipelinedPipeline(m, B, S, N, dev, seed=0, split="heads")
    pp.load(make_batch(B, S, N, seed=1))
    pp.run()
    pp.run()
    torch.cuda.synchronize()
    runs = []
    for stage, lists in (("A", pp.stage_a), ("B", pp.stage_b)):
        for si in range(2):
            for pi, (plan, env) in enumerate(lists[si]):
                runs.append((f"{stage}{si}.{pi}", plan, env))
    extra = [(f"slot{si}", sl.parts[0]) for si, sl in enumerate(pp.slots)]
    owners = [sl.parts[0].kp.plan for sl in pp.slots]  # the stage views own no buffers
    names = _names(pp)
    rep = audit(runs, extra=extra, names=names, owners=owners)
    rep["n_names"] = len(names)
    print(f"audit B={B} S={S} N={N}: {rep['ops']} calls, {rep['regions']} buffers "
          f"({rep['bytes'] / 1e9:.2f} GB, {rep['named']} named) watched; {rep['n_violations']} stray writes, "
          f"{rep['n_input_changes']} const-input writes")
    for v in rep["violations"] + rep["input_changes"]:
        print("  ", v)
    return rep


def test_header_params_cover_plan_entry_points():
    """Every entry point a plan calls has its pointer parameters classified from the header."""
    params = header_pointer_params()
    for name in ("krrn_gcn_conv_f32", "krrn_conv3x3_wino_x3_f32", "krrn_gemm_panel_x3_f32", "krrn_knn_f32",
                 "krrn_pnp_ransac_f32", "krrn_points_gather_f32", "krrn_blas_gemm_run"):
        w, r = params[name]
        assert w and r, name
    w, r = params["krrn_gcn_conv_f32"]
    assert w == [14] and r == [0, 3, 7, 10, 11, 12]


@pytest.mark.gpu
def test_write_audit_small_after_history(dev):
    _history(dev)
    rep = _audit_pipeline(dev, 4, 64, 256)
    assert rep["ops"] > 800 and rep["named"] == rep["n_names"] and rep["regions"] > 100
    assert rep["n_violations"] == 0 and rep["n_input_changes"] == 0, rep


@pytest.mark.gpu
def test_write_audit_benched_shape(dev):
    rep = _audit_pipeline(dev, 64, 120, 1000)
    assert rep["ops"] > 800 and rep["named"] == rep["n_names"] and rep["regions"] > 100 and rep["bytes"] > 1e9
    assert rep["n_violations"] == 0 and rep["n_input_changes"] == 0, rep
