"""Serial per-op write-set audit of compiled launch plans (test infrastructure).

Every C-ABI call of one or more plans runs alone, in order, on one stream; after each call the
raw bits of EVERY device buffer the plans own are checksummed. A buffer whose checksum changed must
be one the call was given a writable pointer into: a pointer parameter declared without `const` in
include/krrn_hip.h (the `out` / `workspace` fields of a krrn_conv_desc / krrn_small_desc, the `out`
array of krrn_randperm_multi_i32). Any other changed buffer is a write outside the call's declared
outputs: an out-of-bounds or stray store, found at the call that makes it whatever the timing, so
a write that only corrupts a concurrently running consumer under graph / stream overlap shows up
here with no concurrency at all. Calls that change one of their own const inputs are reported too.

Checksums are int64 sums of the buffer's 32-bit words (8-bit for byte buffers): any single changed
word changes the sum. A buffer the call points into counts as the call's whole buffer, so writes
into the wrong region of a buffer the call legitimately writes are not seen at this granularity.
"""
from __future__ import annotations

import bisect
import ctypes
import os
import re
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "krrn_hip.h")


def header_pointer_params(path: str = HEADER) -> Dict[str, Tuple[List[int], List[int]]]:
    """{entry point: (writable pointer arg positions, const pointer arg positions)} from the
    prototypes of include/krrn_hip.h (the trailing `void* stream` is neither)."""
    text = re.sub(r"/\*.*?\*/", " ", open(path).read(), flags=re.S)
    out = {}
    for name, params in re.findall(r"\bint\s+(krrn_\w+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
        ps = [p.strip() for p in params.split(",")]
        w, r = [], []
        for i, p in enumerate(ps):
            if "*" not in p or p.endswith("stream"):
                continue
            (r if p.startswith("const") else w).append(i)
        out[name] = (w, r)
    return out


_DESC_OUT = ("out", "workspace")
_DESC_IN = ("in_", "wt", "scale", "bias", "bias2", "res")


def _flatten(x, acc: list, seen: set):
    if id(x) in seen:
        return
    seen.add(id(x))
    if isinstance(x, torch.Tensor):
        acc.append(x)
    elif isinstance(x, (list, tuple)):
        for y in x:
            _flatten(y, acc, seen)
    elif isinstance(x, dict):
        for y in x.values():
            _flatten(y, acc, seen)
    elif hasattr(x, "__dict__") and not isinstance(x, (type, ctypes._SimpleCData)):
        for y in vars(x).values():
            if isinstance(y, (torch.Tensor, list, tuple, dict)):
                _flatten(y, acc, seen)


class Region:
    __slots__ = ("lo", "hi", "t", "label")

    def __init__(self, t: torch.Tensor, label: str):
        st = t.untyped_storage()
        self.lo = st.data_ptr()
        self.hi = self.lo + st.nbytes()
        self.t = t
        self.label = label


def plan_regions(objs: Sequence[Tuple[str, Any]]) -> List[Region]:
    """Every distinct CUDA storage reachable from the given (label, object) pairs (plans' buffers,
    plan objects' tensor attributes), sorted by address; overlapping storages are merged into the
    first one."""
    regs: Dict[int, Region] = {}
    for label, obj in objs:
        ts: list = []
        _flatten(obj, ts, set())
        for t in ts:
            if not t.is_cuda or t.untyped_storage().nbytes() == 0:
                continue
            r = Region(t, label)
            if r.lo not in regs:
                regs[r.lo] = r
    out = sorted(regs.values(), key=lambda r: r.lo)
    merged: List[Region] = []
    for r in out:
        if merged and r.lo < merged[-1].hi:
            continue
        merged.append(r)
    return merged


def checksums(regs: Sequence[Region]) -> torch.Tensor:
    sums = []
    for r in regs:
        st = r.t.untyped_storage()
        n = st.nbytes()
        u8 = torch.empty(0, dtype=torch.uint8, device=r.t.device).set_(st, 0, (n,))
        if n % 4 == 0:
            sums.append(torch.sum(u8.view(torch.int32), dtype=torch.int64))
        else:
            sums.append(torch.sum(u8, dtype=torch.int64))
    return torch.stack(sums).cpu()


class _Locator:
    def __init__(self, regs: Sequence[Region]):
        self.regs = regs
        self.los = [r.lo for r in regs]

    def find(self, p: int) -> Optional[int]:
        if not p:
            return None
        i = bisect.bisect_right(self.los, p) - 1
        if i >= 0 and self.regs[i].lo <= p < self.regs[i].hi:
            return i
        return None


def _ptr_value(a, env) -> Optional[int]:
    from pose_estimation_amd.runtime import Late
    if isinstance(a, Late):
        v = env.get(a.key)
        return v.data_ptr() if isinstance(v, torch.Tensor) else None
    if isinstance(a, ctypes.c_void_p):
        return a.value
    return None


def op_pointer_sets(op, env, loc: _Locator, host_objs: Dict[int, Any],
                    params: Dict[str, Tuple[List[int], List[int]]]) -> Tuple[set, set]:
    """(region indices the op may write, region indices it only reads)."""
    w_idx, r_idx = params.get(op.name, ([], []))
    wr, rd = set(), set()

    def add(p, writable):
        i = loc.find(p) if p else None
        if i is not None:
            (wr if writable else rd).add(i)

    for pos, a in enumerate(op.args[:-1]):  # the last one is the stream
        if isinstance(a, ctypes.Array):  # host arrays of device pointers (randperm_multi's outs)
            if a._type_ is ctypes.c_void_p:
                for v in a:
                    add(v, pos in w_idx)
            continue
        p = _ptr_value(a, env)
        if p is None:
            continue
        obj = host_objs.get(p)
        if obj is not None:  # a krrn_conv_desc array passed by address
            for d in obj:
                for f in _DESC_OUT:
                    if hasattr(d, f):
                        add(getattr(d, f), True)
                for f in _DESC_IN:
                    if hasattr(d, f):
                        add(getattr(d, f), False)
            continue
        add(p, pos in w_idx)
    return wr, rd - wr


def _host_desc_arrays(plans) -> Dict[int, Any]:
    from pose_estimation_amd.runtime import ConvDesc
    out = {}
    for plan in plans:
        stack = list(plan.buffers)
        while stack:
            x = stack.pop()
            if isinstance(x, (list, tuple)):
                stack.extend(x)
            elif isinstance(x, ctypes.Array) and x._type_ is ConvDesc:
                out[ctypes.addressof(x)] = x
    return out


def audit(runs: Sequence[Tuple[str, Any, dict]], extra: Sequence[Tuple[str, Any]] = (),
          names: Optional[Dict[str, torch.Tensor]] = None, max_report: int = 20,
          owners: Sequence[Any] = ()) -> Dict[str, Any]:
    """runs: (label, Plan, env) in execution order. Every plan buffer of every plan and of `owners`
    (the whole plans that sub-plan views in `runs` were cut from: a view owns no buffers) and the
    tensors reachable from `extra` are watched; `names` labels some of them in the report. Returns
    {'ops': n, 'regions': n, 'bytes': n, 'violations': [...], 'input_changes': [...]}: a violation is
    (label, op index, entry point, region label + shape, stream id)."""
    from pose_estimation_amd.runtime import Op
    params = header_pointer_params()
    plans = [p for _, p, _ in runs] + list(owners)
    objs = ([(f"{lab}.buffers", p.buffers) for lab, p, _ in runs] +
            [(f"owner{i}.buffers", p.buffers) for i, p in enumerate(owners)] + list(extra))
    regs = plan_regions(objs)
    loc = _Locator(regs)
    named = 0
    for nm, t in (names or {}).items():
        i = loc.find(t.data_ptr()) if isinstance(t, torch.Tensor) and t.is_cuda else None
        if i is not None:
            regs[i].label = nm
            named += 1
    host = _host_desc_arrays(plans)
    dev = regs[0].t.device
    stream = torch.cuda.current_stream(dev)
    torch.cuda.synchronize(dev)
    prev = checksums(regs)
    viol, inchg = [], []
    nops = 0
    for lab, plan, env in runs:
        env = dict(env)
        plan._streams(env, serial=True)
        for oi, op in enumerate(plan.ops):
            if not isinstance(op, Op):
                continue
            wr, rd = op_pointer_sets(op, env, loc, host, params)
            op(env)
            stream.synchronize()
            cur = checksums(regs)
            changed = set((cur != prev).nonzero().flatten().tolist())
            prev = cur
            nops += 1
            for i in sorted(changed - wr):
                rec = (lab, oi, op.name, f"{regs[i].label}{tuple(regs[i].t.shape)}", op.sid,
                       "const input" if i in rd else "not an argument")
                (inchg if i in rd else viol).append(rec)
    return {"ops": nops, "regions": len(regs), "bytes": sum(r.hi - r.lo for r in regs), "named": named,
            "violations": viol[:max_report], "n_violations": len(viol),
            "input_changes": inchg[:max_report], "n_input_changes": len(inchg)}
