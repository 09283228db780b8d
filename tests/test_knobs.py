"""The package's environment surface (pose_estimation_amd/knobs.py): every KRRN_* name the Python
package reads is declared there with a default and a meaning, nothing reads os.environ around it,
and the C-ABI library reads no environment at all (its tuning is fixed at build time)."""
import os
import re

import pytest

from pose_estimation_amd import knobs

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pose_estimation_amd")


def _sources(ext):
    for root, _, files in os.walk(PKG):
        for f in files:
            if f.endswith(ext):
                p = os.path.join(root, f)
                with open(p) as fh:
                    yield p, fh.read()


def test_every_knob_read_is_declared():
    used = set()
    for p, s in _sources(".py"):
        used |= set(re.findall(r'knobs\.(?:flag|integer|text)\("(KRRN_[A-Z0-9_]+)"\)', s))
    assert used, "no knob reads found"
    assert used <= set(knobs.KNOBS), used - set(knobs.KNOBS)
    # and nothing declared is dead
    assert set(knobs.KNOBS) <= used, set(knobs.KNOBS) - used


def test_no_environment_reads_outside_the_registry():
    allowed = {"knobs.py": None, "distributed.py": {"WORLD_SIZE", "RANK", "LOCAL_RANK"}}
    for p, s in _sources(".py"):
        name = os.path.basename(p)
        reads = re.findall(r'os\.(?:environ|getenv)[\.\[(]?(?:get\()?\s*"?([A-Z_]*)', s)
        if name == "knobs.py":
            continue
        if name in allowed:
            assert set(reads) <= allowed[name], (p, reads)
        else:
            assert not reads, (p, reads)


def test_library_reads_no_environment():
    for p, s in _sources(".hip"):
        assert "getenv" not in s, p
    for p, s in _sources(".h"):
        assert "getenv" not in s, p


def test_undeclared_knob_is_an_error():
    with pytest.raises(KeyError):
        knobs.flag("KRRN_NOT_A_KNOB")


def test_defaults_are_the_shipped_configuration(monkeypatch):
    for k in knobs.KNOBS:
        monkeypatch.delenv(k, raising=False)
    assert knobs.flag("KRRN_WINO_X3") and knobs.flag("KRRN_GRAPH") and not knobs.flag("KRRN_DIAG_DROP")
    assert knobs.integer("KRRN_FUSION_CHUNK") == 16 and knobs.text("KRRN_HIP_LIB") is None
    monkeypatch.setenv("KRRN_FUSE_EDGES", "0")
    assert not knobs.flag("KRRN_FUSE_EDGES")
