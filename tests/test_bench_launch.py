"""bench.py's multi-rank launch (`--gpus N` without torchrun: N fresh rank processes) in its
dry-run form on CPU (gloo, a host-delay step, the per-crop record all-gather): the driver's
SCALE command path prints one line with n_gpus = N and the whole-job crop rate."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus2_dry_run():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "4",
                        "--warmup", "1", "--batch", "8"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 16 and d["dry_run"]
    # value = crops over all ranks / max-over-ranks time
    assert abs(d["value"] - 2 * 8 * 4 / (d["ms_per_step"] * 4 / 1e3)) / d["value"] < 0.01


def test_bench_world_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_bench_config3_gpus2_dry_run():
    """BASELINE config 3 mode: one global batch of 256 crops bucketed by S (LineMOD histogram), every
    bucket split across the 2 ranks (distributed.bucket_shard), records all-gathered; strong scaling."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "3", "--gpus", "2", "--dry-run",
                        "--steps", "3", "--warmup", "1"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    c = d["config"]
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and c["global_batch"] == 256
    assert sum(c["buckets"].values()) == 256
    # rank 0 holds the first half (rounded up) of every bucket
    assert all(c["rank0_buckets"][S] == (n + 1) // 2 for S, n in c["buckets"].items())
    assert abs(d["value"] - 256 * 3 / (d["ms_per_step"] * 3 / 1e3)) / d["value"] < 0.01
