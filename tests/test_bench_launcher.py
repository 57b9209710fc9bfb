"""bench.py's own 1 -> N launcher, exercised on CPU (gloo, world_size 2).

`python bench.py --gpus N` without an external torchrun spawns N rank processes
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* = 127.0.0.1) before touching HIP; this is
the code the driver's `--gpus 8` run hits.  `--cpu-dry` swaps only the device encode
for the oracle and RCCL for gloo, so the launcher, the barrier-bracketed timing, the
per-rank gather and the JSON line are the production ones."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                       text=True, timeout=timeout, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [1, 2])
def test_bench_launcher_cpu_dry(oracle_mod, world):
    stripe = 10 * 256 * 2 * 64  # sc = 128
    d = _run(["--gpus", str(world), "--cpu-dry", "--stripe-bytes", str(stripe), "--steps", "3",
              "--warmup", "1", "--cpu-seconds", "0"])
    assert d["n_gpus"] == world
    assert d["cpu_dry"] is True
    assert len(d["per_rank"]["wall_ms_per_step"]) == world
    assert all(d["per_rank"]["verified"])
    assert d["scaling"] == "weak" and d["steps"] == 3
    assert d["config"]["parallelism"] == f"stripe-per-gpu x{world}"
    # value = all ranks' bytes / the slowest rank's time
    padded = d["config"]["padded_stripe_bytes"]
    slowest = max(d["per_rank"]["wall_ms_per_step"]) * 1e-3 * d["steps"]
    assert d["value"] == pytest.approx(world * d["steps"] * padded / slowest / 2**30, rel=0.02)
    for key in ("metric", "value", "unit", "ms_per_step", "higher_is_better", "vs_baseline", "dtype",
                "data", "config", "roofline"):
        assert key in d


def test_bench_launcher_rank_failure_stops_job(oracle_mod):
    """A rank that dies before the rendezvous (bad ordinal, OOM ...) must not leave the
    other rank blocked in init / barrier: the launcher sees the first non-zero exit,
    terminates the rest and exits non-zero, well within 60 s."""
    import time
    stripe = 10 * 256 * 2 * 64
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-dry",
                        "--stripe-bytes", str(stripe), "--steps", "3", "--warmup", "1", "--cpu-seconds", "0",
                        "--fail-rank", "1"], capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    el = time.monotonic() - t0
    assert r.returncode != 0
    assert "rank 1 exited with 3" in r.stderr, r.stderr[-2000:]
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert el < 60, el


def test_bench_rank_rejects_missing_device():
    """A rank whose LOCAL_RANK has no GPU fails fast with a clear message (here: no GPU at
    all in the container, LOCAL_RANK 0)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update({"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-seconds", "0"],
                       capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert r.returncode == 2
    assert "only 0 GPU(s) visible" in r.stderr


def test_bench_launcher_builds_stale_oracle_once(oracle_mod, tmp_path):
    """With a stale liboracle.so (clay_oracle.c newer than it, as a fresh checkout can leave
    it), a world-2 run builds the checker exactly once -- in the launcher parent, before any
    rank starts -- instead of N ranks running make on, and loading, the same file at once."""
    src = os.path.join(ROOT, "oracle", "clay_oracle.c")
    so = os.path.join(ROOT, "oracle", "liboracle.so")
    src_st = os.stat(src)
    # make the library stale by moving it into the past (never the source into the future: a
    # future source mtime would keep every later build in other processes rebuilding)
    os.utime(so, (src_st.st_atime - 10, src_st.st_mtime - 10))
    log = tmp_path / "make.log"
    wrapper = tmp_path / "make"
    wrapper.write_text(f"#!/bin/sh\necho \"$@\" >> {log}\nexec /usr/bin/make \"$@\"\n")
    wrapper.chmod(0o755)
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    env["PATH"] = f"{tmp_path}:{env.get('PATH', '')}"
    stripe = 10 * 256 * 2 * 64
    try:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-dry",
                            "--stripe-bytes", str(stripe), "--steps", "2", "--warmup", "1", "--cpu-seconds", "0"],
                           capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    finally:
        os.utime(src, (src_st.st_atime, src_st.st_mtime))  # the source's times are untouched
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert all(d["per_rank"]["verified"])
    makes = log.read_text().splitlines() if log.exists() else []
    assert len(makes) == 1, makes
    assert os.path.getmtime(so) >= os.path.getmtime(src)
