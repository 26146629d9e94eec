"""`python bench.py --gpus N` launches its own N ranks.

The driver's scaling run calls `python bench.py --gpus N` without torchrun; the
parent must start N rank processes (torch.distributed.run) before any GPU call,
wait for them and print ONE line carrying n_gpus = N and the process group's
world size.  --dry-run exercises that machinery on the CPU (gloo, no libpnr):
launcher, band shards, one all-gather per step, max-over-ranks timing."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, extra=()):
    env = dict(os.environ, PNR_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "3",
                        "--warmup", "1", "--dry-run", *extra], capture_output=True, text=True, env=env,
                       timeout=240, cwd=ROOT)
    return p


@pytest.mark.parametrize("n", [2, 3])
def test_bench_self_launches_n_ranks(n):
    p = _run(n)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["rccl_world"] == n and rec["dist_backend"] == "gloo"
    assert rec["frames_equal"] is True
    assert len(rec["ms_per_step_per_rank"]) == n
    assert rec["ms_per_step"] == max(rec["ms_per_step_per_rank"])
    assert "torch.distributed.run" in rec["launcher"]


def test_bench_single_rank_dry_run_needs_no_launcher():
    p = _run(1)
    assert p.returncode == 0, p.stderr[-3000:]
    rec = json.loads(p.stdout.strip())
    assert rec["n_gpus"] == 1 and "launcher" not in rec


def test_bench_launcher_reports_a_failing_rank():
    # an unknown flag makes every rank exit 2: the parent must exit non-zero, print no line
    env = dict(os.environ, PNR_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                        "--steps", "1", "--warmup", "0"], capture_output=True, text=True,
                       env=dict(env, PNR_BENCH_FAIL_RANK="1"), timeout=240, cwd=ROOT)
    assert p.returncode != 0
    assert p.stdout.strip() == ""
    assert "exited" in p.stderr
