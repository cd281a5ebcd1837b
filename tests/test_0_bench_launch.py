"""bench.py started directly with --gpus N > 1 (no torch.distributed.run):
it launches the N rank processes itself before any GPU call and relays rank
0's JSON line (bench.py launch_ranks).

CPU: the launcher's failure paths -- a rank that exits non-zero makes the
parent stop the other ranks (which are blocked in the gloo rendezvous) and
exit with that rank's code. GPU: two gloo ranks sharing the box's one GPU
render the headline frame (tiles t % 2) and reduce the film; the counters
equal a one-rank run's.

The test process itself never touches the GPU (this module sorts first).
"""
import json
import os
import subprocess
import sys
import time

import pytest

from tests.conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=120):
    env = dict(os.environ, **(env_extra or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    t0 = time.time()
    r = subprocess.run([sys.executable, BENCH] + args, env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout)
    return r, time.time() - t0


@pytest.mark.parametrize("fail_rank", [1, 0])
def test_launcher_failing_rank_stops_all(fail_rank):
    # the failing rank exits before any GPU call; the other one waits in the
    # gloo rendezvous until the launcher terminates it
    r, dt = _run(["--gpus", "2", "--backend", "gloo", "--steps", "1", "--warmup", "0", "--no-cpu"],
                 {"YK_BENCH_FAIL_RANK": str(fail_rank)})
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert f"rank {fail_rank} exited with 3" in r.stderr
    assert r.stdout.strip() == ""
    assert dt < 90


def test_world_size_mismatch_refused():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--no-cpu"], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_self_launch_two_ranks_gloo():
    common = ["--steps", "1", "--warmup", "0", "--no-cpu"]
    r2, _ = _run(["--gpus", "2", "--backend", "gloo"] + common, timeout=500)
    assert r2.returncode == 0, r2.stderr[-3000:]
    lines = [ln for ln in r2.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r2.stdout
    two = json.loads(lines[0])
    r1, _ = _run(["--gpus", "1"] + common, timeout=300)
    assert r1.returncode == 0, r1.stderr[-3000:]
    one = json.loads([ln for ln in r1.stdout.splitlines() if ln.startswith("{")][0])
    assert two["n_gpus"] == 2 and two["config"]["parallelism"] == "tiles%2"
    assert two["ms_reduce"] > 0
    for k in ("closest_rays", "shadow_rays", "camera_samples"):
        assert two["config"][k] == one["config"][k], (k, two["config"][k], one["config"][k])
    assert two["config"]["camera_samples"] == 1920 * 1080 * 256
    assert one["n_gpus"] == 1 and one["ms_reduce"] == 0
