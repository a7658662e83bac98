"""bench.py's multi-rank launch path on the CPU (gloo): `python bench.py --gpus 2` without torchrun's environment
starts the two ranks itself (torch.distributed.run as a child process), every rank verifies the process group's
size against --gpus, and rank 0 prints exactly one JSON line with n_gpus 2. The ranks run the shipping FleetNode
loop (the mixed config: per-rank shards of all three models, per-tick command all-gather) with the fp64 oracle
behind the solver interface (tests/cpu_fleet_solver.py), as the other gloo tests do; on the GPU box the same
path runs BatchSolver over RCCL. A --gpus that disagrees with the launched world size exits non-zero."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")


def _run(args, env_extra=None, timeout=300):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "NMPC_BENCH_LAUNCHER"):
        env.pop(k, None)
    env["PYTHONPATH"] = os.pathsep.join([TESTS, ROOT, env.get("PYTHONPATH", "")])
    env["OMP_NUM_THREADS"] = "1"
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


CPU = ["--device", "cpu", "--test-solver", "cpu_fleet_solver:OracleFleetSolver", "--steps", "2", "--warmup", "1",
       "--closed-loop-warmup", "2", "--no-cpu-baseline"]


def test_gpus2_launches_two_ranks_and_prints_one_line():
    p = _run(["--gpus", "2", "--config", "mixed", "--batch-per-gpu", "6", *CPU])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["ranks"] == 2 and r["config"]["backend"] == "gloo"
    assert r["config"]["launcher"] == "bench.py --gpus 2"
    assert r["config"]["batch_per_gpu"] == 6 and r["config"]["global_batch"] == 12
    assert r["config"]["rccl_gather"] is True  # mixed at world > 1: the whole-fleet gather
    assert r["failed_solves"] == 0 and r["value"] > 0
    # value: robots of all ranks x steps / the max-over-ranks timed region (2 steps)
    assert abs(r["value"] - (2 * 6) * 2 / (r["ms_per_step"] * 2e-3)) / r["value"] < 1e-3


def test_world_size_mismatch_exits_nonzero():
    # a "torchrun" environment of one rank with --gpus 2: the check fails before any work
    p = _run(["--gpus", "2", "--config", "metric", "--batch-per-gpu", "2", *CPU],
             env_extra={"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0"})
    assert p.returncode == 3 and not p.stdout.strip(), (p.returncode, p.stdout, p.stderr[-2000:])
    assert "process group has 1 rank" in p.stderr


def test_single_rank_default():
    p = _run(["--config", "metric", "--batch-per-gpu", "3", *CPU])
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip())
    assert r["n_gpus"] == 1 and r["config"]["ranks"] == 1 and r["config"]["backend"] is None
