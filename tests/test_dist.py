"""Multi-process instance sharding on CPU (gloo, world_size 2): the contract bench.py uses on RCCL.

Each rank owns a contiguous shard of the seeded fleet (sharding.shard_range + make_fleet(start=...)), steps
its robots in closed loop, and the per-tick commands are all-gathered to every rank; the result must equal
the single-process run of the whole fleet exactly (instances are independent: no data-path collective).
The per-rank solver here is the CPU oracle, since the test runs without a GPU; the GPU path is the same code
with BatchSolver in place of the oracle (bench.py).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nmpc_nav_control_amd.sharding import CommandGather, TimedRegion, mixed_counts, shard_range

MODEL, N, TOTAL, TICKS = "diff", 10, 11, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from helpers import oracle_closed_loop
        lo, hi = shard_range(TOTAL, rank, world)
        counts = [b - a for a, b in (shard_range(TOTAL, r, world) for r in range(world))]
        log = []
        with TimedRegion() as tr:
            oracle_closed_loop(MODEL, N, hi - lo, TICKS, start=lo, u0_log=log)
        gather = CommandGather(2, counts, torch.device("cpu"))
        fleet = [gather([torch.from_numpy(u.T.astype(np.float32))]).numpy() for u in log]
        if rank == 0:
            np.savez(out, u0=np.stack(fleet), elapsed=tr.elapsed)
    finally:
        dist.destroy_process_group()


def test_shard_range_covers_fleet():
    for total in (0, 1, 7, 4096, 65536):
        for world in (1, 2, 3, 8):
            rs = [shard_range(total, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)
    assert mixed_counts(8192, ["diff", "omni4", "tric"]) == [("diff", 2731), ("omni4", 2731), ("tric", 2730)]


def test_gloo_world2_sharded_equals_single(tmp_path):
    from helpers import oracle_closed_loop
    out = str(tmp_path / "r0.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    log = []
    oracle_closed_loop(MODEL, N, TOTAL, TICKS, u0_log=log)
    ref = np.stack([u.T.astype(np.float32) for u in log])
    assert got["u0"].shape == ref.shape
    assert np.array_equal(got["u0"], ref)
    assert float(got["elapsed"]) > 0


# ---- the shipping driver loop (nmpc_nav_control_amd/fleet.py, bench.py) on gloo -----------------------------
MIXED = [("diff", 3), ("omni4", 2), ("tric", 3)]  # robots per rank and model (weak scaling)
MIX_N, MIX_TICKS, MIX_SEED = 8, 3, 20250824 + 4


def _node(world, rank, models, decoupled=False):
    from cpu_fleet_solver import OracleFleetSolver
    from nmpc_nav_control_amd.fleet import FleetNode
    return FleetNode(models, MIX_N, MIX_SEED, torch.device("cpu"), rank=rank, world=world, gather=True,
                     solver_factory=OracleFleetSolver, decoupled=decoupled)


def _fleet_worker(rank, world, port, out, decoupled=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        node = _node(world, rank, MIXED, decoupled)
        assert node.decoupled == decoupled
        logs = []
        with TimedRegion() as tr:
            for _ in range(MIX_TICKS):
                node.step()  # bench.py's timed step: tick_all + accumulate + all-gather of [u0; status]
                logs.append(node.gathered.numpy().copy())
        if rank == 0:
            np.savez(out, g=np.stack(logs), elapsed=tr.elapsed, iters=node.iters_sum.numpy(),
                     fails=node.fail_cnt.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("decoupled", [False, True])
def test_gloo_world2_fleet_node_equals_single(tmp_path, decoupled):
    """World 2 over gloo runs bench.py's FleetNode (mixed diff+omni4+tric fleet, per-rank instance shards,
    per-tick all-gather of u0 + status through sharding.CommandGather) with the oracle behind the solver
    interface; the gathered fleet commands equal a single-process joined node holding the whole fleet, bit for
    bit. decoupled=True runs the decoupled-stream code path (each fleet stages its commands into a double-buffered
    slot after its own tick, the gather collects the slot), which on the GPU keeps the streams' closed loops
    independent while gathering every tick (bench.py's mixed config at world > 1)."""
    out = str(tmp_path / "fleet.npz")
    mp.spawn(_fleet_worker, args=(2, _free_port(), out, decoupled), nprocs=2, join=True)
    got = np.load(out)
    single = _node(1, 0, [(m, 2 * b) for m, b in MIXED])
    ref = []
    for _ in range(MIX_TICKS):
        single.step()
        ref.append(single.gathered.numpy().copy())
    ref = np.stack(ref)  # [T][5][sum 2B]: model-major
    # the world-2 gather is rank-major: [rank 0: diff, omni4, tric | rank 1: diff, omni4, tric]
    cols = []
    off_single = np.cumsum([0] + [2 * b for _, b in MIXED])
    per_rank = sum(b for _, b in MIXED)
    for r in range(2):
        for j, (_, b) in enumerate(MIXED):
            cols.append(ref[:, :, off_single[j] + r * b: off_single[j] + (r + 1) * b])
    ref_rank_major = np.concatenate(cols, axis=2)
    assert got["g"].shape == ref_rank_major.shape == (MIX_TICKS, 5, 2 * per_rank)
    assert np.array_equal(got["g"], ref_rank_major)
    assert (got["g"][:, 4] == 0).all()  # every solve succeeded
    assert np.abs(got["g"][:, :4]).max() > 0  # the commands are not trivially zero
    assert float(got["elapsed"]) > 0 and (got["fails"] == 0).all() and (got["iters"] > 0).all()


def test_stream_groups_hold_the_same_robots():
    """FleetNode groups (bench.py's metric / tric configs run 2): each model's rank-local robots split into
    contiguous groups that are separate Fleets; with the oracle behind the solver interface the grouped node's
    commands equal the ungrouped node's bit for bit (on the CPU the groups tick in turn, without streams)."""
    from cpu_fleet_solver import OracleFleetSolver
    from nmpc_nav_control_amd.fleet import FleetNode
    models = [("diff", 5), ("tric", 4)]
    mk = lambda g: FleetNode(models, MIX_N, MIX_SEED, torch.device("cpu"), groups=g,  # noqa: E731
                             solver_factory=OracleFleetSolver)
    one, three = mk(1), mk(3)
    assert [f.B for f in three.fleets] == [2, 2, 1, 2, 1, 1] and not three.decoupled
    for _ in range(MIX_TICKS):
        one.step()
        three.step()
    for name in ("u0", "cmd", "status"):
        a = torch.cat([getattr(f, name) for f in one.fleets], dim=-1)
        b = torch.cat([getattr(f, name) for f in three.fleets], dim=-1)
        assert torch.equal(a, b), name
    assert torch.equal(one.iters_sum, three.iters_sum)
