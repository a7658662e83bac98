"""The stationary bench loop's goal / path renewal (scenario.py, fleet_sim.hip), on the CPU.

The reference's node solves only while it holds a goal or a path and resets its controller on every new one
(NMPCNavControlROS.cpp:304-327); the bench fleet re-issues goals / paths on arrival or after a ttl. These tests pin
the host mirror of the harness hash to the library's (a host function: no GPU), the renewal rule, and that a
renewal depends only on (seed, global index, event count): world 2 over gloo equals one process, renewals included.
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nmpc_nav_control_amd._lib import lib
from nmpc_nav_control_amd.scenario import RENEW, fleet_hash, fleet_ttl, fleet_u, make_fleet, renew_step

SHORT = dict(ttl_min=1, ttl_max=3)  # a renewal every 1-3 ticks


def test_hash_matches_library():
    L = lib()
    rng = np.random.default_rng(0)
    for _ in range(200):
        seed, idx, c = (int(v) for v in rng.integers(0, 2 ** 32, 3, dtype=np.uint64))
        assert L.nmpc_fleet_hash(seed, idx, c) == int(fleet_hash(seed, idx, c))
    # vectorised over robots, and the draws are 24-bit uniforms
    idx = np.arange(100000, dtype=np.uint64)
    u = fleet_u(20250825, idx, 1, 0)
    assert ((u >= 0) & (u < 1)).all() and abs(u.mean() - 0.5) < 0.01
    assert np.array_equal(u * 16777216.0, np.floor(u * 16777216.0))


def test_initial_ttl_spreads_renewals():
    fl = make_fleet("diff", 4096, seed=7)
    t = fl["ttl"]
    assert t.min() >= 1 and t.max() <= RENEW["ttl_max"]
    # uniform first ttl: about 1/ttl_max of the fleet renews at every tick from the start
    assert abs(np.mean(t <= 24) - 24 / RENEW["ttl_max"]) < 0.02
    # a shard holds the robots of the same global indices
    sh = make_fleet("diff", 1000, seed=7, start=1500)
    assert np.array_equal(sh["ttl"], t[1500:2500])
    ttl = fleet_ttl(7, np.arange(4096), 3, RENEW["ttl_min"], RENEW["ttl_max"])
    assert ttl.min() >= RENEW["ttl_min"] and ttl.max() <= RENEW["ttl_max"]


def test_renew_rule():
    fl = make_fleet("diff", 64, seed=3)
    path, s = fl["path"].astype(np.float64), fl["s"].astype(np.float64)
    ev, ttl = fl["ev"].copy(), np.full(64, 5, np.int32)
    goal = int(np.nonzero(path[5] < 0)[0][0])
    arc = int(np.nonzero(path[5] > 0)[0][0])
    far = np.array([100.0, 100.0, 0.0])
    # ttl counts down without a renewal
    assert renew_step("diff", path, s, far, ev, ttl, 3, 0, goal) == 0 and ttl[goal] == 4 and ev[goal] == 0
    # arrival (within 1 cm and 1 deg of the goal) renews at once
    at = path[:3, goal].copy()
    at[2] += np.deg2rad(0.5)
    assert renew_step("diff", path, s, at, ev, ttl, 3, 0, goal) == 1 and ev[goal] == 1
    r = np.hypot(path[0, goal] - at[0], path[1, goal] - at[1])
    u = fleet_u(3, goal, 1, 1)
    assert abs(r - (RENEW["goal_r_lo"] + (RENEW["goal_r_hi"] - RENEW["goal_r_lo"]) * u)) < 1e-12
    assert ttl[goal] == fleet_ttl(3, goal, 1, RENEW["ttl_min"], RENEW["ttl_max"])
    # the heading error decides too (1 deg)
    at2 = path[:3, goal].copy()
    at2[2] += np.deg2rad(5.0)
    ttl[goal] = 9
    assert renew_step("diff", path, s, at2, ev, ttl, 3, 0, goal) == 0
    # a path robot whose ttl runs out gets a new arc near the robot, progress 0
    ttl[arc], s[arc] = 1, 2.0
    pose = path[:3, arc] + np.array([0.05, 0.0, 0.1])
    assert renew_step("diff", path, s, pose, ev, ttl, 3, 0, arc) == 1
    assert s[arc] == 0 and np.hypot(*(path[:2, arc] - pose[:2])) <= 0.2 and abs(path[2, arc] - pose[2]) <= 0.3
    assert 3.0 <= path[5, arc] <= 5.0 and 0.2 <= path[4, arc] <= 0.8


# ---- world 2 over gloo with renewals every 1-3 ticks -------------------------------------------------------
MODELS = [("diff", 3), ("tric", 2)]
N, TICKS, SEED = 8, 5, 20250824 + 9


def _node(world, rank, models):
    from cpu_fleet_solver import OracleFleetSolver
    from nmpc_nav_control_amd.fleet import FleetNode
    return FleetNode(models, N, SEED, torch.device("cpu"), rank=rank, world=world, gather=True,
                     solver_factory=OracleFleetSolver, renew=SHORT)


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        node = _node(world, rank, MODELS)
        logs = []
        for _ in range(TICKS):
            node.step()
            logs.append(node.gathered.numpy().copy())
        ev = torch.cat([f.ev for f in node.fleets]).numpy()
        if rank == 0:
            np.savez(out, g=np.stack(logs), renewals=int(node.cold_cnt.sum()))
        dist.all_reduce(torch.tensor([int(ev.sum())]))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_renewals_equal_single(tmp_path):
    """The renewals of each robot (new goal / path, reset on the next solve) depend on its global index only:
    world 2 over gloo gathers the same fleet commands as one process, bit for bit, over ticks with renewals."""
    out = str(tmp_path / "renew.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    single = _node(1, 0, [(m, 2 * b) for m, b in MODELS])
    ref = []
    for _ in range(TICKS):
        single.step()
        ref.append(single.gathered.numpy().copy())
    ref = np.stack(ref)
    cols, off = [], np.cumsum([0] + [2 * b for _, b in MODELS])
    for r in range(2):
        for j, (_, b) in enumerate(MODELS):
            cols.append(ref[:, :, off[j] + r * b: off[j] + (r + 1) * b])
    assert np.array_equal(got["g"], np.concatenate(cols, axis=2))
    evs = torch.cat([f.ev for f in single.fleets]).numpy()
    assert evs.min() >= 1, evs  # every robot renewed at least once (ttl <= 3)
    assert int(single.cold_cnt.sum()) > 0 and (got["g"][:, 4] == 0).all()
