#!/usr/bin/env python3
"""Time the batched PathDiscretizer (nmpc_path_discretize) on the device: seeded multi-segment paths
(lines and cubic Beziers, 1-4 segments per robot), N+1 = 41 poses per robot at dt = 1/40 s, inputs resident in
HBM. Prints one JSON line: robots/s, ms per launch (HIP events on the launch stream), bytes moved per launch.

With --tick: a whole path-following tick of diff robots (N = num_poses - 1), the two-launch form
(nmpc_path_discretize + nmpc_batch_run) against the one-launch nmpc_batch_run_path, ms per tick each.

usage: python tools/bench_path.py [--B 4096] [--num-poses 41] [--iters 50] [--tick]
"""
import argparse
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from nmpc_nav_control_amd.path import SEG_DOUBLES, discretize  # noqa: E402


def seeded_paths(B, max_segs=4, seed=20250824):
    rng = np.random.default_rng(seed)
    segs = np.zeros((B, max_segs, SEG_DOUBLES))
    nseg = rng.integers(1, max_segs + 1, B).astype(np.int32)
    p = rng.uniform(-2, 2, (B, 2))
    h = rng.uniform(-math.pi, math.pi, B)
    for j in range(max_segs):
        L = rng.uniform(0.5, 1.5, B)
        turn = rng.uniform(-1.0, 1.0, B)
        q = p + L[:, None] * np.stack([np.cos(h + turn / 2), np.sin(h + turn / 2)], 1)
        a = (L / 3)[:, None]
        P1 = p + a * np.stack([np.cos(h), np.sin(h)], 1)
        P2 = q - a * np.stack([np.cos(h + turn), np.sin(h + turn)], 1)
        c = [p, 3 * (P1 - p), 3 * (P2 - 2 * P1 + p), q - 3 * P2 + 3 * P1 - p]
        for k in range(4):
            segs[:, j, k], segs[:, j, 4 + k] = c[k][:, 0], c[k][:, 1]
        segs[:, j, 8] = h
        segs[:, j, 12] = rng.uniform(0.2, 0.8, B)
        p, h = q, h + turn
    nearest_u = rng.uniform(0, 1, B) * 0.5
    return segs, nseg, nearest_u


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--num-poses", type=int, default=41)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--tick", action="store_true")
    a = ap.parse_args(argv)
    if a.tick:
        return tick(a)
    dev = torch.device("cuda:0")
    segs, nseg, nu = seeded_paths(a.B)
    S, NS, U = (torch.from_numpy(x).to(dev) for x in (segs, nseg, nu))
    traj = torch.empty((a.num_poses, 3, a.B), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream()
    for _ in range(5):
        discretize(S, NS, U, 1 / 40, a.num_poses, traj=traj)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(a.iters):
        discretize(S, NS, U, 1 / 40, a.num_poses, traj=traj)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    # compulsory bytes: each robot's segment records + nseg + nearest_u in, the fp32 poses out
    nbytes = int(nseg.sum()) * SEG_DOUBLES * 8 + a.B * (4 + 8) + a.num_poses * 3 * 4 * a.B
    print(json.dumps(dict(metric="getNextNPoses robots/s", value=round(a.B / (ms * 1e-3), 1), B=a.B,
                          num_poses=a.num_poses, ms_per_launch=round(ms, 4), bytes_per_launch=nbytes,
                          achieved_GBs=round(nbytes / (ms * 1e-3) / 1e9, 2),
                          bound="latency (sequential fp64 march per robot)")), flush=True)


def tick(a):
    """Path-following tick: discretize + run (two launches) vs run_path (one launch), same robots and state.
    Each variant runs its own solver handle through `iters` warm-started ticks on fixed measurements."""
    from nmpc_nav_control_amd.batch import BatchSolver
    from nmpc_nav_control_amd.path import discretize as disc
    dev = torch.device("cuda:0")
    N, B = a.num_poses - 1, a.B
    segs, nseg, nu = seeded_paths(B)
    S, NS, U = (torch.from_numpy(x).to(dev) for x in (segs, nseg, nu))
    traj = torch.empty((N + 1, 3, B), dtype=torch.float32, device=dev)
    disc(S, NS, U, 1 / 40, N + 1, traj=traj)
    pose = traj[0].clone()
    vel = torch.zeros(3, B, device=dev)
    res = {}
    for name in ("two_launch", "one_launch"):
        s = BatchSolver("diff", N, B, device=dev)
        u0 = torch.zeros(2, B, device=dev)
        st = torch.zeros(B, dtype=torch.int32, device=dev)

        def step():
            if name == "two_launch":
                disc(S, NS, U, 1 / 40, N + 1, traj=traj)
                s.run(pose, vel, traj, u0=u0, status=st)
            else:
                s.run_path(pose, vel, S, NS, U, 1 / 40, traj_out=None, u0=u0, status=st)
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            step()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) / a.iters, 4)
        res[name + "_failed"] = int((st != 0).sum())
    print(json.dumps(dict(metric="path-following tick ms (diff N=%d, B=%d)" % (N, B), **res)), flush=True)


if __name__ == "__main__":
    main()
