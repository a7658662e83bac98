#!/usr/bin/env python3
"""IPM iteration statistics of the metric workload (diagnostic, GPU box).

Runs the bench fleet in closed loop and records, per tick, every robot's executed IPM iterations and exit
residuals, then reports the robot / wave (4 teams) / chip distributions that set the kernel time. With
--dump, the pre-tick state of the last few ticks (iterate, carried refs, measurements, references) is
saved so a tick can be replayed on the CPU oracle.
usage: python tools/iter_stats.py [--config metric] [--ticks 30] [--dump gpurun_out/iter_dump.npz]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import CONFIGS  # noqa: E402
from nmpc_nav_control_amd.fleet import Fleet  # noqa: E402
from nmpc_nav_control_amd.scenario import DEFAULT_SEED, make_fleet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="metric", choices=sorted(CONFIGS))
    ap.add_argument("--warm", type=int, default=20)
    ap.add_argument("--ticks", type=int, default=30)
    ap.add_argument("--dump", default=None)
    ap.add_argument("--dump-ticks", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = CONFIGS[args.config]
    m, B = cfg["models"][0]
    f = Fleet(m, B, cfg["N"], DEFAULT_SEED + cfg["idx"], dev)
    is_path = make_fleet(m, B, seed=DEFAULT_SEED + cfg["idx"])["is_path"]
    res = torch.zeros(3, B, device=dev)
    for _ in range(args.warm):
        f.tick()
    its, resid, dumps = [], [], []
    for t in range(args.ticks):
        if args.dump and t >= args.ticks - args.dump_ticks:
            torch.cuda.synchronize()
            xv, uv, cv = f.solver.state()
            dumps.append(dict(xbar=xv.to_tensor()[:, :B].cpu().numpy(), ubar=uv.to_tensor()[:, :B].cpu().numpy(),
                              carried=cv.to_tensor()[:, :B].cpu().numpy(), pose=f.pose.cpu().numpy(),
                              vel=f.vel.cpu().numpy(), traj=f.traj.cpu().numpy(), tlen=f.tlen.cpu().numpy(),
                              steer=None if f.steer is None else f.steer.cpu().numpy()))
        f.solver.run(f.pose, f.vel, f.traj, steer=f.steer, traj_len=f.tlen, cmd=f.cmd, u0=f.u0, status=f.status,
                     qp_iter=f.qp_iter, qp_res=res)
        if dumps and len(dumps) == t - (args.ticks - args.dump_ticks) + 1:
            dumps[-1]["qp_iter"] = f.qp_iter.cpu().numpy()
            dumps[-1]["u0"] = f.u0.cpu().numpy()
        its.append(f.qp_iter.cpu().numpy().copy())
        resid.append(res.cpu().numpy().copy())
        f.advance()
    its = np.array(its)  # [ticks][B]
    waves = its.reshape(args.ticks, -1, 4).max(axis=2)
    out = {
        "config": args.config,
        "robot_mean": float(its.mean()), "robot_hist": np.bincount(its.ravel()).tolist(),
        "wave_mean": float(waves.mean()), "wave_hist": np.bincount(waves.ravel()).tolist(),
        "chip_max_per_tick": its.max(axis=1).tolist(),
        "robot_mean_path": float(its[:, is_path].mean()), "robot_mean_goal": float(its[:, ~is_path].mean()),
        "tail_ge12_path_frac": float(is_path[np.nonzero((its >= 12).any(axis=0))[0]].mean())
        if (its >= 12).any() else None,
        "robots_ever_ge12": int((its >= 12).any(axis=0).sum()),
        "robot_p99": float(np.percentile(its, 99)), "robot_p999": float(np.percentile(its, 99.9)),
    }
    # does a robot's difficulty persist across ticks?
    hard = its >= 12
    out["hard_next_tick_given_hard"] = float((hard[1:] & hard[:-1]).sum() / max(1, hard[:-1].sum()))
    print(json.dumps(out), flush=True)
    if args.dump:
        np.savez_compressed(args.dump, its=its, resid=np.array(resid), is_path=is_path,
                            **{f"t{i}_{k}": v for i, d in enumerate(dumps) for k, v in d.items() if v is not None})


if __name__ == "__main__":
    main()
