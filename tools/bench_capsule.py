#!/usr/bin/env python3
"""Per-robot latency of the drop-in acados capsule ABI, driven the way the reference's ROS node drives it.

One NMPCNavControlDiff (nmpc_nav_control_amd/controller.py, the mirror of NMPCNavControlDiff.cpp) at the shipped
codegen horizon follows an arc in closed loop; each tick is NMPCNavControlDiff::run(): ocp_nlp_*_set calls,
{name}_acados_solve (host->device copies, one launch, synchronize, device->host copies), ocp_nlp_out_get. Reports
the wall time per run() and the solver's own time_tot, then the per-robot cost of {name}_acados_batch_solve over
n capsules, and the fp64 CPU oracle's time for the same solve on one core (reference point; acados itself is not
runnable here).
usage: python tools/bench_capsule.py [--N 80] [--ticks 200] [--batch 64,512]
"""
import argparse
import json
import os
import sys
import time

import ctypes

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from nmpc_nav_control_amd.controller import CmdVelDiff, NMPCNavControlDiff, Pose, Vel, batch_solve  # noqa: E402

W = [10, 10, 5, 0, 0, 0, 0, 1, 1]


def refs(t0, n):
    s = 0.02 * (t0 + np.arange(1, n + 1))
    return [Pose(0.5 * np.cos(0.6 * si), 0.5 * np.sin(0.6 * si), 0.6 * si + np.pi / 2) for si in s]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=80)
    ap.add_argument("--ticks", type=int, default=200)
    ap.add_argument("--batch", default="64,512")
    args = ap.parse_args()
    ctl = NMPCNavControlDiff(1 / 40, 0.270, 0.1, 1.0, 1.0, W, N=args.N)
    N = ctl.getHorizon()
    pose, vel = np.array([0.5, 0.0, np.pi / 2]), np.array([0.0, 0.0, 0.0])
    wall, tot = [], []
    for t in range(args.ticks):
        cmd = CmdVelDiff()
        t0 = time.perf_counter()
        ok, ms = ctl.run(Pose(*pose), Vel(*vel), refs(t, N + 1), cmd)
        wall.append((time.perf_counter() - t0) * 1e3)
        tot.append(ms)
        assert ok
        # kinematic plant: apply the command for one control period
        pose = pose + (1 / 40) * np.array([cmd.v * np.cos(pose[2]), cmd.v * np.sin(pose[2]), cmd.w])
        vel = np.array([cmd.v, 0.0, cmd.w])
    w = np.array(wall[10:])
    tt = np.array(tot[10:])
    out = {"N": N, "ticks": args.ticks, "run_wall_ms_mean": float(w.mean()), "run_wall_ms_p50": float(np.median(w)),
           "run_wall_ms_p99": float(np.percentile(w, 99)), "time_tot_ms_mean": float(tt.mean())}
    # batch_solve over n capsules with the state of the closed loop above
    for n in [int(v) for v in args.batch.split(",") if v]:
        ctls = [NMPCNavControlDiff(1 / 40, 0.270, 0.1, 1.0, 1.0, W, N=args.N) for _ in range(n)]
        for i, c in enumerate(ctls):
            x0 = np.array([0.5 + 0.01 * i, 0.0, np.pi / 2, 0.1, 0.1, 0.1, 0.1])
            c._cset(0, "lbx", x0)
            c._cset(0, "ubx", x0)
            for k, p in enumerate(refs(i, N + 1)):
                c.yref[k, :3] = [p.x, p.y, p.theta]
                c._wset(k, "yref", c.yref[k, : (c.nx if k == N else c.ny)])
        batch_solve(ctls)  # warm-up
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            st = batch_solve(ctls)
        dt = (time.perf_counter() - t0) / reps
        out[f"batch{n}_ms"] = dt * 1e3
        out[f"batch{n}_us_per_robot"] = dt * 1e6 / n
        out[f"batch{n}_failed"] = int((st != 0).sum())
        # the shim's own split of the last call: time_tot (pack + copies + launch + copies back), time_qp
        # (launch + copies back), executed IPM iterations
        c0 = ctls[0]
        tt, tq = ctypes.c_double(), ctypes.c_double()
        c0._L.ocp_nlp_get(c0._solver, b"time_tot", ctypes.byref(tt))
        c0._L.ocp_nlp_get(c0._solver, b"time_qp", ctypes.byref(tq))
        its = []
        for c in ctls:
            v = ctypes.c_int()
            c._L.ocp_nlp_get(c._solver, b"qp_iter", ctypes.byref(v))
            its.append(v.value)
        out[f"batch{n}_time_tot_ms"] = tt.value * 1e3
        out[f"batch{n}_time_qp_ms"] = tq.value * 1e3
        out[f"batch{n}_qp_iter_max"] = max(its)
    # the fp64 oracle on one core for the same kind of solve (reference point)
    try:
        from oracle.oracle import Oracle
        o = Oracle("diff", N)
        xb, ub = o.iterate_create()
        x0, yref, We = o.prepare(pose, vel, 0.0, np.array([[p.x, p.y, p.theta] for p in refs(0, N + 1)]),
                                 np.zeros(2))
        reps = 50
        t0 = time.perf_counter()
        for _ in range(reps):
            o.sqp_rti(xb, ub, x0, yref, We)
        out["oracle_fp64_1core_ms"] = (time.perf_counter() - t0) / reps * 1e3
    except Exception as e:  # the oracle is a reference point only
        out["oracle_fp64_1core_ms"] = f"unavailable: {e}"
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
