#!/usr/bin/env python3
"""Study behind the IPM's infeasibility exit (DESIGN.md "Stopping rule"): the single-direction IPM of the
emulator (tools/ipm_emu.py, the device algorithm in fp64) on the QPs of a seeded closed-loop fleet with goal /
path renewals (the bench workload: reset ticks included), plus the same QPs made infeasible the way the failure
test does it (a carried vel-ref far outside its bound, so stage 1 cannot satisfy |v_ref| <= v_max).

Prints, per population, the distribution over robots of the largest bound multiplier seen at any iteration and
of the primal residual at the iterations where the multiplier crosses a threshold, so that a rule "stop with
status 4 once max lambda > L while res_ineq > R" can be checked for false positives on feasible robots.
usage: python tools/infeas_study.py [--robots 256] [--ticks 40] [--model diff] [--N 40]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--robots", type=int, default=256)
    ap.add_argument("--ticks", type=int, default=40)
    ap.add_argument("--model", default="diff")
    ap.add_argument("--N", type=int, default=40)
    ap.add_argument("--ttl", type=int, nargs=2, default=(10, 30))
    a = ap.parse_args()
    from cpu_fleet_solver import OracleFleetSolver
    from ipm_emu import Emu
    from nmpc_nav_control_amd.fleet import Fleet
    from oracle.oracle import Oracle

    f = Fleet(a.model, a.robots, a.N, 20250825, "cpu", renew=dict(ttl_min=a.ttl[0], ttl_max=a.ttl[1]),
              solver_factory=lambda m, n, b, device: OracleFleetSolver(m, n, b))
    o = Oracle(a.model, a.N)
    single = lambda mu, al, it: np.clip((1 - al) ** 2, 0.01, 0.5)  # noqa: E731
    feas, infe = [], []
    for t in range(a.ticks):
        sn = f.snapshot()
        if t >= 5 and t % 5 == 0:
            qs, qb = [], []
            for i in range(a.robots):
                rs = sn["reset"][i] if sn["reset"] is not None else 0
                xb = np.zeros_like(sn["xbar"][i]) if rs else sn["xbar"][i]
                ub = np.zeros_like(sn["ubar"][i]) if rs else sn["ubar"][i]
                n = int(sn["tlen"][i])
                st = sn["steer"][i] if sn["steer"] is not None else 0.0
                x0, yref, We = o.prepare(sn["pose"][i], sn["vel"][i], st, sn["traj"][i][:n], sn["carried"][i])
                qs.append(o.build_qp(xb, ub, x0, yref, We))
                bad = sn["carried"][i].copy()
                bad[0] = 50.0 if i % 2 else 1.5  # far outside, and just outside (one step of a_max dt cannot fix it)
                x0b, yrefb, Web = o.prepare(sn["pose"][i], sn["vel"][i], st, sn["traj"][i][:n], bad)
                qb.append(o.build_qp(xb, ub, x0b, yrefb, Web))
            for lst, store in ((qs, feas), (qb, infe)):
                Q = {k: np.stack([q[k] for q in lst]) for k in lst[0]}
                Q["idxbx"] = np.array([o.prm.idxbx[j] for j in range(o.nbx)])
                tr = []
                r = Emu(Q).solve(single=single, trace=tr)
                store.append((r["iters"], tr))
        f.tick()

    def summarize(name, runs):
        lmax = np.concatenate([np.max([t["lmax"] for t in tr], axis=0) for _, tr in runs])
        iters = np.concatenate([it for it, _ in runs])
        print(f"{name}: {lmax.size} robots, iterations mean {iters.mean():.1f} p99 {np.percentile(iters, 99):.0f} "
              f"max {iters.max()}")
        for q in (50, 99, 99.9, 100):
            print(f"   max lambda over the IPM, p{q}: {np.percentile(lmax, q):.3g}")
        for L in (1e3, 1e4, 1e5, 1e6, 1e8):
            # first iteration where lambda > L: the primal residual there
            first = []
            for _, tr in runs:
                lm = np.stack([t["lmax"] for t in tr])
                ri = np.stack([t["res_ineq"] for t in tr])
                dn = np.stack([t["done"] for t in tr])
                for b in range(lm.shape[1]):
                    hit = np.nonzero((lm[:, b] > L) & ~dn[:, b])[0]
                    if hit.size:
                        first.append((hit[0], ri[hit[0], b]))
            if first:
                its = np.array([x[0] for x in first])
                ris = np.array([x[1] for x in first])
                print(f"   lambda > {L:.0e}: {len(first)} robots, first at it {its.min()}..{its.max()} "
                      f"(median {np.median(its):.0f}), res_ineq there min {ris.min():.2e} median {np.median(ris):.2e}")
            else:
                print(f"   lambda > {L:.0e}: none")

    summarize("feasible (bench loop, renewals)", feas)
    summarize("infeasible (carried ref 50 / 1.5)", infe)


if __name__ == "__main__":
    torch.set_num_threads(1)
    main()
