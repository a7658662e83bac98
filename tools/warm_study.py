#!/usr/bin/env python3
"""IPM start-point study on dumped stationary bench ticks (tools/tick_dump.py): the device's single-direction IPM
(tools/ipm_emu.py, fp64) on every robot's QP of the dumped ticks under several start rules, reporting per rule the
mean iterations, the tail (p99, p99.9, max) and the per-tick maximum over robots, which sets the launch time at one
wave per SIMD. The GPU's own counts of the same ticks are printed first (they follow the emulator's closely).
usage: python tools/warm_study.py gpurun_out/r03c/tick_dump_metric.npz [--model diff] [--N 40] [--n 4096]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def build(d, t, model, N, n):
    from oracle.oracle import Oracle
    o = Oracle(model, N)
    p = f"t{t}_"
    B = min(n, d[p + "pose"].shape[0])
    qs = []
    for i in range(B):
        rs = int(d[p + "reset"][i]) if (p + "reset") in d else 0
        xb = np.zeros((N + 1, o.nx)) if rs else d[p + "xbar"][i].astype(np.float64)
        ub = np.zeros((N, o.nu)) if rs else d[p + "ubar"][i].astype(np.float64)
        nt = int(d[p + "tlen"][i])
        st = float(d[p + "steer"][i]) if (p + "steer") in d else 0.0
        x0, yref, We = o.prepare(d[p + "pose"][i].astype(np.float64), d[p + "vel"][i].astype(np.float64), st,
                                 d[p + "traj"][i][:nt].astype(np.float64), d[p + "carried"][i].astype(np.float64))
        qs.append(o.build_qp(xb, ub, x0, yref, We))
    Q = {k: np.stack([q[k] for q in qs]) for k in qs[0]}
    Q["idxbx"] = np.array([o.prm.idxbx[j] for j in range(o.nbx)])
    lam = d[p + "lam"][:B].astype(np.float64)  # [B][N+1][nv][2]
    warm = d[p + "warm"][:B].astype(bool)
    if (p + "reset") in d:
        warm &= d[p + "reset"][:B] == 0
    return Q, lam, warm, d[p + "gpu_iter"][:B]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--model", default="diff")
    ap.add_argument("--N", type=int, default=40)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--ticks", type=int, default=3)
    a = ap.parse_args()
    from ipm_emu import Emu
    d = np.load(a.dump)
    single = lambda mu, al, it: np.clip((1 - al) ** 2, 0.01, 0.5)  # noqa: E731
    rules = {
        "cold": None,
        "warm k=0.2": (0.2, 1e3),
        "warm k=1.0": (1.0, 1e3),
        "warm k=0.01": (0.01, 1e3),
    }
    res = {k: [] for k in list(rules) + ["gpu", "adaptive(prev<=12)"]}
    for t in range(a.ticks):
        Q, lam, warm, gpu = build(d, t, a.model, a.N, a.n)
        res["gpu"].append(gpu)
        it = {}
        for name, r in rules.items():
            w = None
            if r is not None:
                kap, cap = r
                # robots without a valid warm flag start cold (mu0 / t): the device's rule
                lp = np.where(warm[:, None, None], lam[..., 0], np.nan)
                up = np.where(warm[:, None, None], lam[..., 1], np.nan)
                w = (lp, up, kap, cap)
            e = Emu(Q)
            if w is not None:
                # per robot: warm where flagged, cold elsewhere
                cold = Emu(Q).solve(single=single)["iters"]
                ws = e.solve(single=single, warm=(np.nan_to_num(w[0]), np.nan_to_num(w[1]), w[2], w[3]))["iters"]
                it[name] = np.where(warm, ws, cold)
            else:
                it[name] = e.solve(single=single)["iters"]
            res[name].append(it[name])
        prev = d[f"t{t}_gpu_iter"] if t == 0 else res["gpu"][t - 1]
        res["adaptive(prev<=12)"].append(np.where(warm & (prev[:len(warm)] <= 12), it["warm k=0.2"], it["cold"]))
    print(f"{'rule':24s} {'mean':>6s} {'p99':>5s} {'p99.9':>6s} {'max':>4s}  per-tick max")
    for name, v in res.items():
        allv = np.concatenate(v)
        print(f"{name:24s} {allv.mean():6.2f} {np.percentile(allv, 99):5.1f} {np.percentile(allv, 99.9):6.1f} "
              f"{allv.max():4d}  {[int(x.max()) for x in v]}")


if __name__ == "__main__":
    main()
