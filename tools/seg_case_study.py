#!/usr/bin/env python3
"""The segmented Riccati inside the device IPM (tools/ipm_emu.py) on the QPs of tests/test_gpu_seg.py's first
tick (the oracle closed loop of tests/helpers.py, cold start): per robot the IPM iteration count with the serial
solve and with the segmented one for each master form of tools/seg_ipm_study.seg_riccati, and the u0 difference.
usage: python tools/seg_case_study.py [--model diff] [--N 80] [--B 9] [--S 2 5 8] [--masters gj chol cholcc]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="diff")
    ap.add_argument("--N", type=int, default=80)
    ap.add_argument("--B", type=int, default=9)
    ap.add_argument("--S", type=int, nargs="+", default=[2, 5, 8])
    ap.add_argument("--masters", nargs="+", default=["gj", "chol", "cholcc"])
    a = ap.parse_args()
    from helpers import oracle_closed_loop
    from ipm_emu import Emu
    from seg_ipm_study import seg_riccati
    o, rec = oracle_closed_loop(a.model, a.N, a.B, 2)
    qs = [o.build_qp(r[3], r[4], r[0], r[1], r[2]) for r in rec]
    Q = {k: np.stack([q[k] for q in qs]) for k in qs[0]}
    Q["idxbx"] = np.array([o.prm.idxbx[j] for j in range(o.nbx)])
    single = lambda mu, al, it: np.clip((1 - al) ** 2, 0.01, 0.5)  # noqa: E731

    def run(ric=None):
        e = Emu(Q)
        if ric is not None:
            e.riccati = lambda sig, gh, e=e: ric(e, sig, gh)
        r = e.solve(single=single)
        return r["iters"], r["z"][:, 0, :e.nu]
    it_s, u_s = run()
    print("serial      iters", it_s.tolist())
    for S in a.S:
        if a.N % S:
            continue
        for m in a.masters:
            it, u = run(lambda e, sig, gh, S=S, m=m: seg_riccati(e, sig, gh, S, os.environ.get("SENS64") is None, m))
            print(f"S={S} {m:7s} iters", it.tolist(), f"u0 max diff {np.nanmax(np.abs(u - u_s)):.2e}")


if __name__ == "__main__":
    main()
