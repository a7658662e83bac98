"""Generate the golden fixtures of tests/golden/ from the fp64 CPU oracle.

The reference holds no golden vectors for this path (acados, CasADi and the
generated solver code are absent), so the fixtures are produced here from oracle/nmpc_oracle.c and pinned
independently by tests/test_oracle.py (numpy restatement of the model ODEs, finite-difference Jacobians,
KKT certificates of every QP solution and a dense active-set re-solve). Parity with acados itself is
unpinned.

Run:  python tests/golden/make_golden.py      (writes tests/golden/<model>_N<N>.npz)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from helpers import oracle_closed_loop  # noqa: E402

from oracle.oracle import Oracle  # noqa: E402

CASES = [("diff", 20, 24, 6), ("omni4", 20, 24, 6), ("tric", 20, 24, 6), ("diff", 40, 8, 4)]
SEED = 20250824


def make(model, N, B, ticks):
    o, rec = oracle_closed_loop(model, N, B, ticks, seed=SEED)
    out = {k: [] for k in ("x0", "yref", "We", "xbar", "ubar", "xbar_new", "ubar_new", "status", "qp_iter")}
    for r in rec:
        s, st, xb, ub = o.sqp_rti(r[3], r[4], r[0], r[1], r[2])
        for k, v in zip(("x0", "yref", "We", "xbar", "ubar"), r):
            out[k].append(v)
        out["xbar_new"].append(xb)
        out["ubar_new"].append(ub)
        out["status"].append(s)
        out["qp_iter"].append(st["qp_iter"])
    # RK4 + sensitivities at the first stage of each warm iterate
    rk = {k: [] for k in ("rk_x", "rk_u", "rk_xn", "rk_A", "rk_B")}
    for r in rec:
        x, u = r[3][0], r[4][0]
        xn, A, B = o.rk4(x, u)
        for k, v in zip(rk, (x, u, xn, A, B)):
            rk[k].append(v)
    arrs = {k: np.array(v) for k, v in {**out, **rk}.items()}
    arrs["meta"] = np.array([model, str(N), str(B), str(ticks), str(SEED)])
    return arrs


def main():
    for model, N, B, ticks in CASES:
        arrs = make(model, N, B, ticks)
        path = os.path.join(HERE, f"{model}_N{N}.npz")
        np.savez_compressed(path, **arrs)
        print(path, os.path.getsize(path), "bytes, qp_iter mean", arrs["qp_iter"].mean())


if __name__ == "__main__":
    main()
