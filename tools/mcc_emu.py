#!/usr/bin/env python3
"""Design study (diagnostic, not a test oracle): Gondzio multiple centrality correctors on top of the device's
Mehrotra IPM, on QPs of real bench ticks (tools/iter_stats.py --dump), with the batched fp64 emulator.

After the Mehrotra direction (dz, alpha), a robot whose step alpha is below `amin` tries up to `k` correctors:
trial step a~ = min(1, alpha + da); trial complementarity products v = (l + a~ dl)(t + a~ dt); products outside
[bmin sigma mu, bmax sigma mu] are projected into it and the difference is the corrector's complementarity
target; one more solve through the same factor (a C1 + F1 sweep pair on the device, ~0.35 of an iteration)
gives dz_c; the corrected direction dz + dz_c is kept when its step grows by at least gamma da.
Kernel time follows the chip's slowest robot, so the figure of merit is the cost (iterations + 0.35 x
correctors) of the tail: max and p99.9 over robots, and the wave (4-team) mean.
usage: python tools/mcc_emu.py gpurun_out/iter_dump.npz [--n 4096] [--tick 0]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from ipm_emu import Emu, load_qps  # noqa: E402

C_CORR = 0.35  # device cost of one extra corrector (C1 + F1 sweeps) in IPM iterations (DESIGN.md phase cycles)


class MccEmu(Emu):
    def __init__(self, Q, k=0, amin=0.5, da=0.2, bmin=0.1, bmax=10.0, gamma=0.1, **kw):
        super().__init__(Q, **kw)
        self.k, self.amin, self.da, self.bmin, self.bmax, self.gamma = k, amin, da, bmin, bmax, gamma

    def solve(self):
        B, bnd = self.B, self.bnd
        z, tl, tu, ll, lu = self.init()
        done = np.zeros(B, bool)
        iters = np.zeros(B, int)
        ncorr = np.zeros(B, int)
        zsol = np.zeros_like(z)
        mu_prev = np.full(B, 3e38)
        m2 = 2.0 * self.m
        for it in range(self.iter_max + 1):
            rl = np.where(bnd, z - self.lb - tl, 0.0)
            rr = np.where(bnd, self.ub - z - tu, 0.0)
            res_ineq = np.maximum(np.abs(rl), np.abs(rr)).max(axis=(1, 2))
            mu = (ll * tl + lu * tu).sum(axis=(1, 2)) / m2
            cmax = np.maximum(ll * tl, lu * tu).max(axis=(1, 2))
            pi, rz = self.adjoint(z, ll - lu)
            res_stat = np.abs(rz).max(axis=(1, 2))
            cmax_ok = cmax <= self.cmax_ratio * self.tol_comp
            stalled = (mu <= self.tol_comp) & (mu > 0.5 * mu_prev)
            stop = (res_ineq <= self.tol_ineq) & (((res_stat <= self.tol_stat) & (mu <= self.tol_comp) & cmax_ok) |
                                                  (mu <= 1e-2 * self.tol_comp) | (stalled & cmax_ok))
            stop |= it >= self.iter_max
            new = stop & ~done
            zsol[new] = z[new]
            iters[new] = it
            done |= stop
            mu_prev = mu
            if done.all():
                break
            itl, itu = 1.0 / tl, 1.0 / tu
            sig = np.where(bnd, ll * itl + lu * itu, 0.0)

            def rhs(tgl, tgu, base=True):
                gh = np.where(bnd, -(tgl - ll * rl) * itl + ll + (tgu - lu * rr) * itu - lu, 0.0)
                return (rz + gh) if base else gh

            def dirs(dz, tgl, tgu):
                return (dz + rl, -dz + rr, (tgl - ll * (tl + rl) - ll * dz) * itl, (tgu - lu * (tu + rr) + lu * dz) * itu)

            def amax(v, dv):
                with np.errstate(divide="ignore", invalid="ignore"):
                    a = np.where(bnd & (dv < 0), -v / dv, 1e30)
                return a.min(axis=(1, 2))

            def step(d):
                return np.minimum.reduce([amax(tl, d[0]), amax(tu, d[1]), amax(ll, d[2]), amax(lu, d[3])])
            zero = np.zeros_like(z)
            dza, _ = self.riccati(sig, rhs(zero, zero))
            da_ = dirs(dza, zero, zero)
            a_aff = np.minimum(1.0, step(da_))
            A_ = a_aff[:, None, None]
            mu_aff = (((ll + A_ * da_[2]) * (tl + A_ * da_[0]) + (lu + A_ * da_[3]) * (tu + A_ * da_[1])) *
                      bnd).sum(axis=(1, 2)) / m2
            sigma = np.minimum(np.clip(np.where(mu > 0, mu_aff / mu, 0.0), 0, None) ** 3, 1.0)
            smu = (sigma * mu)[:, None, None]
            tgl = smu - A_ * da_[2] * da_[0]
            tgu = smu - A_ * da_[3] * da_[1]
            dz, _ = self.riccati(sig, rhs(tgl, tgu))
            d = dirs(dz, tgl, tgu)
            alpha = np.minimum(1.0, self.tau * step(d))
            # Gondzio centrality correctors
            for _ in range(self.k):
                want = ~done & (alpha < self.amin)
                if not want.any():
                    break
                ncorr[want] += 1
                at = np.minimum(1.0, alpha + self.da)[:, None, None]
                vl = (ll + at * d[2]) * (tl + at * d[0])
                vu = (lu + at * d[3]) * (tu + at * d[1])
                lo, hi = self.bmin * smu, self.bmax * smu
                cl = np.where(bnd, np.clip(vl, lo, hi) - vl, 0.0)
                cu = np.where(bnd, np.clip(vu, lo, hi) - vu, 0.0)
                cl = np.maximum(cl, -hi)
                cu = np.maximum(cu, -hi)
                tgl2, tgu2 = tgl + cl, tgu + cu
                dz2, _ = self.riccati(sig, rhs(tgl2, tgu2))
                d2 = dirs(dz2, tgl2, tgu2)
                a2 = np.minimum(1.0, self.tau * step(d2))
                acc = want & (a2 >= alpha + self.gamma * self.da)
                am = acc[:, None, None]
                dz = np.where(am, dz2, dz)
                d = tuple(np.where(am, x2, x1) for x1, x2 in zip(d, d2))
                tgl, tgu = np.where(am, tgl2, tgl), np.where(am, tgu2, tgu)
                alpha = np.where(acc, a2, alpha)
            small = alpha < 0.1
            if small.any():
                smu2 = (np.maximum(sigma, 0.3) * mu)[:, None, None]
                dz2, _ = self.riccati(sig, rhs(smu2 + 0 * z, smu2 + 0 * z))
                d2 = dirs(dz2, smu2 + 0 * z, smu2 + 0 * z)
                a2 = np.minimum(1.0, self.tau * step(d2))
                sm = small[:, None, None]
                dz = np.where(sm, dz2, dz)
                d = tuple(np.where(sm, x2, x1) for x1, x2 in zip(d, d2))
                alpha = np.where(small, a2, alpha)
                ncorr[small & ~done] += 1
            a = np.where(done, 0.0, alpha)[:, None, None]
            z = z + a * dz
            tl, tu = tl + a * d[0] * bnd, tu + a * d[1] * bnd
            ll, lu = ll + a * d[2] * bnd, lu + a * d[3] * bnd
        return dict(iters=iters, ncorr=ncorr, z=zsol)


def report(name, r, base, nu):
    cost = r["iters"] + C_CORR * r["ncorr"]
    w = cost.reshape(-1, 4).max(axis=1)
    du0 = np.abs(r["z"][:, 0, :nu] - base["z"][:, 0, :nu]).max()
    print(f"{name:34s} iters mean {r['iters'].mean():5.2f} max {r['iters'].max():3d} | cost mean {cost.mean():5.2f} "
          f"p99.9 {np.percentile(cost, 99.9):5.2f} max {cost.max():5.2f} | wave mean {w.mean():5.2f} | du0 {du0:.1e}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--tick", type=int, default=0)
    ap.add_argument("--model", default="diff")
    ap.add_argument("--N", type=int, default=40)
    args = ap.parse_args()
    Q = load_qps(args.dump, args.tick, args.n, args.model, args.N)
    gi = Q["gpu_iter"]
    base = MccEmu(Q).solve()
    print(f"gpu iters mean {gi.mean():.2f} max {gi.max()} | emu corr {np.corrcoef(base['iters'], gi)[0, 1]:.3f}")
    nu = Q["B"].shape[3]
    report("baseline (Mehrotra + safeguard)", base, base, nu)
    for k, amin, da in [(1, 0.5, 0.2), (1, 0.9, 0.2), (2, 0.5, 0.2), (2, 0.9, 0.3), (1, 0.3, 0.3), (3, 0.9, 0.3)]:
        report(f"gondzio k={k} amin={amin} da={da}", MccEmu(Q, k=k, amin=amin, da=da).solve(), base, nu)


if __name__ == "__main__":
    main()
