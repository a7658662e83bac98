#!/usr/bin/env python3
"""Batched numpy emulator of the device QP (diagnostic; design studies of the IPM, not a test oracle).

Same algorithm as k_sqp_rti_team / oracle/nmpc_oracle.c oc_qp_ipm (dynamics-feasible Mehrotra IPM over the
delta-form OCP-QP, Riccati recursion, fp32-style stopping rule of the device) vectorised over robots in fp64,
plus the variants studied in DESIGN.md: `single=` is the device's default one-direction rule
(qp_ipm = NMPC_IPM_SINGLE: solve(single=lambda mu, a, it: np.clip((1 - a) ** 2, 0.01, 0.5))), `polish=` the
active-set polish. Input: the QPs of a dumped closed-loop tick
(tools/iter_stats.py --dump) built by the oracle's oc_build_qp.
usage: python tools/ipm_emu.py gpurun_out/iter_dump.npz [--tick 0] [--n 4096]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load_qps(path, tick, n, model="diff", N=40):
    from oracle.oracle import Oracle
    d = np.load(path)
    o = Oracle(model, N)
    nx, nu = o.nx, o.nu
    p = f"t{tick}_"
    B = min(n, d[p + "pose"].shape[1])
    qs = []
    for i in range(B):
        x0, yref, We = o.prepare(d[p + "pose"][:, i], d[p + "vel"][:, i], 0.0 if (p + "steer") not in d else
                                 d[p + "steer"][i], d[p + "traj"][:int(d[p + "tlen"][i]), :, i],
                                 d[p + "carried"][:, i])
        xb = d[p + "xbar"][:, i].reshape(N + 1, nx).astype(np.float64)
        ub = d[p + "ubar"][:, i].reshape(N, nu).astype(np.float64)
        qs.append(o.build_qp(xb, ub, x0, yref, We))
    Q = {k: np.stack([q[k] for q in qs]) for k in qs[0]}
    Q["idxbx"] = np.array([o.prm.idxbx[i] for i in range(o.nbx)])
    Q["gpu_iter"] = d[p + "qp_iter"][:B]
    return Q


class Emu:
    def __init__(self, Q, thr0=0.25, mu0=1.0, tau=0.995, tol_stat=1e-4, tol_ineq=1e-6, tol_comp=1e-10,
                 cmax_ratio=30.0, iter_max=50):
        self.Q = Q
        self.B, self.N, self.nx, _ = Q["A"].shape
        self.nu = Q["B"].shape[3]
        self.thr0, self.mu0, self.tau = thr0, mu0, tau
        self.tol_stat, self.tol_ineq, self.tol_comp, self.cmax_ratio = tol_stat, tol_ineq, tol_comp, cmax_ratio
        self.iter_max = iter_max
        B, N, nx, nu = self.B, self.N, self.nx, self.nu
        nv = nx + nu
        self.nv = nv
        # stage variables z[k] = [u_k; x_k] (u_N and x_0 fixed at 0 in delta form)
        H = np.zeros((B, N + 1, nv))
        g = np.zeros((B, N + 1, nv))
        H[:, :N, :nu] = Q["Hu"]
        g[:, :N, :nu] = Q["gu"]
        H[:, :, nu:] = Q["Hx"]
        g[:, :, nu:] = Q["gx"]
        lb = np.full((B, N + 1, nv), -1e30)
        ub = np.full((B, N + 1, nv), 1e30)
        lb[:, :N, :nu] = Q["lbu"]
        ub[:, :N, :nu] = Q["ubu"]
        for c, i in enumerate(Q["idxbx"]):
            lb[:, 1:, nu + i] = Q["lbx"][:, 1:, c]
            ub[:, 1:, nu + i] = Q["ubx"][:, 1:, c]
        bnd = lb > -1e29
        self.H, self.g, self.lb, self.ub, self.bnd = H, g, lb, ub, bnd
        self.m = bnd.sum(axis=(1, 2))
        self.fixed = np.zeros((N + 1, nv), bool)
        self.fixed[N, :nu] = True
        self.fixed[0, nu:] = True

    def dyn(self, dz):
        """dx_{k+1} = A dx_k + B du_k for the variable part (x0 fixed)."""
        Q, N, nu = self.Q, self.N, self.nu
        for k in range(N):
            dz[:, k + 1, nu:] = np.einsum("bij,bj->bi", Q["A"][:, k], dz[:, k, nu:]) + \
                np.einsum("bij,bj->bi", Q["B"][:, k], dz[:, k, :nu])
        return dz

    def init(self, start=None, warm=None):
        """warm: (ll_prev, lu_prev, kappa, cap) [B][N+1][nv] previous multipliers -> the device's warm start
        max(min(lambda_prev, cap), kappa / t); the first centring target then uses the measured mu."""
        B, N, nv, nu = self.B, self.N, self.nv, self.nu
        z = np.zeros((B, N + 1, nv))
        z[:, 0, nu:] = self.Q["dx0"]
        self.dyn(z)
        if start is not None:  # primal start from one Riccati solve of the QP with bound weights `start`
            pi, rz = self.adjoint(z, np.zeros_like(z))
            dz, _ = self.riccati(np.where(self.bnd, start, 0.0), rz)
            z = z + dz
        bnd = self.bnd
        tl = np.where(bnd, np.maximum(z - self.lb, self.thr0), 1e30)
        tu = np.where(bnd, np.maximum(self.ub - z, self.thr0), 1e30)
        ll = np.where(bnd, self.mu0 / tl, 0.0)
        lu = np.where(bnd, self.mu0 / tu, 0.0)
        if warm is not None:
            lp, up, kap, cap = warm
            ll = np.where(bnd, np.maximum(np.minimum(lp, cap), kap / tl), 0.0)
            lu = np.where(bnd, np.maximum(np.minimum(up, cap), kap / tu), 0.0)
        return z, tl, tu, ll, lu

    def adjoint(self, z, lam):
        """pi_k (k = 1..N) from the state stationarity; returns (pi, r) with r the full stationarity residual
        (0 on the state slots by construction)."""
        Q, N, nu = self.Q, self.N, self.nu
        pi = np.zeros((self.B, N + 2, self.nx))
        r = self.H * z + self.g - lam
        for k in range(N, 0, -1):
            s = r[:, k, nu:].copy()
            if k < N:
                s += np.einsum("bli,bl->bi", Q["A"][:, k], pi[:, k + 1])
            pi[:, k] = s
        rr = np.zeros_like(r)
        for k in range(N):
            rr[:, k, :nu] = r[:, k, :nu] + np.einsum("bli,bl->bi", Q["B"][:, k], pi[:, k + 1])
        return pi, rr

    def riccati(self, sig, ghat):
        """Solve the Newton system for the delta-form QP with diagonal weights H + sig and rhs ghat (stage-wise
        gradient of the model); returns dz (feasible: dx_0 = 0, dynamics)."""
        Q, N, nx, nu = self.Q, self.N, self.nx, self.nu
        D = self.H + sig
        P = np.zeros((self.B, nx, nx))
        p = np.zeros((self.B, nx))
        idx = np.arange(nx)
        P[:, idx, idx] = D[:, N, nu:]
        p[:] = ghat[:, N, nu:]
        K = np.zeros((self.B, N, nu, nx))
        kf = np.zeros((self.B, N, nu))
        ok = np.ones(self.B, bool)
        for k in range(N - 1, -1, -1):
            A, Bm = Q["A"][:, k], Q["B"][:, k]
            PA = P @ A
            PB = P @ Bm
            Quu = np.einsum("bli,blj->bij", Bm, PB)
            Quu[:, np.arange(nu), np.arange(nu)] += D[:, k, :nu]
            Qux = np.einsum("bli,blj->bij", Bm, PA)
            Qxx = np.einsum("bli,blj->bij", A, PA)
            Qxx[:, idx, idx] += D[:, k, nu:]
            qu = ghat[:, k, :nu] + np.einsum("bli,bl->bi", Bm, p)
            qx = ghat[:, k, nu:] + np.einsum("bli,bl->bi", A, p)
            ok &= np.all(np.linalg.eigvalsh(Quu) > 0, axis=1)
            Qi = np.linalg.inv(Quu)
            K[:, k] = -Qi @ Qux
            kf[:, k] = -np.einsum("bij,bj->bi", Qi, qu)
            P = Qxx + np.einsum("bji,bjk->bik", Qux, K[:, k])
            P = 0.5 * (P + P.transpose(0, 2, 1))
            p = qx + np.einsum("bji,bj->bi", Qux, kf[:, k])
        dz = np.zeros((self.B, N + 1, self.nv))
        for k in range(N):
            dz[:, k, :nu] = np.einsum("bij,bj->bi", K[:, k], dz[:, k, nu:]) + kf[:, k]
            dz[:, k + 1, nu:] = np.einsum("bij,bj->bi", Q["A"][:, k], dz[:, k, nu:]) + \
                np.einsum("bij,bj->bi", Q["B"][:, k], dz[:, k, :nu])
        return dz, ok

    def solve(self, polish=None, verbose=False, single=None, start=None, eta_scale=1.0, lag2=None, trace=None,
              warm=None, sd_hi=0.5):
        """Run the IPM on every robot. polish: None or dict(mu=threshold, rho=..., tol=...) -- after the
        residual test of an iteration whose mu is below the threshold, try the active-set polish; a robot whose
        polish passes its KKT test stops there. Returns per-robot iterations, polish attempts, solutions."""
        B, bnd = self.B, self.bnd
        z, tl, tu, ll, lu = self.init(start, warm)
        done = np.zeros(B, bool)
        iters = np.zeros(B, int)
        attempts = np.zeros(B, int)
        zsol = np.zeros_like(z)
        polished = np.zeros(B, bool)
        mu_prev = np.full(B, 3e38)
        alpha_prev = np.zeros(B)
        m2 = 2.0 * self.m
        for it in range(self.iter_max + 1):
            rl = np.where(bnd, z - self.lb - tl, 0.0)
            rr = np.where(bnd, self.ub - z - tu, 0.0)
            res_ineq = np.maximum(np.abs(rl), np.abs(rr)).max(axis=(1, 2))
            comp = ll * tl + lu * tu
            mu = comp.sum(axis=(1, 2)) / m2
            cmax = np.maximum(ll * tl, lu * tu).max(axis=(1, 2))
            pi, rz = self.adjoint(z, ll - lu)
            res_stat = np.abs(rz).max(axis=(1, 2))
            stat_ok = res_stat <= self.tol_stat
            cmax_ok = cmax <= self.cmax_ratio * self.tol_comp
            stalled = (mu <= self.tol_comp) & (mu > 0.5 * mu_prev)
            stop = (res_ineq <= self.tol_ineq) & ((stat_ok & (mu <= self.tol_comp) & cmax_ok) |
                                                  (mu <= 1e-2 * self.tol_comp) | (stalled & cmax_ok))
            stop |= it >= self.iter_max
            if trace is not None:  # per-iteration state of every robot (infeasibility / stagnation studies)
                lmax = np.where(self.bnd, np.maximum(ll, lu), 0.0).max(axis=(1, 2))
                trace.append(dict(it=it, res_ineq=res_ineq, res_stat=res_stat, mu=mu, lmax=lmax,
                                  alpha=alpha_prev.copy(), done=done.copy()))
            new = stop & ~done
            zsol[new] = z[new]
            iters[new] = it
            done |= stop
            mu_prev = mu
            if polish is not None:
                cand = ~done & (mu <= polish["mu"])
                if cand.any():
                    attempts[cand] += 1
                    zp, okp = self.polish(z, tl, tu, ll, lu, polish)
                    acc = cand & okp
                    zsol[acc] = zp[acc]
                    iters[acc] = it + polish.get("cost", 1.0)
                    polished |= acc
                    done |= acc
            if done.all():
                break
            # predictor
            itl, itu = 1.0 / tl, 1.0 / tu
            sig = np.where(bnd, ll * itl + lu * itu, 0.0)

            def rhs(tgl, tgu):
                gh = np.where(bnd, -(tgl - ll * rl) * itl + ll + (tgu - lu * rr) * itu - lu, 0.0)
                return rz + gh

            def dirs(dz, tgl, tgu):
                dtl = dz + rl
                dtu = -dz + rr
                dll = (tgl - ll * (tl + rl) - ll * dz) * itl
                dlu = (tgu - lu * (tu + rr) + lu * dz) * itu
                return dtl, dtu, dll, dlu

            def amax(v, dv):
                with np.errstate(divide="ignore", invalid="ignore"):
                    a = np.where(bnd & (dv < 0), -v / dv, 1e30)
                return a.min(axis=(1, 2))
            zero = np.zeros_like(z)
            if single is not None:  # one direction per iteration, centring sigma from a rule (no predictor)
                sg = single(mu, alpha_prev, it)
                smu = (sg * mu)[:, None, None] + 0 * z
                tgl_, tgu_ = smu, smu
                if lag2 is not None and it > 0:  # lagged second-order term from the previous direction
                    A_ = (lag2 * alpha_prev)[:, None, None]
                    tgl_ = smu - A_ * d_prev[2] * d_prev[0]
                    tgu_ = smu - A_ * d_prev[3] * d_prev[1]
                dz, _ = self.riccati(sig, rhs(tgl_, tgu_))
                d = dirs(dz, tgl_, tgu_)
                d_prev = d
                am = np.minimum.reduce([amax(tl, d[0]), amax(tu, d[1]), amax(ll, d[2]), amax(lu, d[3])])
                alpha = np.minimum(1.0, self.tau * am)
                alpha_prev = alpha
                a = np.where(done, 0.0, alpha)[:, None, None]
                z = z + a * dz
                tl, tu = tl + a * d[0] * bnd, tu + a * d[1] * bnd
                ll, lu = ll + a * d[2] * bnd, lu + a * d[3] * bnd
                continue
            dza, _ = self.riccati(sig, rhs(zero, zero))
            da = dirs(dza, zero, zero)
            am = np.minimum.reduce([amax(tl, da[0]), amax(tu, da[1]), amax(ll, da[2]), amax(lu, da[3])])
            a_aff = np.minimum(1.0, am)
            A_ = a_aff[:, None, None]
            mu_aff = (((ll + A_ * da[2]) * (tl + A_ * da[0]) + (lu + A_ * da[3]) * (tu + A_ * da[1])) *
                      bnd).sum(axis=(1, 2)) / m2
            s = np.clip(np.where(mu > 0, mu_aff / mu, 0.0), 0, None)
            sigma = np.minimum(s ** 3, 1.0)
            smu = (sigma * mu)[:, None, None]
            tgl = smu - eta_scale * A_ * da[2] * da[0]  # eta_scale 0: no second-order correction
            tgu = smu - eta_scale * A_ * da[3] * da[1]
            dz, _ = self.riccati(sig, rhs(tgl, tgu))
            d = dirs(dz, tgl, tgu)
            am = np.minimum.reduce([amax(tl, d[0]), amax(tu, d[1]), amax(ll, d[2]), amax(lu, d[3])])
            alpha = np.minimum(1.0, self.tau * am)
            small = alpha < 0.1
            if small.any():
                smu2 = (np.maximum(sigma, 0.3) * mu)[:, None, None]
                dz2, _ = self.riccati(sig, rhs(smu2 + 0 * z, smu2 + 0 * z))
                d2 = dirs(dz2, smu2 + 0 * z, smu2 + 0 * z)
                am2 = np.minimum.reduce([amax(tl, d2[0]), amax(tu, d2[1]), amax(ll, d2[2]), amax(lu, d2[3])])
                a2 = np.minimum(1.0, self.tau * am2)
                sm = small[:, None, None]
                dz = np.where(sm, dz2, dz)
                d = tuple(np.where(sm, x2, x1) for x1, x2 in zip(d, d2))
                alpha = np.where(small, a2, alpha)
            a = np.where(done, 0.0, alpha)[:, None, None]
            z = z + a * dz
            tl = tl + a * d[0] * bnd
            tu = tu + a * d[1] * bnd
            ll = ll + a * d[2] * bnd
            lu = lu + a * d[3] * bnd
            if verbose:
                print(it, float(np.median(mu)), float(mu.max()), int(done.sum()))
        return dict(iters=iters, attempts=attempts, z=zsol, polished=polished)

    def polish(self, z, tl, tu, ll, lu, opt):
        """Active-set polish: bounds with lambda > t (the IPM's own activity guess) are fixed at their value by
        a penalty rho, the rest dropped; one Riccati solve from z gives the equality-QP solution zp. Accept when
        every dropped bound holds (within tol) and every fixed bound's multiplier rho (b - zp) has the right sign
        (>= -tol)."""
        bnd = self.bnd
        rho = opt.get("rho", 1e10)
        tol = opt.get("tol", 1e-6)
        act_l = bnd & (ll > tl)
        act_u = bnd & (lu > tu)
        sig = np.where(act_l | act_u, rho, 0.0)
        target = np.where(act_l, self.lb, np.where(act_u, self.ub, 0.0))
        # rhs: stationarity of the equality QP without bound multipliers + penalty gradient
        pi, rz = self.adjoint(z, np.zeros_like(z))
        gh = rz + np.where(act_l | act_u, rho * (z - target), 0.0)
        dz, ok = self.riccati(sig, gh)
        zp = z + dz
        lam_l = np.where(act_l, rho * (self.lb - zp), 0.0)
        lam_u = np.where(act_u, rho * (zp - self.ub), 0.0)
        feas = np.where(bnd & ~act_l & ~act_u,
                        np.maximum(self.lb - zp, zp - self.ub), -1.0).max(axis=(1, 2)) <= tol
        sign = np.minimum(lam_l, lam_u).min(axis=(1, 2)) >= -opt.get("ltol", tol)
        return zp, ok & feas & sign


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--tick", type=int, default=0)
    ap.add_argument("--n", type=int, default=1024)
    args = ap.parse_args()
    Q = load_qps(args.dump, args.tick, args.n)
    e = Emu(Q)
    base = e.solve()
    gi = Q["gpu_iter"]
    print("baseline emu iters mean %.2f max %d | gpu mean %.2f max %d | corr %.3f" %
          (base["iters"].mean(), base["iters"].max(), gi.mean(), gi.max(), np.corrcoef(base["iters"], gi)[0, 1]))
    nu = e.nu
    for thr in (1e-2, 1e-3, 1e-4, 1e-5):
        r = e.solve(polish=dict(mu=thr, rho=1e10, tol=1e-7))
        du0 = np.abs(r["z"][:, 0, :nu] - base["z"][:, 0, :nu]).max()
        w = r["iters"].reshape(-1, 4).max(axis=1)
        print(f"polish mu<={thr:g}: iters mean {r['iters'].mean():.2f} max {r['iters'].max()} wave mean {w.mean():.2f}"
              f" | attempts mean {r['attempts'].mean():.2f} | polished {r['polished'].mean():.3f} | du0 {du0:.2e}")


if __name__ == "__main__":
    main()
