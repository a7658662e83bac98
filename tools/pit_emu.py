#!/usr/bin/env python3
"""Design study (not a test oracle): a two-sided, parallel-in-time solve of the IPM's Newton system.

The device QP step (k_sqp_rti_team, tools/ipm_emu.py) is one backward Riccati sweep over the N+1 stages and
forward / backward solves through the same chain, so one robot's IPM iteration is a serial chain of 4 x (N+1)
stage steps. Here the horizon is cut at stage m:
  * stages m..N: the usual backward Riccati (cost-to-go V_m of x_m; x_m's own cost left out);
  * stages 0..m-1: the same Riccati step on the time-reversed dynamics x_j = A_j^-1 x_{j+1} - A_j^-1 B_j u_j,
    run from j = 0 up to m-1 with the stage pair (u_j, x_{j+1}) as one record and the fixed x_0 as a terminal
    penalty rho/2 |x_0|^2 (cost-to-arrive W_m of x_m, x_m's cost included);
  * x_m from (P_m + W_m) x_m = -(p_m + w_m), then both halves are rolled out from the middle (u_k = K_k x_k +
    k_k forward for k >= m, u_j = K~_j x_{j+1} + k~_j backward for j < m).
Both halves run the SAME per-stage arithmetic on different records, i.e. they can be two DPP rows of one
wave, which halves each sweep's chain. Also checked: the Newton rhs needs no costates -- on a dynamics-feasible
iterate the Lagrangian gradient and the objective gradient differ by G'pi terms that telescope to pi_0' dx_0
= 0 -- so the halves need no adjoint recursion across the cut.

usage: python tools/pit_emu.py [--B 256] [--ticks 21] [--rho 1e8]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from ipm_emu import Emu  # noqa: E402


def make_qps(model="diff", N=40, B=256, ticks=21, seed=20250825):
    """QPs of a closed-loop tick of the seeded bench fleet, built by the oracle (CPU only)."""
    from cpu_fleet_solver import OracleFleetSolver
    from nmpc_nav_control_amd.fleet import Fleet
    from oracle.oracle import Oracle
    f = Fleet(model, B, N, seed, "cpu", solver_factory=lambda m, n, b, device: OracleFleetSolver(m, n, b))
    for _ in range(ticks):
        f.tick()
    sn = f.snapshot()
    o = Oracle(model, N)
    qs = []
    for i in range(B):
        tl = int(sn["tlen"][i])
        x0, yref, We = o.prepare(sn["pose"][i], sn["vel"][i], 0.0 if sn["steer"] is None else sn["steer"][i],
                                 sn["traj"][i, :tl], sn["carried"][i])
        qs.append(o.build_qp(sn["xbar"][i], sn["ubar"][i], x0, yref, We))
    Q = {k: np.stack([q[k] for q in qs]) for k in qs[0]}
    Q["idxbx"] = np.array([o.prm.idxbx[i] for i in range(o.nbx)])
    return Q


def riccati_step(P, p, G, Dv, gv, nu):
    """One Riccati step: stage variables v = [u; x] with diagonal weights Dv, gradient gv, next-state map
    x_next = G v, cost-to-go (P, p) on x_next. Returns (P_x, p_x, K, k) with u = K x + k."""
    PG = P @ G
    M = np.einsum("bli,blj->bij", G, PG)
    idx = np.arange(M.shape[1])
    M[:, idx, idx] += Dv
    q = gv + np.einsum("bli,bl->bi", G, p)
    Muu, Mux, Mxx = M[:, :nu, :nu], M[:, :nu, nu:], M[:, nu:, nu:]
    Mi = np.linalg.inv(Muu)
    K = -Mi @ Mux
    k = -np.einsum("bij,bj->bi", Mi, q[:, :nu])
    Px = Mxx + np.einsum("bji,bjk->bik", Mux, K)
    Px = 0.5 * (Px + Px.transpose(0, 2, 1))
    px = q[:, nu:] + np.einsum("bji,bj->bi", Mux, k)
    return Px, px, K, k


class PitEmu(Emu):
    """Emu whose Newton systems are solved two-sided (split at m) and whose rhs can drop the costates."""

    def __init__(self, Q, m=None, rho=1e8, objective_rhs=True, **kw):
        super().__init__(Q, **kw)
        self.m = (self.N + 1) // 2 if m is None else m
        self.rho = rho
        self.objective_rhs = objective_rhs
        A, Bm = Q["A"], Q["B"]
        Ai = np.linalg.inv(A)
        self.Grev = np.concatenate([-Ai @ Bm, Ai], axis=3)  # [B~ A~] per stage
        self.Gfwd = np.concatenate([Bm, A], axis=3)

    def adjoint(self, z, lam):
        if not self.objective_rhs:
            return super().adjoint(z, lam)
        # objective gradient only (no costates); the u-stationarity for the stopping test still uses the true
        # adjoint residual, computed separately (the device would track it)
        pi, rr = super().adjoint(z, lam)
        r = self.H * z + self.g - lam
        r[:, 0, self.nu:] = 0.0  # x_0 is not a variable
        self._rr = rr
        return pi, r

    def riccati(self, sig, ghat):
        B, N, nx, nu, m = self.B, self.N, self.nx, self.nu, self.m
        D = self.H + sig
        # second half: stages m..N, x_m's own cost left out
        P = np.zeros((B, nx, nx))
        P[:, np.arange(nx), np.arange(nx)] = D[:, N, nu:]
        p = ghat[:, N, nu:].copy()
        K, kf = {}, {}
        for k in range(N - 1, m - 1, -1):
            Dv, gv = D[:, k].copy(), ghat[:, k].copy()
            if k == m:
                Dv[:, nu:] = 0.0
                gv[:, nu:] = 0.0
            P, p, K[k], kf[k] = riccati_step(P, p, self.Gfwd[:, k], Dv, gv, nu)
        # first half, time-reversed: record j = (u_j, x_{j+1}), next state x_j, terminal rho/2 |x_0|^2
        W = np.zeros((B, nx, nx))
        W[:, np.arange(nx), np.arange(nx)] = self.rho
        w = np.zeros((B, nx))
        Kr, kr = {}, {}
        for j in range(m):
            Dv = np.concatenate([D[:, j, :nu], D[:, j + 1, nu:]], axis=1)
            gv = np.concatenate([ghat[:, j, :nu], ghat[:, j + 1, nu:]], axis=1)
            W, w, Kr[j], kr[j] = riccati_step(W, w, self.Grev[:, j], Dv, gv, nu)
        xm = -np.linalg.solve(P + W, (p + w)[:, :, None])[:, :, 0]
        dz = np.zeros((B, N + 1, self.nv))
        dz[:, m, nu:] = xm
        for k in range(m, N):
            dz[:, k, :nu] = np.einsum("bij,bj->bi", K[k], dz[:, k, nu:]) + kf[k]
            dz[:, k + 1, nu:] = np.einsum("bij,bj->bi", self.Gfwd[:, k], dz[:, k])
        x0 = None
        for j in range(m - 1, -1, -1):
            dz[:, j, :nu] = np.einsum("bij,bj->bi", Kr[j], dz[:, j + 1, nu:]) + kr[j]
            v = np.concatenate([dz[:, j, :nu], dz[:, j + 1, nu:]], axis=1)
            xj = np.einsum("bij,bj->bi", self.Grev[:, j], v)
            if j > 0:
                dz[:, j, nu:] = xj
            else:
                x0 = xj
        self.last_x0 = x0
        return dz, np.ones(B, bool)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--ticks", type=int, default=21)
    ap.add_argument("--rho", type=float, default=1e8)
    ap.add_argument("--model", default="diff")
    ap.add_argument("--N", type=int, default=40)
    args = ap.parse_args()
    Q = make_qps(args.model, args.N, args.B, args.ticks)
    base = Emu(Q).solve()
    # 1) one Newton system, both solvers, same rhs
    e0 = Emu(Q)
    z, tl, tu, ll, lu = e0.init()
    sig = np.where(e0.bnd, ll / tl + lu / tu, 0.0)
    _, rz = e0.adjoint(z, ll - lu)
    dz_ref, _ = e0.riccati(sig, rz)
    pe = PitEmu(Q, rho=args.rho, objective_rhs=False)
    dz_pit, _ = pe.riccati(sig, rz)
    print(f"one Newton system: max |dz_pit - dz_ref| {np.abs(dz_pit - dz_ref).max():.2e}, |x0| {np.abs(pe.last_x0).max():.2e}")
    r = e0.H * z + e0.g - (ll - lu)
    r[:, 0, e0.nu:] = 0.0
    dz_obj, _ = e0.riccati(sig, r)
    print(f"objective-gradient rhs (no costates): max |dz - dz_ref| {np.abs(dz_obj - dz_ref).max():.2e}")
    # 2) whole IPM
    for obj in (False, True):
        pit = PitEmu(Q, rho=args.rho, objective_rhs=obj).solve()
        du0 = np.abs(pit["z"][:, 0, :e0.nu] - base["z"][:, 0, :e0.nu]).max()
        dz = np.abs(pit["z"] - base["z"]).max()
        print(f"IPM two-sided (objective rhs {obj}): iters mean {pit['iters'].mean():.2f} max {pit['iters'].max()} "
              f"| standard mean {base['iters'].mean():.2f} max {base['iters'].max()} | same iters "
              f"{(pit['iters'] == base['iters']).mean():.3f} | du0 {du0:.2e} dz {dz:.2e}")


if __name__ == "__main__":
    main()
