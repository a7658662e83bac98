#!/usr/bin/env python3
"""Study: can the Riccati factorisation of the team kernel run in fp32?

The device factors M = H + Sigma + G^T P G and forms P_k = Qxx - Qxu Quu^-1 Qux in fp64 (DESIGN.md §5 "Why the
factor is fp64"). This emulator runs the device's single-direction IPM (tools/ipm_emu.py, warm rule of the dumped
ticks as tools/tail_study.py) with the factorisation in one of these precisions / forms:
  fp64    the device: factor and Schur complement in fp64, the rhs recursion in fp32;
  fp32    the same classic recursion entirely in fp32;
  wform   fp32 with the bounded integrator states moved into the inputs. The bounded states of every model are
          reference integrators x_b' = x_b + dt u_b (nmpc_models.hpp gmask rows 5/6, 7..10), so a huge barrier
          weight sigma on x_{k+1,b} enters stage k as sigma g g^T with g = (dt e_u_b, e_x_b): the Schur
          complement cancels sigma (Sigma - dt^2 Sigma^2 / (R + dt^2 Sigma)), which fp32 cannot hold. With the input
          coordinate w_b = g^T z = x_{k+1,b} in place of u_b (z = T z', exact), that weight is sigma e_w e_w^T in the
          INPUT block and the Schur complement has no cancellation. The choice is per robot, stage and bound: w-form
          when sigma_x(k+1, b) > sigma_u(k, b) (an active input bound in the w-form would cancel the same way);
  splitsig fp32 classic recursion in the original variables with each bounded state's barrier weight kept out of
          P and entered at its input's pivot, the one cancelling Schur update in closed form (_splitsig);
  sqrt    fp32 square-root Riccati: P = L L^T, the stage factor from a QR (numpy's Householder) of
          [diag(sqrt(D_k)); L_{k+1}^T G_k] (backward stable, columnwise).
Reports per variant: iteration counts (mean, per-tick max, wave-of-4 max mean), u0 and trajectory error against the
fp64 variant, and the number of robots whose solve hit the iteration cap.
usage: python tools/fp32_factor_study.py gpurun_out/tick_dump_metric.npz [--ticks 3] [--n 4096]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from ipm_emu import Emu  # noqa: E402

F32 = np.float32


def _sym(P):
    return 0.5 * (P + np.swapaxes(P, 1, 2))


class PrecEmu(Emu):
    def __init__(self, Q, variant, **kw):
        super().__init__(Q, **kw)
        self.variant = variant
        self.idxbx = np.asarray(Q["idxbx"])

    def riccati(self, sig, ghat):
        if self.variant == "fp64":
            return self._classic(sig, ghat, np.float64)
        if self.variant == "fp32":
            return self._classic(sig, ghat, F32)
        if self.variant == "wform":
            return self._wform(sig, ghat)
        if self.variant == "sqrt":
            return self._sqrt(sig, ghat)
        if self.variant == "splitsig":
            return self._splitsig(sig, ghat)
        raise ValueError(self.variant)

    # rhs recursion in fp32 for every variant (the device's), factor in `ft`
    def _classic(self, sig, ghat, ft):
        Q, N, nx, nu = self.Q, self.N, self.nx, self.nu
        D = (self.H + sig).astype(ft)
        gh = ghat.astype(F32)
        idx = np.arange(nx)
        P = np.zeros((self.B, nx, nx), ft)
        P[:, idx, idx] = D[:, N, nu:]
        p = gh[:, N, nu:].copy()
        K = np.zeros((self.B, N, nu, nx), F32)
        kf = np.zeros((self.B, N, nu), F32)
        for k in range(N - 1, -1, -1):
            A, Bm = Q["A"][:, k].astype(ft), Q["B"][:, k].astype(ft)
            PA, PB = P @ A, P @ Bm
            Quu = np.swapaxes(Bm, 1, 2) @ PB
            Quu[:, np.arange(nu), np.arange(nu)] += D[:, k, :nu]
            Qux = np.swapaxes(Bm, 1, 2) @ PA
            Qxx = np.swapaxes(A, 1, 2) @ PA
            Qxx[:, idx, idx] += D[:, k, nu:]
            Qi = np.linalg.inv(Quu)
            Kk = -(Qi @ Qux)
            P = _sym(Qxx + np.swapaxes(Qux, 1, 2) @ Kk)
            A32, B32 = A.astype(F32), Bm.astype(F32)
            qu = gh[:, k, :nu] + np.einsum("bli,bl->bi", B32, p)
            qx = gh[:, k, nu:] + np.einsum("bli,bl->bi", A32, p)
            kf[:, k] = -np.einsum("bij,bj->bi", Qi.astype(F32), qu)
            K[:, k] = Kk.astype(F32)
            p = qx + np.einsum("bji,bj->bi", Qux.astype(F32), kf[:, k])
        return self._forward(K, kf), np.ones(self.B, bool)

    def _forward(self, K, kf):
        Q, N, nu = self.Q, self.N, self.nu
        dz = np.zeros((self.B, N + 1, self.nv))
        for k in range(N):
            dz[:, k, :nu] = np.einsum("bij,bj->bi", K[:, k], dz[:, k, nu:]) + kf[:, k]
            dz[:, k + 1, nu:] = np.einsum("bij,bj->bi", Q["A"][:, k], dz[:, k, nu:]) + \
                np.einsum("bij,bj->bi", Q["B"][:, k], dz[:, k, :nu])
        return dz

    def _wform(self, sig, ghat):
        Q, N, nx, nu, nv, B = self.Q, self.N, self.nx, self.nu, self.nv, self.B
        D = (self.H + sig).astype(F32)
        Hx = self.H.astype(F32)
        gh = ghat.astype(F32)
        idx = np.arange(nx)
        ib = self.idxbx  # bounded state b is driven by input b (x_b' = x_b + dt u_b)
        nb = len(ib)
        # w-form at stage k for bound b: the state weight of x_{k+1, ib[b]} beats the input weight of u_{k, b}
        wm = sig[:, 1:, nu + ib] > sig[:, :N, :nb]  # [B][N][nb]
        # P_{k+1} excludes the barrier weight of a w-formed bound (it goes to the input block of stage k)
        P = np.zeros((B, nx, nx), F32)
        dN = D[:, N, nu:].copy()
        dN[:, ib] = np.where(wm[:, N - 1], Hx[:, N, nu + ib], dN[:, ib])
        P[:, idx, idx] = dN
        p = gh[:, N, nu:].copy()
        K = np.zeros((B, N, nu, nx), F32)
        kf = np.zeros((B, N, nu), F32)
        for k in range(N - 1, -1, -1):
            A, Bm = Q["A"][:, k].astype(F32), Q["B"][:, k].astype(F32)
            G = np.concatenate([Bm, A], axis=2)  # [B][nx][nv], z = (u, x)
            Dk = D[:, k].copy()
            if k > 0:  # stage-k states whose barrier weight went to stage k-1's inputs
                Dk[:, nu + ib] = np.where(wm[:, k - 1], Hx[:, k, nu + ib], Dk[:, nu + ib])
            M = np.swapaxes(G, 1, 2) @ (P @ G)
            M[:, np.arange(nv), np.arange(nv)] += Dk
            q = np.concatenate([gh[:, k, :nu], gh[:, k, nu:]], axis=1) + np.einsum("bli,bl->bi", G, p)
            # z = T z': u_b = (w_b - sum_{j != u_b} g_j z'_j) / g_{u_b} for the w-formed b
            T = np.broadcast_to(np.eye(nv, dtype=F32), (B, nv, nv)).copy()
            sw = np.zeros((B, nv), F32)  # barrier weights moved to w_b
            for b in range(nb):
                m = wm[:, k, b]
                g = G[:, ib[b], :]  # row of x_{k+1, ib[b]}
                gu = g[:, b]
                row = -g / gu[:, None]
                row[:, b] = 1.0 / gu
                T[:, b, :] = np.where(m[:, None], row, T[:, b, :])
                sw[:, b] = np.where(m, sig[:, k + 1, nu + ib[b]], 0.0)
            Mp = np.swapaxes(T, 1, 2) @ M @ T
            Mp[:, np.arange(nv), np.arange(nv)] += sw
            qp_ = np.einsum("bji,bj->bi", T, q)
            Quu, Qux, Qxx = Mp[:, :nu, :nu], Mp[:, :nu, nu:], Mp[:, nu:, nu:]
            Qi = np.linalg.inv(Quu)
            Kp = -(Qi @ Qux)
            kfp = -np.einsum("bij,bj->bi", Qi, qp_[:, :nu])
            P = _sym(Qxx + np.swapaxes(Qux, 1, 2) @ Kp)
            p = qp_[:, nu:] + np.einsum("bji,bj->bi", Qux, kfp)
            # back to u: u = T_uu u' + T_ux x with u' = Kp x + kfp
            Tuu, Tux = T[:, :nu, :nu], T[:, :nu, nu:]
            K[:, k] = Tuu @ Kp + Tux
            kf[:, k] = np.einsum("bij,bj->bi", Tuu, kfp)
        return self._forward(K, kf), np.ones(B, bool)

    def _splitsig(self, sig, ghat):
        """fp32 classic recursion in the original variables, with the barrier weight s_b of each bounded state kept
        out of P (P = P~ + sum_b s_b e_ib e_ib^T) and entered at the pivot of the input b that drives it (row ib of
        [B A] is h e_u_b + e_x_ib): the pivot gets h^2 s_b, entry (x_ib, u_b) h s_b, and the one Schur update that
        cancels s_b, the diagonal (x_ib, x_ib), is computed as
            [s (a - 2 h c + h^2 e) + (a e - c^2)] / (h^2 s + a)
        from the s-free a = M_bb, c = M_{x_ib, b}, e = M_{x_ib, x_ib} (exact algebra, no s - s). Everything in fp32,
        the right-looking row Cholesky of the input block as the device runs it."""
        Q, N, nx, nu, nv, B = self.Q, self.N, self.nx, self.nu, self.nv, self.B
        D = (self.H + sig).astype(F32)
        Hx = self.H.astype(F32)
        gh = ghat.astype(F32)
        idx = np.arange(nx)
        ib = self.idxbx
        nb = len(ib)
        sx = sig[:, :, nu + ib].astype(F32)  # [B][N+1][nb] the bounded states' barrier weights, kept out of P
        P = np.zeros((B, nx, nx), F32)
        dN = D[:, N, nu:].copy()
        dN[:, ib] = Hx[:, N, nu + ib]
        P[:, idx, idx] = dN
        p = gh[:, N, nu:].copy()
        K = np.zeros((B, N, nu, nx), F32)
        kf = np.zeros((B, N, nu), F32)
        for k in range(N - 1, -1, -1):
            A, Bm = Q["A"][:, k].astype(F32), Q["B"][:, k].astype(F32)
            G = np.concatenate([Bm, A], axis=2)
            Dk = D[:, k].copy()
            if k > 0:
                Dk[:, nu + ib] = Hx[:, k, nu + ib]
            M = np.swapaxes(G, 1, 2) @ (P @ G)
            M[:, np.arange(nv), np.arange(nv)] += Dk
            q = np.concatenate([gh[:, k, :nu], gh[:, k, nu:]], axis=1) + np.einsum("bli,bl->bi", G, p)
            # right-looking Cholesky of the input block, pivots in turn; L column j in Lc[:, :, j]
            Lc = np.zeros((B, nv, nu), F32)
            for j in range(nu):
                xj = nu + ib[j] if j < nb else None
                if xj is not None:
                    s_ = sx[:, k + 1, j]
                    h = G[:, ib[j], j]
                    a, c, e = M[:, j, j].copy(), M[:, xj, j].copy(), M[:, xj, xj].copy()
                    M[:, j, j] += h * h * s_
                    M[:, xj, j] += h * s_
                    M[:, j, xj] += h * s_
                piv = M[:, j, j]
                l = M[:, :, j] / np.sqrt(piv)[:, None]
                l[:, :j] = 0.0
                Lc[:, :, j] = l
                M = M - l[:, :, None] * l[:, None, :]
                if xj is not None:
                    M[:, xj, xj] = (s_ * (a - 2 * h * c + h * h * e) + (a * e - c * c)) / (h * h * s_ + a)
            Luu, Lxu = Lc[:, :nu, :], Lc[:, nu:, :]
            Li = np.linalg.inv(Luu)
            P = _sym(M[:, nu:, nu:])
            # u = -Luu^-T (Luu^-1 q_u + Lxu^T x)
            y = np.einsum("bij,bj->bi", Li, q[:, :nu])
            K[:, k] = -np.swapaxes(Li, 1, 2) @ np.swapaxes(Lxu, 1, 2)
            kf[:, k] = -np.einsum("bji,bj->bi", Li, y)
            p = q[:, nu:] - np.einsum("bij,bj->bi", Lxu, y)
        return self._forward(K, kf), np.ones(B, bool)

    def _sqrt(self, sig, ghat):
        Q, N, nx, nu, nv, B = self.Q, self.N, self.nx, self.nu, self.nv, self.B
        D = (self.H + sig).astype(F32)
        gh = ghat.astype(F32)
        idx = np.arange(nx)
        L = np.zeros((B, nx, nx), F32)  # P = L L^T
        L[:, idx, idx] = np.sqrt(D[:, N, nu:])
        p = gh[:, N, nu:].copy()
        K = np.zeros((B, N, nu, nx), F32)
        kf = np.zeros((B, N, nu), F32)
        for k in range(N - 1, -1, -1):
            A, Bm = Q["A"][:, k].astype(F32), Q["B"][:, k].astype(F32)
            G = np.concatenate([Bm, A], axis=2)
            S = np.zeros((B, nv + nx, nv), F32)
            S[:, np.arange(nv), np.arange(nv)] = np.sqrt(D[:, k])
            S[:, nv:] = np.swapaxes(L, 1, 2) @ G
            R = np.linalg.qr(S, mode="r")  # [B][nv][nv] upper, R^T R = M
            Ruu, Rux, Rxx = R[:, :nu, :nu], R[:, :nu, nu:], R[:, nu:, nu:]
            Ri = np.linalg.inv(Ruu)
            Kk = -(Ri @ Rux)
            L = np.swapaxes(Rxx, 1, 2)
            q = np.concatenate([gh[:, k, :nu], gh[:, k, nu:]], axis=1) + np.einsum("bli,bl->bi", G, p)
            # Quu^-1 qu = Ri Ri^T qu; p_k = qx + Qxu kf = qx - Rux^T Ri^T qu
            v = np.einsum("bji,bj->bi", Ri, q[:, :nu])  # Ri^T qu
            kf[:, k] = -np.einsum("bij,bj->bi", Ri, v)
            K[:, k] = Kk
            p = q[:, nu:] - np.einsum("bji,bj->bi", Rux, v)
        return self._forward(K, kf), np.ones(B, bool)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--model", default="diff")
    ap.add_argument("--N", type=int, default=40)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--ticks", type=int, default=3)
    ap.add_argument("--kappa", type=float, default=0.2)
    ap.add_argument("--variants", default="fp64,fp32,wform,splitsig,sqrt")
    a = ap.parse_args()
    from warm_study import build
    d = np.load(a.dump)
    single = lambda mu, al, it: np.clip((1 - al) ** 2, 0.01, 0.5)  # noqa: E731
    variants = a.variants.split(",")
    res = {v: dict(it=[], du0=[], dx=[], cap=0) for v in variants}
    gpu_all = []
    for t in range(a.ticks):
        Q, lam, warm, gpu = build(d, t, a.model, a.N, a.n)
        gpu_all.append(gpu)
        wst = (np.nan_to_num(lam[..., 0]), np.nan_to_num(lam[..., 1]), a.kappa, 1e3)
        ref = None
        for v in variants:
            cold = PrecEmu(Q, v).solve(single=single)
            wrm = PrecEmu(Q, v).solve(single=single, warm=wst)
            it = np.where(warm, wrm["iters"], cold["iters"])
            z = np.where(warm[:, None, None], wrm["z"], cold["z"])
            if ref is None:
                ref = z
            nu = Q["B"].shape[3]
            res[v]["it"].append(it)
            res[v]["du0"].append(np.abs(z[:, 0, :nu] - ref[:, 0, :nu]).max(axis=1))
            res[v]["dx"].append(np.abs(z[:, 1:, nu:] - ref[:, 1:, nu:]).max(axis=(1, 2)))
            res[v]["cap"] += int((it >= 50).sum())
            print(f"tick {t} {v:6s}: iters mean {it.mean():.2f} max {it.max()}  du0 max {res[v]['du0'][-1].max():.2e}"
                  f"  (gpu mean {gpu.mean():.2f} max {gpu.max()})", flush=True)
    print(f"\n{'variant':8s} {'mean':>6s} {'p99':>5s} {'max':>4s} {'wave-max':>8s} {'du0 max':>9s} {'du0 p99':>9s} "
          f"{'dx max':>9s} {'capped':>6s}")
    for v in variants:
        r = res[v]
        allv = np.concatenate(r["it"])
        wm = np.mean([x[: len(x) // 4 * 4].reshape(-1, 4).max(1).mean() for x in r["it"]])
        du0 = np.concatenate(r["du0"])
        dx = np.concatenate(r["dx"])
        print(f"{v:8s} {allv.mean():6.2f} {np.percentile(allv, 99):5.1f} {allv.max():4d} {wm:8.2f} {du0.max():9.2e} "
              f"{np.percentile(du0, 99):9.2e} {dx.max():9.2e} {r['cap']:6d}")


if __name__ == "__main__":
    main()
