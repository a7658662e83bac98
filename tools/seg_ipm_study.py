#!/usr/bin/env python3
"""The segmented Riccati inside the device IPM, on real bench QPs (design check for k_sqp_rti_rowpar SEG).

tools/seg_emu.py checks one Newton direction on synthetic QPs; this runs the whole single-direction IPM of the
device (tools/ipm_emu.py, warm rule as dumped by tools/tick_dump.py) on the QPs of dumped stationary metric ticks
twice: with the serial Riccati and with the segmented one in the kernel's precision (the factor in fp64, the lam
sensitivities Phi / Z / Gam / t rounded to fp32 at every stage, the master in fp64). Reports the iteration counts of
both and the largest u0 difference at exit (the parity tolerance is 1e-3).
usage: python tools/seg_ipm_study.py gpurun_out/tick_dump_metric.npz [--S 4] [--ticks 2] [--n 1024]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def f32(a, on):
    return a.astype(np.float32).astype(np.float64) if on else a


def psd_chol_b(A, drop=True, thr=0.0, rel=0.0):
    """Batched row-distributed right-looking Cholesky of the device (team_common.hpp rowchol): pivots <= thr (or
    <= rel x the column's original diagonal entry) drop their column (drop) or give NaN."""
    L = A.copy()
    n = A.shape[-1]
    d0 = np.diagonal(A, axis1=1, axis2=2).copy()
    for j in range(n):
        p = L[:, j, j].copy()
        ok = (p > thr) & (p > rel * d0[:, j])
        rd = np.where(ok, 1.0 / np.sqrt(np.where(ok, p, 1.0)), 0.0 if drop else np.nan)
        L[:, j:, j] *= rd[:, None]
        L[:, :j, j] = 0.0
        for jp in range(j + 1, n):
            L[:, jp:, jp] -= L[:, jp:, j] * L[:, jp, j][:, None]
    return np.tril(L)


def seg_riccati(emu, sig, ghat, S, sens32=True, master="gj"):
    """Batched segmented solve of emu's Newton system (segments [qL, (q+1)L), the last one through N).
    master: "gj" (Q = Phat X^-1 by a pivoted solve), "chol" (the device: Q = (L R^-T)(L R^-T)', L L' = Phat,
    R R' = I + L' C C' L, C C' = -Gam with dropped non-positive pivots; forward with Gam), "cholcc" (the same with
    C C' in place of Gam everywhere), "cholg" (Q = (L R^-T)(L R^-T)', R R' = I - L' Gam L: no factor of Gam, whose
    semidefinite Cholesky blows up on nearly singular fp32 sums)."""
    Q, N, nx, nu = emu.Q, emu.N, emu.nx, emu.nu
    Bn = emu.B
    D = emu.H + sig
    L = N // S
    assert L * S == N
    idx = np.arange(nx)
    segs = []
    fac = {}
    for q in range(S):
        last = q == S - 1
        P = np.zeros((Bn, nx, nx))
        p = np.zeros((Bn, nx))
        Phi = np.zeros((Bn, nx, nx))
        if last:
            P[:, idx, idx] = D[:, N, nu:]
            p[:] = ghat[:, N, nu:]
        else:
            Phi[:, idx, idx] = 1.0
        Gam = np.zeros((Bn, nx, nx))
        t = np.zeros((Bn, nx))
        for k in range((q + 1) * L - 1, q * L - 1, -1):
            G = np.concatenate([Q["B"][:, k], Q["A"][:, k]], axis=2)  # [B][nx][nv]
            M = np.einsum("bli,blm,bmj->bij", G, P, G)
            M[:, np.arange(nu + nx), np.arange(nu + nx)] += D[:, k]
            w = ghat[:, k] + np.einsum("bli,bl->bi", G, p)
            Y = f32(np.einsum("bli,blc->bic", G, Phi), sens32)
            Lc = np.linalg.cholesky(M[:, :nu, :nu])
            LM = np.linalg.solve(Lc, M[:, :nu, nu:]).transpose(0, 2, 1)  # [B][nx][nu]
            lr = np.linalg.solve(Lc, w[:, :nu, None])[..., 0]
            Z = f32(np.linalg.solve(Lc, Y[:, :nu]), sens32)                # [B][nu][nx]
            P = M[:, nu:, nu:] - LM @ LM.transpose(0, 2, 1)
            P = 0.5 * (P + P.transpose(0, 2, 1))
            p = w[:, nu:] - np.einsum("bij,bj->bi", LM, lr)
            Phi = f32(Y[:, nu:] - LM @ Z, sens32)
            g64 = os.environ.get("GAM64") == "1" or (os.environ.get("GAM64") == "0only" and q == 0)
            Gam = f32(Gam - Z.transpose(0, 2, 1) @ Z, sens32 and not g64)
            t = f32(t - np.einsum("bji,bj->bi", Z, lr), sens32)
            fac[k] = (Lc, LM, lr, Z)
        segs.append(dict(P=P, p=p, Phi=Phi, Gam=Gam, t=t))
    # master (fp64)
    if master.startswith("bidir"):
        s, lam = master_bidir(segs, S, nx, Bn, master)
    elif master == "scan":
        s, lam = master_scan(segs, S, nx, Bn)
    else:
        s, lam = master_serial(segs, S, nx, Bn, master)
    return seg_forward(emu, fac, s, lam, S, L)


def qform_b(A, C):
    """The device master's Q = A (I + C A)^-1 = Y Y', Y = L R^-T, L L' = A (pivots below 1e-13 of their diagonal entry
    dropped), R R' = I + L' C L (sqp_rti_rowpar.hip SEG master, qform)."""
    eye = np.broadcast_to(np.eye(A.shape[-1]), A.shape)
    Lp = psd_chol_b(A, rel=1e-13)
    R = psd_chol_b(eye + Lp.transpose(0, 2, 1) @ C @ Lp, drop=False, thr=0.5)
    Y = np.linalg.solve(R, Lp.transpose(0, 2, 1)).transpose(0, 2, 1)
    return Y @ Y.transpose(0, 2, 1)


def master_bidir(segs, S, nx, Bn, variant="bidir"):
    """The round-5 device master: the backward sweep from S - 1 down to m = S / 2 and the dual sweep
    s_i = -Shat_i lam_i + shat_i from 1 up to m, joined at m, then propagated outwards."""
    mv = lambda A, x: np.einsum("bij,bj->bi", A, x)  # noqa: E731
    tr = lambda A: A.transpose(0, 2, 1)  # noqa: E731
    m = S // 2
    Ph, ph = segs[S - 1]["P"], segs[S - 1]["p"]
    Qs, cs, phs = {}, {}, {}
    for i in range(S - 2, m - 1, -1):
        sg = segs[i]
        Qm = qform_b(Ph, -sg["Gam"])
        c = sg["t"] + mv(sg["Gam"], ph)
        Qs[i], cs[i], phs[i] = Qm, c, ph
        Ph = sg["P"] + sg["Phi"] @ Qm @ tr(sg["Phi"])
        ph = sg["p"] + mv(sg["Phi"], mv(Qm, c) + ph)
    Sh, sh = -segs[0]["Gam"], segs[0]["t"]
    Qd, us = {}, {}
    for i in range(1, m):
        sg = segs[i]
        if variant == "bidir_gj":
            Qm = np.linalg.solve(np.eye(nx) + sg["P"] @ Sh, Sh.transpose(0, 2, 1)).transpose(0, 2, 1)
        else:
            Qm = qform_b(Sh, sg["P"])
        u = sh - mv(Qm, sg["p"] + mv(sg["P"], sh))
        Qd[i], us[i] = Qm, u
        Sh = -sg["Gam"] + tr(sg["Phi"]) @ Qm @ sg["Phi"]
        sh = sg["t"] + mv(tr(sg["Phi"]), u)
    Qj = np.linalg.solve(np.eye(nx) + Sh @ Ph, Ph.transpose(0, 2, 1)).transpose(0, 2, 1) if variant == "bidir_gj" \
        else qform_b(Ph, Sh)
    s = [None] * S
    lam = [None] * (S + 1)
    s[0], lam[S] = np.zeros((Bn, nx)), np.zeros((Bn, nx))
    lam[m] = ph + mv(Qj, sh - mv(Sh, ph))
    s[m] = sh - mv(Sh, lam[m])
    for i in range(m, S - 1):
        sg = segs[i]
        fs = mv(tr(sg["Phi"]), s[i])
        lam[i + 1] = mv(Qs[i], fs + cs[i]) + phs[i]
        s[i + 1] = fs + mv(sg["Gam"], lam[i + 1]) + sg["t"]
    for i in range(m - 1, 0, -1):
        sg = segs[i]
        fl = mv(sg["Phi"], lam[i + 1])
        s[i] = us[i] - mv(Qd[i], fl)
        lam[i] = mv(sg["P"], s[i]) + sg["p"] + fl
    return s, lam


def master_scan(segs, S, nx, Bn):
    """Tree (parallel-scan) form of the master: adjacent segments combine pairwise, level by level, into one element
    (P, p, Phi, C = -Gam, t) of the same two-point form; the boundary values then expand back down the tree. Each
    combine takes Qb = P_b (I + C_a P_b)^-1 and Qa = C_a (I + P_b C_a)^-1 (both qform_b, independent), so a level
    costs one master step whatever its width: depth log2 S against the bidirectional master's S / 2."""
    mv = lambda A, x: np.einsum("bij,bj->bi", A, x)  # noqa: E731
    tr = lambda A: A.transpose(0, 2, 1)  # noqa: E731
    eye = np.broadcast_to(np.eye(nx), (Bn, nx, nx))
    level = [dict(P=g["P"], p=g["p"], Phi=g["Phi"], C=-g["Gam"], t=g["t"], lo=i, hi=i + 1) for i, g in enumerate(segs)]
    levels = [level]
    while len(level) > 1:
        nxt = []
        for k in range(0, len(level) - 1, 2):
            a, b = level[k], level[k + 1]
            Qb = qform_b(b["P"], a["C"])
            Qa = qform_b(a["C"], b["P"])
            E = eye - b["P"] @ Qa  # (I + P_b C_a)^-1
            v = a["t"] - mv(a["C"], b["p"])
            nxt.append(dict(P=a["P"] + a["Phi"] @ Qb @ tr(a["Phi"]), p=a["p"] + mv(a["Phi"], mv(Qb, v) + b["p"]),
                            Phi=a["Phi"] @ E @ b["Phi"], C=b["C"] + tr(b["Phi"]) @ Qa @ b["Phi"],
                            t=b["t"] + mv(tr(b["Phi"]) @ tr(E), v), lo=a["lo"], hi=b["hi"], a=a, b=b, Qa=Qa, E=E))
        if len(level) % 2:
            nxt.append(level[-1])
        levels.append(nxt)
        level = nxt
    s = [None] * S
    lam = [None] * (S + 1)
    s[0], lam[S] = np.zeros((Bn, nx)), np.zeros((Bn, nx))

    def expand(nd):
        if "a" not in nd:
            return
        a, b = nd["a"], nd["b"]
        si, lo = s[a["lo"]], lam[b["hi"]]
        v = a["t"] - mv(a["C"], b["p"])
        sm = mv(tr(nd["E"]), mv(tr(a["Phi"]), si) + v) - mv(nd["Qa"], mv(b["Phi"], lo))
        s[b["lo"]] = sm
        lam[b["lo"]] = mv(b["P"], sm) + b["p"] + mv(b["Phi"], lo)
        expand(a)
        expand(b)
    expand(levels[-1][0])
    return s, lam


def master_serial(segs, S, nx, Bn, master):
    Ph, ph = segs[S - 1]["P"], segs[S - 1]["p"]
    Qs, cs, phs = [None] * S, [None] * S, [None] * S
    eye = np.broadcast_to(np.eye(nx), (Bn, nx, nx))
    for i in range(S - 2, -1, -1):
        sg = segs[i]
        if master == "gj":
            X = eye - sg["Gam"] @ Ph
            Qm = np.linalg.solve(X.transpose(0, 2, 1), Ph)  # X^-T Phat (= Phat X^-1, symmetric)
        elif master == "cholg":
            Lp = psd_chol_b(Ph, rel=1e-13)
            K = eye + Lp.transpose(0, 2, 1) @ (-sg["Gam"]) @ Lp
            R = psd_chol_b(K, drop=False, thr=0.5)
            Y = np.linalg.solve(R, Lp.transpose(0, 2, 1)).transpose(0, 2, 1)
            Qm = Y @ Y.transpose(0, 2, 1)
        else:
            C = psd_chol_b(-sg["Gam"])
            if master == "cholcc":
                sg["Gam"] = -(C @ C.transpose(0, 2, 1))
            Lp = psd_chol_b(Ph)
            V = Lp.transpose(0, 2, 1) @ C
            R = psd_chol_b(eye + V @ V.transpose(0, 2, 1), drop=False, thr=0.5)
            Y = np.linalg.solve(R, Lp.transpose(0, 2, 1)).transpose(0, 2, 1)
            Qm = Y @ Y.transpose(0, 2, 1)
        c = sg["t"] + np.einsum("bij,bj->bi", sg["Gam"], ph)
        Qs[i], cs[i], phs[i] = Qm, c, ph
        if i >= 1:
            Ph = sg["P"] + sg["Phi"] @ Qm @ sg["Phi"].transpose(0, 2, 1)
            ph = sg["p"] + np.einsum("bij,bj->bi", sg["Phi"], np.einsum("bij,bj->bi", Qm, c) + ph)
    s = [np.zeros((Bn, nx))]
    lam = [None] * (S + 1)
    lam[S] = np.zeros((Bn, nx))
    for i in range(S - 1):
        sg = segs[i]
        v = np.einsum("bli,bl->bi", sg["Phi"], s[i]) + cs[i]
        lam[i + 1] = np.einsum("bij,bj->bi", Qs[i], v) + phs[i]
        s.append(np.einsum("bli,bl->bi", sg["Phi"], s[i]) + np.einsum("bij,bj->bi", sg["Gam"], lam[i + 1]) + sg["t"])
    return s, lam


def seg_forward(emu, fac, s, lam, S, L):
    Q, N, nx, nu, Bn = emu.Q, emu.N, emu.nx, emu.nu, emu.B
    dz = np.zeros((Bn, N + 1, nu + nx))
    for q in range(S):
        x = f32(s[q], True)  # the kernel hands s_q and lam_{q+1} to the segments in fp32
        lm = f32(lam[q + 1], True)
        dz[:, q * L, nu:] = x if q > 0 else dz[:, 0, nu:]
        for k in range(q * L, (q + 1) * L):
            Lc, LM, lr, Z = fac[k]
            lrt = lr + np.einsum("bjc,bc->bj", Z, lm)
            u = -np.linalg.solve(Lc.transpose(0, 2, 1), (lrt + np.einsum("bij,bi->bj", LM, x))[..., None])[..., 0]
            dz[:, k, :nu] = u
            x = np.einsum("bij,bj->bi", Q["A"][:, k], x) + np.einsum("bij,bj->bi", Q["B"][:, k], u)
            dz[:, k + 1, nu:] = x
    return dz, np.ones(Bn, bool)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--model", default="diff")
    ap.add_argument("--N", type=int, default=40)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--ticks", type=int, default=2)
    ap.add_argument("--S", type=int, nargs="+", default=[4])
    ap.add_argument("--kappa", type=float, default=0.2)
    ap.add_argument("--f64-sens", action="store_true")
    a = ap.parse_args()
    from ipm_emu import Emu
    from warm_study import build
    d = np.load(a.dump)
    single = lambda mu, al, it: np.clip((1 - al) ** 2, 0.01, 0.5)  # noqa: E731
    for t in range(a.ticks):
        Q, lam, warm, gpu = build(d, t, a.model, a.N, a.n)
        wst = (np.nan_to_num(lam[..., 0]), np.nan_to_num(lam[..., 1]), a.kappa, 1e3)

        def run(riccati=None):
            e_c, e_w = Emu(Q), Emu(Q)
            if riccati is not None:
                e_c.riccati = lambda sig, gh, e=e_c: riccati(e, sig, gh)
                e_w.riccati = lambda sig, gh, e=e_w: riccati(e, sig, gh)
            rc, rw = e_c.solve(single=single), e_w.solve(single=single, warm=wst)
            it = np.where(warm, rw["iters"], rc["iters"])
            u0 = np.where(warm[:, None], rw["z"][:, 0, :e_c.nu], rc["z"][:, 0, :e_c.nu])
            return it, u0
        it_s, u_s = run()
        print(f"tick {t}: serial   iters mean {it_s.mean():.2f} max {it_s.max()} (gpu mean {gpu.mean():.2f} max "
              f"{gpu.max()})")
        for S in a.S:
            it_g, u_g = run(lambda e, sig, gh, S=S: seg_riccati(e, sig, gh, S, not a.f64_sens))
            print(f"tick {t}: S={S:2d}     iters mean {it_g.mean():.2f} max {it_g.max()}; |diff iters| max "
                  f"{np.abs(it_g - it_s).max()}; u0 max-abs diff {np.abs(u_g - u_s).max():.2e}")


if __name__ == "__main__":
    main()
