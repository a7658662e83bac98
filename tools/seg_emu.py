"""Horizon-segmented Riccati solve of the IPM's Newton system -- numpy emulator (design check, CPU only).

The QP of one IPM direction (sqp_rti_team.hip / sqp_rti_rowpar.hip, absolute form): stages k = 0..N with
z_k = (u_k, x_k), diagonal Hessians H_k (stage weights + barrier weights Sigma), gradients g_k, dynamics
x_{k+1} = G_k z_k (G = [B A], the iterate is dynamics-feasible) and x_0 = 0 fixed. The serial Riccati recursion
over N+1 stages is the chain that sets one robot's latency. Split the horizon into S segments [a_i, a_{i+1}):

  * segment i < S-1 is solved for a FREE end costate lam (the multiplier of x_{a_{i+1}} = G z_{a_{i+1}-1}): its
    backward Riccati starts from P = 0, p = lam, and carries p = pbar + Phi lam, the value's lam terms
    1/2 lam' Gam lam + t' lam, and per stage Z = L^-1 (G' Phi)_u, the lam-sensitivity of the stored rhs LR;
  * segment S-1 is the usual terminal Riccati;
  * the master recursion over the S segment boundaries (state s_i = x_{a_i}, costate lam_i) is a two-point
    problem:  s_{i+1} = Phi_i' s_i + Gam_i lam_{i+1} + t_i,  lam_i = P_i s_i + pbar_i + Phi_i lam_{i+1};
    backward lam_i = Phat_i s_i + phat_i with X_i = I - Gam_i Phat_{i+1} (Gam <= 0, so X = I + PSD x PSD,
    eigenvalues >= 1), forward s_0 = 0, s_{i+1} = X_i^-1 (Phi_i' s_i + t_i + Gam_i phat_{i+1});
  * each segment then runs its forward recursion from s_i with LR = LRbar + Z lam_{i+1}.

The segments' backward and forward passes are independent (one DPP row each), so a robot's chain becomes
(N+1)/S stage steps + S master steps + (N+1)/S forward steps. This emulator checks that the segmented
direction equals the serial one, including barrier weights up to 1e12 and states the inputs cannot reach.

usage: python tools/seg_emu.py [--model diff] [--N 40] [--S 4] [--trials 50] [--sig-max 1e12] [--f32-sens]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_qp(o, N, rng, sig_max, pinned=False):
    """A delta-form QP like the kernel's: G_k from the oracle's RK4 sensitivities at random states, H_k = stage
    weights (dt-scaled) + barrier weights (log-uniform, a few at sig_max), random gradients."""
    nx, nu = o.nx, o.nu
    W = np.array([o.prm.W[i] for i in range(nx + nu)])
    dt = o.prm.dt
    G, H, g = [], [], []
    for k in range(N + 1):
        x = rng.uniform(-0.5, 0.5, nx)
        x[2] = rng.uniform(-np.pi, np.pi)
        u = rng.uniform(-0.5, 0.5, nu)
        _, A, B = o.rk4(x, u)
        G.append(np.concatenate([B, A], axis=1))
        wz = np.concatenate([W[nx:], W[:nx]]) * (dt if k < N else 1.0)  # (u, x) order
        if k == N:
            wz[:nu] = 0.0
        sig = np.zeros(nu + nx)
        bounded = list(range(nu)) + [nu + o.prm.idxbx[i] for i in range(o.nbx)]
        for v in bounded:
            if (v < nu and k == N) or (v >= nu and k == 0):
                continue
            sig[v] = 10 ** rng.uniform(-4, 2)
            if rng.uniform() < 0.1:
                sig[v] = sig_max * 10 ** rng.uniform(-2, 0)
        if pinned and N // 4 <= k <= 3 * N // 4:  # a velocity ref and an input held at their bounds for half the horizon
            sig[nu + o.prm.idxbx[0]] = sig_max
            sig[0] = sig_max
        h = wz + sig
        if k == 0:
            h[nu:] = 1.0  # x_0 is fixed (dx_0 = 0): any positive curvature
        H.append(h)
        g.append(rng.normal(0, 1, nu + nx) * (1.0 if k < N else 3.0))
    return G, H, g


def riccati_serial(G, H, g, nx, nu, N):
    """Reference: the plain backward Riccati / forward sweep on the whole horizon (fp64)."""
    P = np.diag(H[N][nu:])
    p = g[N][nu:].copy()
    Ks, ks = [None] * N, [None] * N
    for k in range(N - 1, -1, -1):
        M = np.diag(H[k]) + G[k].T @ P @ G[k]
        w = g[k] + G[k].T @ p
        Muu, Mux = M[:nu, :nu], M[:nu, nu:]
        Ks[k] = -np.linalg.solve(Muu, Mux)
        ks[k] = -np.linalg.solve(Muu, w[:nu])
        P = M[nu:, nu:] + Mux.T @ Ks[k]
        P = 0.5 * (P + P.T)
        p = w[nu:] + Mux.T @ ks[k]
    x = np.zeros(nx)
    us, xs = [], [x]
    for k in range(N):
        u = Ks[k] @ x + ks[k]
        x = G[k] @ np.concatenate([u, x])
        us.append(u)
        xs.append(x)
    return np.array(us), np.array(xs)


def seg_backward(G, H, g, nx, nu, N, a0, a1, sens_dtype=np.float64):
    """Backward pass of the segment [a0, a1): returns entry quantities and per-stage factors (L, LM, LRbar, Z)."""
    last = a1 == N + 1
    if last:
        P = np.diag(H[N][nu:])
        p = g[N][nu:].copy()
        Phi = np.zeros((nx, nx))
        kend = N - 1
    else:
        P = np.zeros((nx, nx))
        p = np.zeros(nx)
        Phi = np.eye(nx)
        kend = a1 - 1
    Gam = np.zeros((nx, nx))
    t = np.zeros(nx)
    st = {}
    for k in range(kend, a0 - 1, -1):
        M = np.diag(H[k]) + G[k].T @ P @ G[k]
        w = g[k] + G[k].T @ p
        Y = (G[k].T @ Phi).astype(sens_dtype)
        L = np.linalg.cholesky(M[:nu, :nu])
        LM = np.linalg.solve(L, M[:nu, nu:]).T  # (nx x nu): M_xu L^-T
        lr = np.linalg.solve(L, w[:nu])
        Z = np.linalg.solve(L.astype(sens_dtype), Y[:nu]).astype(sens_dtype)
        P = M[nu:, nu:] - LM @ LM.T
        P = 0.5 * (P + P.T)
        p = w[nu:] - LM @ lr
        Phi = (Y[nu:] - LM.astype(sens_dtype) @ Z).astype(sens_dtype)
        Gam = (Gam - (Z.T @ Z).astype(np.float64)).astype(sens_dtype).astype(np.float64)
        t = (t - Z.T.astype(np.float64) @ lr).astype(sens_dtype).astype(np.float64)
        st[k] = (L, LM, lr, Z.astype(np.float64))
    if last and a0 == N:  # a last segment holding only the terminal stage
        pass
    return dict(P=P, p=p, Phi=Phi.astype(np.float64), Gam=Gam, t=t, st=st, last=last)


def master(segs, nx):
    S = len(segs)
    Ph = [None] * S
    ph = [None] * S
    Ph[S - 1], ph[S - 1] = segs[S - 1]["P"], segs[S - 1]["p"]
    Xs, cs = [None] * S, [None] * S
    for i in range(S - 2, -1, -1):
        sg = segs[i]
        X = np.eye(nx) - sg["Gam"] @ Ph[i + 1]
        c = sg["t"] + sg["Gam"] @ ph[i + 1]
        Xs[i], cs[i] = X, c
        if i >= 1:
            Q = np.linalg.solve(X.T, Ph[i + 1]).T  # Phat X^-1 (Phat symmetric: X' Q' = Phat)
            Ph[i] = sg["P"] + sg["Phi"] @ Q @ sg["Phi"].T
            Ph[i] = 0.5 * (Ph[i] + Ph[i].T)
            ph[i] = sg["p"] + sg["Phi"] @ (Q @ c + ph[i + 1])
    s = [np.zeros(nx)]
    lam = [None] * (S + 1)
    lam[S] = np.zeros(nx)
    for i in range(S - 1):
        sn = np.linalg.solve(Xs[i], segs[i]["Phi"].T @ s[i] + cs[i])
        s.append(sn)
        lam[i + 1] = Ph[i + 1] @ sn + ph[i + 1]
    return s, lam, Xs


def psd_chol(A, thr, drop=True, rel=0.0):
    """Row-distributed right-looking Cholesky of the device (team_common.hpp rowchol): pivots <= thr or <= rel x the
    column's original diagonal entry drop their column (drop) or give NaN."""
    n = len(A)
    L = A.copy()
    d0 = np.diag(A).copy()
    for j in range(n):
        p = L[j, j]
        rd = 1.0 / np.sqrt(p) if (p > thr and p > rel * d0[j]) else (0.0 if drop and p == p else np.nan)
        L[j:, j] *= rd
        L[:j, j] = 0.0
        for jp in range(j + 1, n):
            L[jp:, jp] -= L[jp:, j] * L[jp, j]
    return np.tril(L)




def master_chol(segs, nx):
    """The device master (sqp_rti_rowpar.hip SEG): Q_i = Y Y', Y = L R^-T, L L' = Phat_{i+1} (relative pivot
    threshold 1e-13), R R' = I - L' Gam_i L; forward lam_{i+1} = Q_i (Phi' s_i + c_i) + phat_{i+1},
    s_{i+1} = Phi' s_i + Gam lam + t."""
    S = len(segs)
    Ph, ph = segs[S - 1]["P"], segs[S - 1]["p"]
    Qs, cs, phs = [None] * S, [None] * S, [None] * S
    for i in range(S - 2, -1, -1):
        sg = segs[i]
        Lp = psd_chol(Ph, 0.0, rel=1e-13)
        R = psd_chol(np.eye(nx) - Lp.T @ sg["Gam"] @ Lp, 0.5, drop=False)
        Y = np.linalg.solve(R, Lp.T).T
        Q = Y @ Y.T
        c = sg["t"] + sg["Gam"] @ ph
        Qs[i], cs[i], phs[i] = Q, c, ph
        if i >= 1:
            Ph = sg["P"] + sg["Phi"] @ (Q @ sg["Phi"].T)
            ph = sg["p"] + sg["Phi"] @ (ph + Q @ c)
    s = [np.zeros(nx)]
    lam = [None] * (S + 1)
    lam[S] = np.zeros(nx)
    for i in range(S - 1):
        fs = segs[i]["Phi"].T @ s[i]
        lam[i + 1] = Qs[i] @ (fs + cs[i]) + phs[i]
        s.append(fs + segs[i]["Gam"] @ lam[i + 1] + segs[i]["t"])
    return s, lam, [np.eye(nx)]


def kkt_res(G, H, g, nx, nu, N, us, xs):
    """Largest input-stationarity residual of (us, xs) with the exact adjoint, relative to its terms' size."""
    pi = H[N][nu:] * xs[N] + g[N][nu:]
    worst = 0.0
    for k in range(N - 1, -1, -1):
        B, A = G[k][:, :nu], G[k][:, nu:]
        t1, t2 = H[k][:nu] * us[k] + g[k][:nu], B.T @ pi
        worst = max(worst, np.abs(t1 + t2).max() / (np.abs(t1).max() + np.abs(t2).max() + 1e-300))
        pi = H[k][nu:] * xs[k] + g[k][nu:] + A.T @ pi
    return worst


def riccati_segmented(G, H, g, nx, nu, N, S, sens_dtype=np.float64, chol_master=False, master_fn=None):
    """master_fn(segs, nx) -> (s, lam): another master form (the default: `master`, or `master_chol`)."""
    bnd = np.linspace(0, N + 1, S + 1).round().astype(int)
    segs = [seg_backward(G, H, g, nx, nu, N, bnd[i], bnd[i + 1], sens_dtype) for i in range(S)]
    if master_fn is not None:
        s, lam = master_fn(segs, nx)
        Xs = [np.eye(nx)]
    else:
        s, lam, Xs = (master_chol if chol_master else master)(segs, nx)
    us, xs = np.zeros((N, nu)), np.zeros((N + 1, nx))
    gap = 0.0
    for i in range(S):
        x = s[i]
        xs[bnd[i]] = x
        for k in range(bnd[i], min(bnd[i + 1], N)):
            L, LM, lr, Z = segs[i]["st"][k]
            lr_t = lr + Z @ lam[i + 1]
            u = -np.linalg.solve(L.T, lr_t + LM.T @ x)
            x = G[k] @ np.concatenate([u, x])
            us[k] = u
            xs[k + 1] = x
        if i + 1 < S:
            gap = max(gap, np.abs(x - s[i + 1]).max())  # the segment's own end state against the master's
    cond = max(np.linalg.cond(X) for X in Xs if X is not None) if S > 1 else 1.0
    return us, xs, gap, cond


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="diff")
    ap.add_argument("--N", type=int, default=40)
    ap.add_argument("--S", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--trials", type=int, default=50)
    ap.add_argument("--sig-max", type=float, default=1e12)
    ap.add_argument("--f32-sens", action="store_true", help="Phi / Z / Gam / t in fp32 (P, the factor in fp64)")
    ap.add_argument("--chol-master", action="store_true", help="the device's master (factor of -Gam, no pivoting)")
    ap.add_argument("--pinned", action="store_true", help="a vel-ref state and an input at sig_max over stages N/4..3N/4")
    args = ap.parse_args()
    from oracle.oracle import Oracle
    o = Oracle(args.model, args.N)
    rng = np.random.default_rng(3)
    for S in args.S:
        du, dxm, gaps, conds, rs, rr = [], [], [], [], [], []
        for _ in range(args.trials):
            G, H, g = make_qp(o, args.N, rng, args.sig_max, args.pinned)
            u_ref, x_ref = riccati_serial(G, H, g, o.nx, o.nu, args.N)
            u, x, gap, cond = riccati_segmented(G, H, g, o.nx, o.nu, args.N, S,
                                                np.float32 if args.f32_sens else np.float64, args.chol_master)
            scale = max(1.0, np.abs(u_ref).max())
            du.append(np.abs(u - u_ref).max() / scale)
            dxm.append(np.abs(x - x_ref).max() / max(1.0, np.abs(x_ref).max()))
            gaps.append(gap)
            conds.append(cond)
            rs.append(kkt_res(G, H, g, o.nx, o.nu, args.N, u, x))
            rr.append(kkt_res(G, H, g, o.nx, o.nu, args.N, u_ref, x_ref))
        print(f"{args.model} N={args.N} S={S} sig_max={args.sig_max:g} sens={'fp32' if args.f32_sens else 'fp64'}: "
              f"du rel max {max(du):.2e} median {np.median(du):.2e}; dx rel max {max(dxm):.2e}; "
              f"boundary gap max {max(gaps):.2e}; cond(X) max {max(conds):.2e}; "
              f"rel KKT residual max: segmented {max(rs):.1e}, serial {max(rr):.1e}")


if __name__ == "__main__":
    main()
