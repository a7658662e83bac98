"""Independent dense restatement of one SQP-RTI QP (test infrastructure).

Condenses the delta-form OCP-QP (oracle.build_qp: A, B, b, Hx, Hu, gx, gu, bounds, dx0) into a dense QP
in the inputs only (states eliminated through the dynamics, x0 fixed):
    min 1/2 u'Hu + g'u   s.t.  C u <= d
and solves it with a textbook dense primal-dual Mehrotra interior-point method (numpy.linalg), plus a
KKT-certificate checker. Shares no code with oracle/nmpc_oracle.c (Riccati recursion, different
variables), so agreement pins the oracle's QP solves.
"""
import numpy as np


def condense(q, nbx, idxbx, nbu, idxbu):
    A, B, b, dx0 = q["A"], q["B"], q["b"], q["dx0"]
    N, nx, nu = B.shape[0], B.shape[1], B.shape[2]
    nU = N * nu
    # x_k = Gx[k] @ U + cx[k]
    Gx = np.zeros((N + 1, nx, nU))
    cx = np.zeros((N + 1, nx))
    cx[0] = dx0
    for k in range(N):
        Gx[k + 1] = A[k] @ Gx[k]
        Gx[k + 1][:, k * nu:(k + 1) * nu] += B[k]
        cx[k + 1] = A[k] @ cx[k] + b[k]
    H = np.diag(q["Hu"].reshape(-1)).astype(float)
    g = q["gu"].reshape(-1).astype(float).copy()
    for k in range(1, N + 1):
        Qk = np.diag(q["Hx"][k])
        H += Gx[k].T @ Qk @ Gx[k]
        g += Gx[k].T @ (Qk @ cx[k] + q["gx"][k])
    rows, rhs = [], []
    for k in range(N):
        for i in range(nbu):
            e = np.zeros(nU)
            e[k * nu + idxbu[i]] = 1.0
            rows += [e, -e]
            rhs += [q["ubu"][k, i], -q["lbu"][k, i]]
    for k in range(1, N + 1):
        for i in range(nbx):
            row = Gx[k][idxbx[i]]
            c = cx[k][idxbx[i]]
            rows += [row, -row]
            rhs += [q["ubx"][k, i] - c, -(q["lbx"][k, i] - c)]
    return H, g, np.array(rows), np.array(rhs), Gx, cx


def dense_ipm(H, g, C, d, tol=1e-12, iters=200, thr0=0.5):
    """Mehrotra predictor-corrector on min 1/2 u'Hu + g'u s.t. Cu + s = d, s >= 0, z >= 0 (dense KKT
    solves by numpy.linalg). Second-order term damped by the affine step, pure centring when the
    corrector step is short (same safeguards as the oracle; the linear algebra shares nothing with it)."""
    n, m = H.shape[0], C.shape[0]
    u = np.zeros(n)
    s = np.maximum(d - C @ u, thr0)
    z = 1.0 / s
    for it in range(iters):
        rd = H @ u + g + C.T @ z
        rp = C @ u + s - d
        mu = s @ z / m
        if max(np.abs(rd).max(), np.abs(rp).max()) < tol and mu < tol:
            break
        Kmat = H + C.T @ ((z / s)[:, None] * C)

        def solve(rc):
            r = -rd - C.T @ ((z * rp - rc) / s)
            du = np.linalg.solve(Kmat, r)
            ds = -rp - C @ du
            dz = -(rc + z * ds) / s
            return du, ds, dz

        def step(v, dv):
            neg = dv < 0
            return min(1.0, np.min(-v[neg] / dv[neg])) if neg.any() else 1.0

        du, ds, dz = solve(s * z)
        aa = min(step(s, ds), step(z, dz))
        mu_aff = (s + aa * ds) @ (z + aa * dz) / m
        sigma = min(1.0, (mu_aff / mu) ** 3)
        du, ds, dz = solve(s * z + aa * ds * dz - sigma * mu)
        a = min(1.0, 0.995 * min(step(s, ds), step(z, dz)))
        if a < 0.1:
            du, ds, dz = solve(s * z - max(sigma, 0.3) * mu)
            a = min(1.0, 0.995 * min(step(s, ds), step(z, dz)))
        u, s, z = u + a * du, s + a * ds, z + a * dz
    return u, z, it


def oracle_multipliers(sol, N, nbu, nbx):
    """Map the oracle's per-stage bound multipliers onto the rows of condense()'s C."""
    z = []
    for k in range(N):
        for i in range(nbu):
            z += [sol["lam_ub"][k, i], sol["lam_lb"][k, i]]
    for k in range(1, N + 1):
        off = nbu if k < N else 0
        for i in range(nbx):
            z += [sol["lam_ub"][k, off + i], sol["lam_lb"][k, off + i]]
    return np.array(z)


def kkt_certificate(H, g, C, d, u, z):
    """Max violation of stationarity, primal feasibility, dual feasibility and complementarity."""
    stat = np.abs(H @ u + g + C.T @ z).max()
    prim = max(0.0, (C @ u - d).max())
    dual = max(0.0, (-z).max())
    comp = np.abs(z * (d - C @ u)).max()
    return stat, prim, dual, comp
