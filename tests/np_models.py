"""Independent numpy restatement of the reference's model ODEs (test infrastructure).

Written directly from the CasADi expressions of the reference, not from oracle/nmpc_oracle.c:
  diff2amr  scripts/diff/diff_amr_model.py:42-60
  omni4amr  scripts/omni4/omni4_amr_model.py:52-73
  tric3amr  scripts/tric/tric_amr_model.py:43-55 (cos_alpha = sin(alpha) at :45)
"""
import numpy as np

PARAMS = {"diff": (0.270, 0.1), "omni4": (0.535, 0.1), "tric": (0.270, 0.1, 0.5)}
DIMS = {"diff": (7, 2), "omni4": (11, 4), "tric": (7, 2)}


def f_expl(model, x, u, p=None, tric_sin_bug=True):
    p = PARAMS[model] if p is None else p
    if model == "diff":
        dist_b, tau_v = p
        x_, y_, theta, vl, vr, vl_ref, vr_ref = x
        v = (vr + vl) / 2.0
        w = (vr - vl) / dist_b
        return np.array([v * np.cos(theta), v * np.sin(theta), w,
                         -1.0 / tau_v * vl + 1.0 / tau_v * vl_ref,
                         -1.0 / tau_v * vr + 1.0 / tau_v * vr_ref,
                         u[0], u[1]])
    if model == "omni4":
        l1_plus_l2, tau_v = p
        theta = x[2]
        v1, v2, v3, v4 = x[3:7]
        v = (v1 - v2 + v3 - v4) / 4.0
        vn = (-v1 - v2 + v3 + v4) / 4.0
        w = (-v1 - v2 - v3 - v4) / (2.0 * l1_plus_l2)
        out = [v * np.cos(theta) - vn * np.sin(theta), v * np.sin(theta) + vn * np.cos(theta), w]
        out += [-1.0 / tau_v * x[3 + i] + 1.0 / tau_v * x[7 + i] for i in range(4)]
        out += [u[i] for i in range(4)]
        return np.array(out)
    dist_d, tau_v, tau_a = p
    theta, v, alpha, v_ref, alpha_ref = x[2], x[3], x[4], x[5], x[6]
    cos_alpha = np.sin(alpha) if tric_sin_bug else np.cos(alpha)
    sin_alpha = np.sin(alpha)
    return np.array([v * np.cos(theta) * cos_alpha, v * np.sin(theta) * cos_alpha, v / dist_d * sin_alpha,
                     -1.0 / tau_v * v + 1.0 / tau_v * v_ref, -1.0 / tau_a * alpha + 1.0 / tau_a * alpha_ref,
                     u[0], u[1]])


def rk4(model, x, u, h, **kw):
    k1 = f_expl(model, x, u, **kw)
    k2 = f_expl(model, x + 0.5 * h * k1, u, **kw)
    k3 = f_expl(model, x + 0.5 * h * k2, u, **kw)
    k4 = f_expl(model, x + h * k3, u, **kw)
    return x + h / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)


def fd_jac(fun, z, eps=1e-6):
    f0 = fun(z)
    J = np.zeros((f0.size, z.size))
    for j in range(z.size):
        e = np.zeros_like(z)
        e[j] = eps
        J[:, j] = (fun(z + e) - fun(z - e)) / (2 * eps)
    return J
