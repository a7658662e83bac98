"""Shared helpers of the parity tests: oracle closed loops and SoA/AoS conversions."""
import numpy as np

from nmpc_nav_control_amd.scenario import make_fleet, refs_for
from oracle.oracle import Oracle


def oracle_closed_loop(model, N, B, ticks, seed=20250824, o=None, start=0, u0_log=None):
    """Run the fp64 oracle in closed loop (plant = RK4 of the model) for `ticks` ticks over robots
    [start, start + B) of the seeded fleet. Returns the oracle and, for the last tick, the solve inputs
    (x0, yref, We, xbar, ubar) per robot; appends each tick's u0 [B][nu] to `u0_log` when given."""
    o = o or Oracle(model, N, rule="batched")
    fl = make_fleet(model, B, seed=seed, start=start)
    pose = fl["pose"].T.astype(np.float64).copy()
    vel = fl["vel"].T.astype(np.float64).copy()
    steer = fl["steer"].astype(np.float64).copy()
    carried = fl["carried"].T.astype(np.float64).copy()
    s = fl["s"].astype(np.float64).copy()
    xbar = np.zeros((B, N + 1, o.nx))
    ubar = np.zeros((B, N, o.nu))
    for i in range(B):
        xbar[i], ubar[i] = o.iterate_create()
    last = None
    for t in range(ticks):
        rec = []
        u0s = np.full((B, o.nu), np.nan)
        for i in range(B):
            traj, s[i] = refs_for(fl["path"], i, pose[i], s[i], N, o.prm.dt_ctrl)
            x0, yref, We = o.prepare(pose[i], vel[i], steer[i], traj, carried[i])
            rec.append((x0, yref, We, xbar[i].copy(), ubar[i].copy()))
            st, _, xb, ub = o.sqp_rti(xbar[i], ubar[i], x0, yref, We)
            if st != 0:
                continue
            xbar[i], ubar[i] = xb, ub
            u0s[i] = ub[0]
            _, carried[i] = o.post(x0, ub[0])
            xn, _, _ = o.rk4(x0, ub[0], o.prm.dt_ctrl)
            pose[i] = xn[:3]
            vel[i], steer[i] = plant_measure(model, xn, o.prm.p)
        last = rec
        if u0_log is not None:
            u0_log.append(u0s)
    return o, last


def plant_measure(model, xn, p):
    if model == "diff":
        return np.array([0.5 * (xn[3] + xn[4]), 0.0, (xn[4] - xn[3]) / p[0]]), 0.0
    if model == "omni4":
        return np.array([0.25 * (xn[3] - xn[4] + xn[5] - xn[6]), 0.25 * (-xn[3] - xn[4] + xn[5] + xn[6]),
                         -(xn[3] + xn[4] + xn[5] + xn[6]) / (2.0 * p[0])]), 0.0
    return np.array([xn[3], 0.0, 0.0]), xn[4]
