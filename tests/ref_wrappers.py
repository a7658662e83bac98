"""Driving the reference's own wrapper classes (oracle/ref_driver.cpp, built into oracle/_ref/ by `make -C oracle
ref`) and checking what their run() did against the oracle's restatement of it.

The ticks: per model, a few robots of the seeded fleet in closed loop (the oracle's SQP-RTI step and the plant), and
edge-case robots for the branches of NMPCNavControl{Diff,Omni4,Tric}.cpp run():
  * reference lists of 1, 2, 5, N - 1, N, N + 1 and N + 20 poses (the padding branch, :107-118 of the diff wrapper);
  * +-pi crossings of the robot's heading and of the reference headings, once and many times per list (unwrapAngle,
    NMPCNavControl.cpp:25-31, applied pose by pose);
  * the diff terminal-weight hack on (last two poses equal, or padded) and off (:127-139);
  * tric steering-wheel angles inside and outside the alpha bounds (setSteeringWheelAngle, NMPCNavControlTric.h:67);
  * reset_mpc() between ticks (:177-181).
The per-tick check (check_robot): the wrapper's x0 / yref / W_e equal oc_prepare's bit for bit, its command equals
oc_post's on the u0 the solver returned, bit for bit, and its solve is the oracle's (bit for bit when the solver is
the oracle itself, within the parity tolerance on the device). Test infrastructure only."""
import os
import subprocess

import numpy as np

from nmpc_nav_control_amd.scenario import make_fleet, refs_for
from oracle.oracle import Oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = os.path.join(ROOT, "oracle", "_ref")
EXE = {"oracle": os.path.join(REF_DIR, "ref_wrappers_oracle"), "device": os.path.join(REF_DIR, "ref_wrappers_device")}
MODEL_ID = {"diff": 0, "omni4": 1, "tric": 2}
N = 80  # the horizon the shipped codegen yaml bakes into the generated headers the wrappers compile against


def oracle(model):
    return Oracle(model, N, rule="acados")


def config_line(o):
    """The wrapper constructor's arguments (the ROS-yaml values oc_params_default restates)."""
    prm = o.prm
    v_max, a_max = prm.ubx[0], prm.ubu[0]
    if o.model == "tric":
        amin, amax, damax = prm.lbx[1], prm.ubx[1], prm.ubu[1]
    else:
        amin, amax, damax = -np.pi / 4, np.pi / 4, np.pi / 12
    vals = [MODEL_ID[o.model], prm.dt_ctrl, prm.p[0], prm.p[1], prm.p[2], v_max, a_max, amin, amax, damax, o.ny]
    vals += [prm.W[i] for i in range(o.ny)]
    return " ".join(repr(float(v)) if isinstance(v, float) else str(v) for v in vals)


def _wrap(a):
    return (a + np.pi) % (2.0 * np.pi) - np.pi


def _tick(pose, vel, traj, steer=0.0, reset=0):
    return dict(pose=np.asarray(pose, np.float64), vel=np.asarray(vel, np.float64),
                traj=np.asarray(traj, np.float64).reshape(-1, 3), steer=float(steer), reset=int(reset))


def closed_loop_robots(o, robots, ticks, seed=20251018):
    """Seeded fleet robots in closed loop with the oracle (prepare -> sqp_rti -> post -> RK4 plant), as
    tests/helpers.oracle_closed_loop, recording the wrapper inputs of every tick."""
    from helpers import plant_measure
    model = o.model
    fl = make_fleet(model, robots, seed=seed)
    out = []
    for i in range(robots):
        pose = fl["pose"][:, i].astype(np.float64).copy()
        vel = fl["vel"][:, i].astype(np.float64).copy()
        steer = float(fl["steer"][i])
        carried = np.zeros(o.nbx)  # the wrappers' acados_in_.x0 starts at 0 (NMPCNavControlDiff.cpp:14)
        s = float(fl["s"][i])
        xb, ub = o.iterate_create()
        seq = []
        for t in range(ticks):
            traj, s = refs_for(fl["path"], i, pose, s, N, o.prm.dt_ctrl)
            seq.append(_tick(pose, vel, traj, steer))
            x0, yref, We = o.prepare(pose, vel, steer, traj, carried)
            st, _, xb2, ub2 = o.sqp_rti(xb, ub, x0, yref, We)
            if st != 0:
                break
            xb, ub = xb2, ub2
            _, carried = o.post(x0, ub[0])
            xn, _, _ = o.rk4(x0, ub[0], o.prm.dt_ctrl)
            pose = xn[:3].copy()
            vel, steer = plant_measure(model, xn, o.prm.p)
            steer = float(steer)
        out.append(seq)
    return out


def edge_robots(o, seed=7):
    """Edge-case robots (module docstring): each a list of consecutive ticks on one wrapper."""
    rng = np.random.default_rng(seed)
    model = o.model
    robots = []

    def line(p0, heading, n, step=0.02, turn=0.0):
        th = heading + turn * np.arange(1, n + 1)
        xy = np.cumsum(np.stack([step * np.cos(th), step * np.sin(th)], 1), 0) + np.asarray(p0[:2])
        return np.concatenate([xy, _wrap(th)[:, None]], 1)

    vel = [0.3, 0.05 if model == "omni4" else 0.0, 0.2]
    # list lengths around N + 1 (padding), moving along a line
    seq = []
    pose = np.array([0.5, -0.2, 0.3])
    for n in (1, 2, 5, N - 1, N, N + 1, N + 20, 3):
        seq.append(_tick(pose, vel, line(pose, 0.3, n), steer=0.1))
        pose = pose + np.array([0.01, 0.003, 0.002])
    robots.append(seq)
    # +-pi: the robot's heading and the references cross the cut, once and many times per list
    seq = []
    for th0, turn in ((np.pi - 0.03, 0.01), (-np.pi + 0.02, -0.01), (np.pi - 0.001, 0.5), (-np.pi + 0.4, -0.7),
                      (np.pi, 0.0), (-np.pi, 0.02)):
        pose = np.array([1.0, 2.0, _wrap(th0) if abs(th0) != np.pi else th0])
        seq.append(_tick(pose, vel, line(pose, th0, N + 1, turn=turn), steer=-0.2))
    robots.append(seq)
    # terminal-weight hack on (duplicated last pose, padded list) and off (distinct poses), alternating
    seq = []
    pose = np.array([-1.0, 0.5, -2.0])
    for kind in ("distinct", "dup", "distinct", "short", "distinct", "dup_x_only"):
        tr = line(pose, -2.0, N + 1)
        if kind == "dup":
            tr[-1] = tr[-2]
        elif kind == "short":
            tr = tr[:N // 2]
        elif kind == "dup_x_only":
            tr[-1, 0] = tr[-2, 0]  # only x equal: the hack needs x, y and theta equal
        seq.append(_tick(pose, vel, tr))
    robots.append(seq)
    # steering angles inside and outside the tric alpha bounds (unused by diff / omni4), and resets
    seq = []
    pose = np.array([0.0, 0.0, 0.0])
    for t, st in enumerate((0.0, 0.3, -0.7, 0.785, 1.2, -1.5, 0.05)):
        tr = line(pose, 0.0, N + 1, step=0.02, turn=0.004)
        seq.append(_tick(pose + 0.001 * rng.standard_normal(3), vel, tr, steer=st, reset=int(t in (3, 5))))
    robots.append(seq)
    return robots


def run_driver(kind, o, robots, timeout=600):
    """Feed the robots to the driver; returns one list of tick records per robot."""
    lines = [config_line(o)]
    for seq in robots:
        lines.append("R")
        for t in seq:
            tr = t["traj"]
            vals = [t["reset"], t["steer"], *t["pose"], *t["vel"], len(tr), *tr.ravel()]
            lines.append("T " + " ".join(repr(float(v)) for v in vals))
    lines.append("E")
    r = subprocess.run([EXE[kind]], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    recs, cur = [], None
    for line in r.stdout.splitlines():
        tag, _, rest = line.partition(" ")
        if tag == "tick":
            ok, status, qp_iter = (int(v) for v in rest.split())
            cur = dict(ok=ok, status=status, qp_iter=qp_iter)
            recs.append(cur)
        elif tag == "err":
            cur["err"] = rest
        else:
            cur[tag] = np.array([float(v) for v in rest.split()])
    n = [len(s) for s in robots]
    assert len(recs) == sum(n), (len(recs), n, r.stderr[-2000:])
    out, i = [], 0
    for k in n:
        out.append(recs[i:i + k])
        i += k
    return out, r.stderr


def check_robot(o, seq, recs, solve_tol=None):
    """Checks of one robot's ticks (module docstring). solve_tol None: the solver is the oracle (bit for bit);
    else the device solve, |u0 - oracle| and the predicted trajectory within solve_tol. Returns per-tick u0 errors."""
    nx, nu, ny = o.nx, o.nu, o.ny
    carried = np.zeros(o.nbx)
    xb_track, ub_track = o.iterate_create()
    errs = []
    for t, (tk, rc) in enumerate(zip(seq, recs)):
        where = f"tick {t}"
        assert rc["ok"] == 1 and rc["err"] == "-", (where, rc["err"])
        # pre-solve: what the reference's run() set, against oc_prepare (NMPCNavControl*.cpp pre-solve)
        x0, yref, We = o.prepare(tk["pose"], tk["vel"], tk["steer"], tk["traj"], carried)
        np.testing.assert_array_equal(rc["x0"], x0, err_msg=where + " x0")
        np.testing.assert_array_equal(rc["yref"].reshape(N + 1, ny), yref, err_msg=where + " yref")
        np.testing.assert_array_equal(rc["We"], We, err_msg=where + " W_e")
        # the iterate the solve started from: create / reset / the previous solve's
        xb0 = rc["xb"].reshape(N + 1, nx)
        ub0 = rc["ub"].reshape(N, nu)
        if tk["reset"]:
            xb_track, ub_track = np.zeros_like(xb_track), np.zeros_like(ub_track)
        if solve_tol is None or t == 0 or tk["reset"]:
            np.testing.assert_array_equal(xb0, xb_track, err_msg=where + " iterate before the solve")
            np.testing.assert_array_equal(ub0, ub_track, err_msg=where + " iterate before the solve")
        st, _, xb1, ub1 = o.sqp_rti(xb0, ub0, x0, yref, We)
        assert st == 0, (where, "oracle status", st)
        u0, x1 = rc["u0"], rc["x1"]
        if solve_tol is None:
            np.testing.assert_array_equal(u0, ub1[0], err_msg=where + " u0")
            np.testing.assert_array_equal(x1, xb1[1], err_msg=where + " x1")
        else:
            err = float(np.abs(u0 - ub1[0]).max())
            assert err <= solve_tol, (where, "u0", u0, ub1[0])
            assert float(np.abs(x1 - xb1[1]).max()) <= solve_tol, (where, "x1", x1, xb1[1])
            errs.append(err)
        # post-solve: the wrapper's command from the u0 its solver returned, against oc_post
        cmd, carried = o.post(x0, u0)
        ncmd = 2 if o.model != "omni4" else 3
        np.testing.assert_array_equal(rc["cmd"][:ncmd], cmd[:ncmd], err_msg=where + " cmd")
        xb_track, ub_track = xb1, ub1
    return errs
