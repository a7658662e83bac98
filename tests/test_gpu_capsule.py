"""GPU tests of the drop-in acados capsule ABI (include/acados_solver_{name}.h + acados_c/ocp_nlp_interface.h).

The controller mirrors in nmpc_nav_control_amd/controller.py drive the capsule exactly as the reference's
wrappers do (create, ocp_nlp_constraints_model_set / cost_model_set, {name}_acados_solve, ocp_nlp_out_get,
ocp_nlp_get "time_tot", reset); the fp64 oracle replays the same wrapper semantics (prepare -> sqp_rti -> post)
on the same inputs. Tolerance as in test_gpu_parity.py: |u0 - u0_oracle| <= 1e-3 and commands alike.
"""
import numpy as np
import pytest

from nmpc_nav_control_amd.controller import (CmdVelDiff, CmdVelOmni4, CmdVelTric, NMPCNavControlDiff,
                                             NMPCNavControlOmni4, NMPCNavControlTric, Pose, Vel, batch_solve)
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu
TOL = 1e-3
N = 20
W_DIFF = [10, 10, 5, 0, 0, 0, 0, 1, 1]
W_OMNI = [10, 10, 5] + [0] * 8 + [1, 1, 1, 1]


def make(model):
    if model == "diff":
        return NMPCNavControlDiff(1 / 40, 0.270, 0.1, 1.0, 1.0, W_DIFF, N=N), CmdVelDiff
    if model == "omni4":
        return NMPCNavControlOmni4(1 / 40, 0.535, 0.1, 1.0, 1.0, W_OMNI, N=N), CmdVelOmni4
    d2r = np.pi / 180
    return NMPCNavControlTric(1 / 40, 0.270, 0.1, 0.5, 1.0, 1.0, -45 * d2r, 45 * d2r, 15 * d2r, W_DIFF, N=N), CmdVelTric


def plant(model, o, x0, u0):
    xn, _, _ = o.rk4(x0, u0, 1 / 40)
    if model == "diff":
        vel = (0.5 * (xn[3] + xn[4]), 0.0, (xn[4] - xn[3]) / 0.270)
        return xn, vel, 0.0
    if model == "omni4":
        v = 0.25 * (xn[3] - xn[4] + xn[5] - xn[6])
        vn = 0.25 * (-xn[3] - xn[4] + xn[5] + xn[6])
        w = -(xn[3] + xn[4] + xn[5] + xn[6]) / (2 * 0.535)
        return xn, (v, vn, w), 0.0
    return xn, (xn[3], 0.0, 0.0), xn[4]


def path(t0, n):
    """A gentle arc of n reference poses ahead of time t0 (crosses +-pi in theta to exercise the unwrap)."""
    s = 0.02 * (t0 + np.arange(1, n + 1))
    th = 3.0 + 0.8 * s
    th = (th + np.pi) % (2 * np.pi) - np.pi
    return [Pose(0.3 * np.cos(0.8 * si), 0.3 * np.sin(0.8 * si), thi) for si, thi in zip(s, th)]


@pytest.mark.parametrize("model", ["diff", "omni4", "tric"])
def test_capsule_closed_loop_matches_oracle(built, model):
    ctl, Cmd = make(model)
    assert ctl.getHorizon() == N
    o = Oracle(model, N, rule="acados")  # the capsule ABI: no early exit
    xb, ub = o.iterate_create()
    carried = np.zeros(o.nbx)
    pose, vel, steer = np.array([0.05, -0.02, 2.9]), np.array([0.1, 0.0, 0.05]), 0.0
    if model == "tric":
        ctl.setSteeringWheelAngle(steer)
    for tick in range(8):
        refs = path(tick, N - 3 + tick % 4)  # sometimes shorter than N+1: exercises the padding
        cmd = Cmd()
        ok, ms = ctl.run(Pose(*pose), Vel(*vel), refs, cmd)
        assert ok and ms >= 0.0
        traj = np.array([[p.x, p.y, p.theta] for p in refs])
        x0, yref, We = o.prepare(pose, vel, steer, traj, carried)
        s, st, xb, ub = o.sqp_rti(xb, ub, x0, yref, We)
        assert s == 0
        cmd_o, carried = o.post(x0, ub[0])
        np.testing.assert_allclose(ctl.u0, ub[0], atol=TOL)
        got = [cmd.v, cmd.w] if model == "diff" else ([cmd.v, cmd.vn, cmd.w] if model == "omni4" else [cmd.v, cmd.alpha])
        np.testing.assert_allclose(got, cmd_o[:len(got)], atol=TOL)
        xn, v3, steer = plant(model, o, x0, ub[0])
        pose, vel = xn[:3], np.array(v3)
        if model == "tric":
            ctl.setSteeringWheelAngle(steer)
    # reset_mpc zeroes the iterate (acados reset semantics)
    assert ctl.reset_mpc()
    xs, us = ctl.iterate()
    assert not xs.any() and not us.any()


def test_capsule_errors_raise(built):
    ctl, Cmd = make("diff")
    with pytest.raises(RuntimeError, match="Invalid command velocity type"):
        ctl.run(Pose(), Vel(), path(0, N + 1), CmdVelOmni4())


def test_batch_solve_equals_individual(built):
    """{name}_acados_batch_solve of many capsules = one solve per capsule."""
    ctls = [make("diff")[0] for _ in range(6)]
    twins = [make("diff")[0] for _ in range(6)]
    for i, (a, b) in enumerate(zip(ctls, twins)):
        x0 = np.array([0.1 * i, -0.05 * i, 0.3 * i, 0.1, -0.1, 0.05 * i, -0.05 * i])
        for c in (a, b):
            c._cset(0, "lbx", x0)
            c._cset(0, "ubx", x0)
            c.yref[:, :3] = [0.4, 0.2 * i, 0.1]
            for k in range(N + 1):
                c._wset(k, "yref", c.yref[k, : (c.nx if k == N else c.ny)])
    status = batch_solve(ctls)
    assert (status == 0).all()
    for a, b in zip(ctls, twins):
        b._solve()
        xa, ua = a.iterate()
        xb_, ub_ = b.iterate()
        np.testing.assert_allclose(ua, ub_, atol=1e-6)
        np.testing.assert_allclose(xa, xb_, atol=1e-6)


def _set_tick(c, x0, yref):
    c._cset(0, "lbx", x0)
    c._cset(0, "ubx", x0)
    for k in range(N + 1):
        c._wset(k, "yref", yref[k, : (c.nx if k == N else c.ny)])


def test_capsule_warm_start_and_reset(built):
    """A capsule with qp_warm_start = 2 (acados: primal and dual), solved tick after tick, starts its IPM from its own previous multipliers: a fresh
    capsule given the same inputs and iterate starts cold, in the same launch, and reaches the same QP solution.
    After reset the next solve is cold again: bit-identical to a fresh capsule's solve from a zero iterate."""
    a = make("diff")[0]
    a.solver_opts_set("qp_warm_start", 2)  # (the capsule default is acados' cold start)
    o = Oracle("diff", N, rule="acados")
    x0 = np.array([0.05, -0.02, 2.9, 0.1, 0.05, 0.0, 0.0])
    yref = np.zeros((N + 1, a.ny))
    it_warm = it_cold = 0
    for tick in range(10):
        for k, p in enumerate(path(tick, N + 1)):
            yref[k, :3] = [p.x, p.y, np.unwrap([x0[2], p.theta])[1]]
        cold = make("diff")[0]
        cold.solver_opts_set("qp_warm_start", 2)  # same options as a, so both share one launch; fresh, so cold
        xs, us = a.iterate()
        for k in range(N + 1):
            cold.out_set(k, "x", xs[k])
        for k in range(N):
            cold.out_set(k, "u", us[k])
        for c in (a, cold):
            _set_tick(c, x0, yref)
        assert (batch_solve([a, cold]) == 0).all()
        ua, uc = a.iterate()[1], cold.iterate()[1]
        np.testing.assert_allclose(ua[0], uc[0], atol=2e-4)
        if tick > 0:
            it_warm += a.qp_iter()
            it_cold += cold.qp_iter()
        x0 = o.rk4(x0, ua[0], 1 / 40)[0]
    assert it_warm < it_cold, (it_warm, it_cold)
    assert a.reset_mpc()
    fresh = make("diff")[0]
    fresh.reset_mpc()
    for c in (a, fresh):
        _set_tick(c, x0, yref)
        c._solve()
        assert c.status == 0
    assert a.qp_iter() == fresh.qp_iter()
    np.testing.assert_array_equal(a.iterate()[1], fresh.iterate()[1])
    np.testing.assert_array_equal(a.iterate()[0], fresh.iterate()[0])


def test_unsupported_ocp_data_rejected_and_recovered(built):
    """The shim rejects OCP data the batched kernel does not implement (status 4 -> the wrapper's exception) and
    re-validates after every setter: the cached stage-uniform data must not hide a later change either way."""
    ctl, _ = make("diff")
    x0 = np.array([0.1, -0.05, 0.3, 0.1, -0.1, 0.05, -0.05])
    ctl._cset(0, "lbx", x0)
    ctl._cset(0, "ubx", x0)
    ctl._solve()
    assert ctl.status == 0
    Wd = np.diag(W_DIFF).astype(float)
    Wn = Wd.copy()
    Wn[0, 1] = Wn[1, 0] = 0.5
    ctl._wset(3, "W", Wn.flatten(order="F"))
    with pytest.raises(RuntimeError):
        ctl._solve()
    ctl._wset(3, "W", Wd.flatten(order="F"))
    ctl._solve()
    assert ctl.status == 0
    ctl._cset(5, "lbu", np.array([-0.5, -1.0]))  # stage-varying input bound
    with pytest.raises(RuntimeError):
        ctl._solve()
    ctl._cset(5, "lbu", np.array([-1.0, -1.0]))
    ctl._solve()
    assert ctl.status == 0
    ctl._cset(0, "ubx", x0 + 0.1)  # x0 must stay an equality
    with pytest.raises(RuntimeError):
        ctl._solve()


def test_capsule_cold_start_option_matches_oracle(built):
    """ocp_nlp_solver_opts_set(.., "qp_warm_start", 0): every solve starts the IPM cold, as HPIPM does in the
    reference's generated solver (scripts/diff/generate_c_code.py:68-74). Same QP solutions as the oracle; the
    cold capsule needs at least as many IPM iterations as the warm one over the same closed loop."""
    iters = {}
    for warm in (2, 0):
        ctl, Cmd = make("diff")
        ctl.solver_opts_set("qp_warm_start", warm)
        o = Oracle("diff", N, rule="acados")
        xb, ub = o.iterate_create()
        carried = np.zeros(o.nbx)
        pose, vel = np.array([0.05, -0.02, 2.9]), np.array([0.1, 0.0, 0.05])
        its = []
        for tick in range(10):
            refs = path(tick, N + 1)
            ok, _ = ctl.run(Pose(*pose), Vel(*vel), refs, Cmd())
            assert ok
            its.append(ctl.qp_iter())
            traj = np.array([[p.x, p.y, p.theta] for p in refs])
            x0, yref, We = o.prepare(pose, vel, 0.0, traj, carried)
            s, st, xb, ub = o.sqp_rti(xb, ub, x0, yref, We)
            assert s == 0
            _, carried = o.post(x0, ub[0])
            np.testing.assert_allclose(ctl.u0, ub[0], atol=TOL)
            xn, v3, _ = plant("diff", o, x0, ub[0])
            pose, vel = xn[:3], np.array(v3)
        iters[warm] = its
    assert sum(iters[0][1:]) >= sum(iters[2][1:]), iters


def test_capsule_infeasible_qp_has_no_early_exit(built):
    """The capsule ABI has no early infeasibility exit (qp_infeas_lambda 0, as HPIPM: a hard QP runs on until its
    iteration cap or a numerical failure), while the batched default stops an infeasible QP with status 4 once its
    multipliers diverge (tests/test_gpu_fleet.py). A carried vel-ref of 50 m/s against the 1 m/s bound cannot be
    brought inside it: the capsule runs more IPM iterations than the batched early exit takes."""
    import torch

    from nmpc_nav_control_amd._lib import default_params
    from nmpc_nav_control_amd.batch import BatchSolver
    ctl, Cmd = make("diff")
    ctl.solver_opts_set("qp_iter_max", 40)
    x0 = np.array([0.0, 0.0, 0.2, 0.0, 0.0, 50.0, 0.0])
    ctl._cset(0, "lbx", x0)
    ctl._cset(0, "ubx", x0)
    ctl.yref[:, :3] = [0.5, 0.2, 0.3]
    for k in range(N + 1):
        ctl._wset(k, "yref", ctl.yref[k] if k < N else ctl.yref[k][:ctl.nx])
    getattr(ctl._S, f"{ctl._name}_acados_solve")(ctl._capsule)  # (status not raised: inspected below)
    cap_iter = ctl.qp_iter()
    # the same QP through the batched API (early exit on)
    dev = torch.device("cuda:0")
    prm = default_params("diff", N)
    prm.qp_iter_max = 40
    prm.terminal_hack = 0
    h = BatchSolver("diff", N, 1, params=prm)
    yref = torch.zeros(N + 1, 9, 1, device=dev)
    yref[:, :3, 0] = torch.tensor([0.5, 0.2, 0.3])
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    it = torch.zeros(1, dtype=torch.int32, device=dev)
    h.solve(torch.tensor(x0, dtype=torch.float32, device=dev)[:, None], yref, status=st, qp_iter=it)
    torch.cuda.synchronize()
    assert int(st[0]) == 4 and int(it[0]) < 30, (int(st[0]), int(it[0]))
    assert cap_iter > int(it[0]), (cap_iter, int(it[0]))
