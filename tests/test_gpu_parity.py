"""GPU parity of the HIP SQP-RTI path against the fp64 CPU oracle (same inputs, same warm iterate).

Tolerance (DESIGN.md "Parity"): |u0 - u0_oracle|_inf <= 1e-3 and the predicted state
trajectory within 1e-3 (m / rad / m/s), with the GPU IPM stopped by its fp32 rule (tol_stat 1e-4,
tol_ineq 1e-6, tol_comp 1e-10) and the oracle by its fp64 rule (1e-8 / 1e-8 / 1e-12). The inputs of later
stages are only warm-start data; their fp32 error (up to ~1e-3 mid-horizon, where the cost is flat in u:
R*dt = 0.025 against terminal weights of 1000) is bounded at TOL_UTRAJ.
"""
import numpy as np
import pytest
import torch

from helpers import oracle_closed_loop

from nmpc_nav_control_amd._lib import default_params
from nmpc_nav_control_amd.batch import BatchSolver
from nmpc_nav_control_amd.scenario import make_fleet
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu
TOL_U = 1e-3
TOL_X = 1e-3
TOL_UTRAJ = 5e-3
DEV = torch.device("cuda:0")
MODELS = ["diff", "omni4", "tric"]


def t(a, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device=DEV, dtype=dtype)


def upload_iterate(solver, xbars, ubars):
    """xbars [B][N+1][NX] -> device [(N+1)*NX][cap]."""
    B = len(xbars)
    xv, uv, _ = solver.state()
    X = xv.to_tensor()
    U = uv.to_tensor()
    X[:, :B] = t(np.stack(xbars).reshape(B, -1).T)
    U[:, :B] = t(np.stack(ubars).reshape(B, -1).T)
    xv.copy_from(X)
    uv.copy_from(U)


# IPM direction rules (nmpc_model_params.qp_ipm): the default one direction per iteration, and Mehrotra's
# predictor-corrector (the oracle's rule); both must reach the oracle's QP solution within the tolerance
IPMS = {"single": 1, "mehrotra": 0}


def make_solver(model, N, cap, ipm):
    prm = default_params(model, N)
    prm.qp_ipm = IPMS[ipm]
    return BatchSolver(model, N, cap, params=prm)


@pytest.mark.parametrize("ipm", sorted(IPMS))
@pytest.mark.parametrize("model", MODELS)
# (80: the shipped codegen horizon; 1 and 2: the shortest horizons; B not a multiple of the 4 teams per wave)
@pytest.mark.parametrize("N,B,ticks", [(20, 48, 8), (40, 5, 4), (80, 13, 3), (1, 7, 4), (2, 3, 4)])
def test_solve_matches_oracle(built, ipm, model, N, B, ticks):
    o, rec = oracle_closed_loop(model, N, B, ticks)
    solver = make_solver(model, N, 64, ipm)
    nx, nu, ny = o.nx, o.nu, o.ny
    x0 = np.stack([r[0] for r in rec]).T
    yref = np.stack([r[1] for r in rec]).transpose(1, 2, 0)
    We = np.stack([r[2] for r in rec]).T
    upload_iterate(solver, [r[3] for r in rec], [r[4] for r in rec])
    xtraj = torch.zeros((N + 1) * nx, B, device=DEV)
    utraj = torch.zeros(N * nu, B, device=DEV)
    status = torch.full((B,), -7, dtype=torch.int32, device=DEV)
    qp_iter = torch.zeros(B, dtype=torch.int32, device=DEV)
    solver.solve(t(x0), t(yref), We=t(We), xtraj=xtraj, utraj=utraj, status=status, qp_iter=qp_iter)
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    assert (st == 0).all(), st
    xg = xtraj.cpu().numpy().T.reshape(B, N + 1, nx)
    ug = utraj.cpu().numpy().T.reshape(B, N, nu)
    eu0, eu, ex = 0.0, 0.0, 0.0
    for i, r in enumerate(rec):
        s, stats, xb, ub = o.sqp_rti(r[3], r[4], r[0], r[1], r[2])
        assert s == 0
        eu0 = max(eu0, np.abs(ug[i][0] - ub[0]).max())
        eu = max(eu, np.abs(ug[i] - ub).max())
        ex = max(ex, np.abs(xg[i] - xb).max())
    assert eu0 <= TOL_U, eu0
    assert ex <= TOL_X, ex
    assert eu <= TOL_UTRAJ, eu
    assert qp_iter.cpu().numpy().max() < 50


def test_solve_iterate_equals_resident_solve(built):
    """nmpc_batch_solve_iterate (the capsule ABI's entry: the iterate in caller memory with its own leading
    dimension, updated in place) equals nmpc_batch_solve on the handle's resident iterate bit for bit, on a cold
    tick and on the warm-started tick after it."""
    N, B = 40, 13
    o, rec = oracle_closed_loop("diff", N, B, 2)
    nx, nu = o.nx, o.nu
    a, b = make_solver("diff", N, 64, "single"), make_solver("diff", N, 64, "single")
    upload_iterate(a, [r[3] for r in rec], [r[4] for r in rec])
    ld = B + 3
    xb = torch.zeros((N + 1) * nx, ld, device=DEV)
    ub = torch.zeros(N * nu, ld, device=DEV)
    xb[:, :B] = t(np.stack([r[3] for r in rec]).reshape(B, -1).T)
    ub[:, :B] = t(np.stack([r[4] for r in rec]).reshape(B, -1).T)
    x0 = t(np.stack([r[0] for r in rec]).T)
    yref = t(np.stack([r[1] for r in rec]).transpose(1, 2, 0))
    We = t(np.stack([r[2] for r in rec]).T)
    for tick in range(2):
        outs = []
        for s in (a, b):
            st = torch.full((B,), -7, dtype=torch.int32, device=DEV)
            it = torch.zeros(B, dtype=torch.int32, device=DEV)
            res = torch.zeros(3, B, device=DEV)
            if s is a:
                s.solve(x0, yref, We=We, status=st, qp_iter=it, qp_res=res)
            else:
                s.solve_iterate(x0, yref, xb, ub, We=We, status=st, qp_iter=it, qp_res=res)
            outs.append((st, it, res))
        torch.cuda.synchronize()
        assert (outs[0][0] == 0).all()
        for u, v in zip(*outs):
            assert torch.equal(u, v)
        xv, uv, _ = a.state()
        assert torch.equal(xv.to_tensor()[:, :B], xb[:, :B])
        assert torch.equal(uv.to_tensor()[:, :B], ub[:, :B])
        assert not xb[:, B:].any() and not ub[:, B:].any()  # the padding columns are untouched


@pytest.mark.parametrize("ipm", sorted(IPMS))
@pytest.mark.parametrize("model", MODELS)
@pytest.mark.parametrize("resets", [False, True])
def test_run_closed_loop_matches_oracle(built, ipm, model, resets):
    """Batched run() + closed-loop plant on the GPU; the oracle replays the same per-tick inputs with its own
    fp64 warm-start chain (prepare -> sqp_rti -> post, NMPCNavControl*::run: no shift, x1 -> x0 carry of the
    vel-refs, NMPCNavControlDiff.cpp:168-172). With resets, every fifth robot is reset
    ({name}_acados_reset(capsule, 1), NMPCNavControlDiff.cpp:177-181) before the solves of ticks 3 and 8."""
    N, B, T = 20, 70, 12
    reset_mask = torch.from_numpy((np.arange(B) % 5 == 0).astype(np.uint8)).to(DEV)
    fl = make_fleet(model, B, seed=11)
    solver = make_solver(model, N, B, ipm)
    o = Oracle(model, N, rule="batched")
    _, _, cr = solver.state()
    cr.copy_from(t(fl["carried"]))
    pose, vel, steer, path, s = t(fl["pose"]), t(fl["vel"]), t(fl["steer"]), t(fl["path"]), t(fl["s"])
    steer_arg = steer if model == "tric" else None
    traj = torch.zeros(N + 1, 3, B, device=DEV)
    tlen = torch.zeros(B, dtype=torch.int32, device=DEV)
    cmd = torch.zeros(3, B, device=DEV)
    u0 = torch.zeros(solver.nu, B, device=DEV)
    status = torch.zeros(B, dtype=torch.int32, device=DEV)
    xbar = np.zeros((B, N + 1, o.nx))
    ubar = np.zeros((B, N, o.nu))
    for i in range(B):
        xbar[i], ubar[i] = o.iterate_create()
    carried = np.ascontiguousarray(fl["carried"].T, np.float64)
    solver.fleet_sim_step(path, s, pose, vel, steer_arg, None, None, traj, tlen, advance=False)
    worst = 0.0
    for tick in range(T):
        torch.cuda.synchronize()
        pose_h = np.ascontiguousarray(pose.cpu().numpy().T, np.float64)
        vel_h = np.ascontiguousarray(vel.cpu().numpy().T, np.float64)
        steer_h = np.ascontiguousarray(steer.cpu().numpy(), np.float64)
        traj_h = np.ascontiguousarray(traj.cpu().numpy().transpose(2, 0, 1), np.float64)
        tlen_h = np.ascontiguousarray(tlen.cpu().numpy(), np.int32)
        rs = reset_mask if resets and tick in (3, 8) else None
        solver.run(pose, vel, traj, steer=steer_arg, traj_len=tlen, reset=rs, cmd=cmd, u0=u0, status=status)
        nf, cmd_o, u0_o, st_o, _ = o.batch_tick(pose_h, vel_h, steer_h if model == "tric" else None, traj_h, tlen_h,
                                                None if rs is None else rs.cpu().numpy(), carried, xbar, ubar)
        torch.cuda.synchronize()
        assert nf == 0
        assert (status.cpu().numpy() == 0).all()
        eu = np.abs(u0.cpu().numpy().T - u0_o).max()
        ec = np.abs(cmd.cpu().numpy().T - cmd_o).max()
        worst = max(worst, eu)
        assert eu <= TOL_U, (tick, eu)
        assert ec <= TOL_U, (tick, ec)
        solver.fleet_sim_step(path, s, pose, vel, steer_arg, u0, status, traj, tlen, advance=True)
    assert np.isfinite(worst)


# bench-scale replays of every robot: tests/test_gpu_fleet.py
