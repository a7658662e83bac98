"""Tail hand-off (KArgs::hand_cap): an unsplit team launch stops every team that is still iterating at the top of
IPM iteration hand_cap and the row-parallel tail launch (k_sqp_rti_rowpar_tail, four waves per robot) finishes those
robots from the records, the DZ plane and the IPM scalars the team left ("Tail hand-off").

The robot's QP, its stopping rule and its iteration count are the same as without the hand-off; the tail runs the
row-parallel kernel's arithmetic (sums over stages in another order), so the results agree with the team kernel's
to fp32 rounding amplified by the IPM exit, the tolerance of the row-parallel-vs-team tests (test_gpu_split.py).
Every hand-off path is also covered by the oracle replays of test_gpu_fleet.py, which run the default cap."""
import numpy as np
import pytest
import torch

from helpers import oracle_closed_loop

from nmpc_nav_control_amd._lib import default_params
from nmpc_nav_control_amd.batch import BatchSolver
from nmpc_nav_control_amd.fleet import Fleet
from nmpc_nav_control_amd.path import discretize
from oracle.oracle import path_discretize
from tests.path_cases import random_paths

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 3e-4
SEED = 20250824


def t(a, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device=DEV, dtype=dtype)


def handle(monkeypatch, model, N, cap, hand, grid=None):
    monkeypatch.setenv("NMPC_AMD_HAND_CAP", str(hand))
    if grid is not None:
        monkeypatch.setenv("NMPC_AMD_HAND_GRID", str(grid))
    h = BatchSolver(model, N, cap, params=default_params(model, N))
    monkeypatch.delenv("NMPC_AMD_HAND_CAP")
    if grid is not None:
        monkeypatch.delenv("NMPC_AMD_HAND_GRID")
    return h


def close(u, v):
    return float((u.float() - v.float()).abs().max()) if u.numel() else 0.0


@pytest.mark.parametrize("model,N,hand,grid", [("diff", 40, 12, None), ("diff", 40, 3, 64), ("omni4", 40, 6, None),
                                               ("tric", 60, 6, None)])
def test_handoff_run_matches_team(built, monkeypatch, model, N, hand, grid):
    """The bench's closed loop (run mode, renewals with controller resets) at B = 1024 (an unsplit team launch):
    after 12 ticks, three ticks solved from the same state with and without the hand-off. grid 64 makes the tail
    loop over a list longer than its grid."""
    B = 1024
    monkeypatch.setenv("NMPC_AMD_HAND_CAP", "0")
    f = Fleet(model, B, N, SEED + 7, DEV)
    monkeypatch.delenv("NMPC_AMD_HAND_CAP")
    team = f.solver
    tail = handle(monkeypatch, model, N, B, hand, grid)
    for _ in range(12):
        f.tick()
    handed = 0
    for tick in range(3):
        torch.cuda.synchronize()
        saved = team.save_state()
        outs = []
        for h in (tail, team):  # the team handle last: its post-solve state carries the loop on
            h.restore_state(saved)
            f.solver = h
            f.solve()
            torch.cuda.synchronize()
            outs.append(dict(u0=f.u0.clone(), cmd=f.cmd.clone(), status=f.status.clone(), it=f.qp_iter.clone(),
                             xbar=h.state()[0].to_tensor()[:, :B].clone(),
                             carried=h.state()[2].to_tensor()[:, :B].clone(),
                             warm=h.warm_state()[0].to_tensor()[:B].clone()))
        a, b = outs
        assert (b["status"] == 0).all() and torch.equal(a["status"], b["status"]), tick
        assert close(a["u0"], b["u0"]) <= TOL, (tick, close(a["u0"], b["u0"]))
        assert close(a["cmd"], b["cmd"]) <= TOL, tick
        assert close(a["xbar"], b["xbar"]) <= TOL, tick
        assert close(a["carried"], b["carried"]) <= TOL, tick
        assert (a["it"] - b["it"]).abs().max() <= 3, tick
        assert (a["warm"] != b["warm"]).float().mean() <= 0.01, tick
        handed += int((b["it"] >= hand).sum())
        f.advance()
    assert handed >= 3, handed  # the tail ran


def test_handoff_solve_matches_team(built, monkeypatch):
    """solve mode (the capsule ABI's caller x0 / yref / W_e) at B = 300, cold then warm-started ticks."""
    model, N, B = "diff", 40, 300
    o, rec = oracle_closed_loop(model, N, B, 2)
    nx, nu = o.nx, o.nu
    hs = (handle(monkeypatch, model, N, 512, 3), handle(monkeypatch, model, N, 512, 0))
    x0 = t(np.stack([r[0] for r in rec]).T)
    yref = t(np.stack([r[1] for r in rec]).transpose(1, 2, 0))
    We = t(np.stack([r[2] for r in rec]).T)
    for s in hs:
        xv, uv, _ = s.state()
        X, U = xv.to_tensor(), uv.to_tensor()
        X[:, :B] = t(np.stack([r[3] for r in rec]).reshape(B, -1).T)
        U[:, :B] = t(np.stack([r[4] for r in rec]).reshape(B, -1).T)
        xv.copy_from(X)
        uv.copy_from(U)
    for tick in range(3):
        outs = []
        for s in hs:
            o_ = dict(u0=torch.zeros(nu, B, device=DEV), xtraj=torch.zeros((N + 1) * nx, B, device=DEV),
                      status=torch.full((B,), -7, dtype=torch.int32, device=DEV),
                      qp_iter=torch.zeros(B, dtype=torch.int32, device=DEV),
                      qp_res=torch.zeros(3, B, device=DEV))
            s.solve(x0, yref, We=We, u0=o_["u0"], xtraj=o_["xtraj"], status=o_["status"], qp_iter=o_["qp_iter"],
                    qp_res=o_["qp_res"])
            outs.append(o_)
        torch.cuda.synchronize()
        a, b = outs
        assert (a["status"] == 0).all() and (b["status"] == 0).all(), tick
        assert int((b["qp_iter"] >= 3).sum()) > 0, tick
        assert close(a["u0"], b["u0"]) <= TOL, (tick, close(a["u0"], b["u0"]))
        assert close(a["xtraj"], b["xtraj"]) <= TOL, tick
        assert (a["qp_iter"] - b["qp_iter"]).abs().max() <= 3, tick
        # the tail writes the exit residuals of its robots: the stopping rule's res_ineq held as in the team launch
        assert torch.isfinite(a["qp_res"]).all(), tick
        assert float(a["qp_res"][1].max()) <= max(1e-6, float(b["qp_res"][1].max())), tick


def test_handoff_run_path_matches_team(built, monkeypatch):
    """run_path (getNextNPoses fused into the team launch): the handed-off robots finish in the tail, whose run-mode
    epilogue (carry, inverse kinematics, command) is the same for both run modes."""
    N, B = 40, 300
    rng = np.random.default_rng(13)
    segs, nseg, nu = random_paths(B, seed=13, max_segs=4, reverse_frac=0.2)
    nu[:] = rng.uniform(0, 0.3, B)
    exp_traj, _ = path_discretize(segs, nseg, nu, 1 / 40, N + 1, False)
    pose = exp_traj[:, 0, :].copy()
    pose[:, :2] += rng.uniform(-0.1, 0.1, (B, 2))
    pose[:, 2] += rng.uniform(-0.2, 0.2, B)
    vel = np.zeros((B, 3))
    vel[:, 0] = rng.uniform(0.0, 0.5, B)
    P, V = t(pose.T), t(vel.T)
    S, NS, NU = t(segs, torch.float64), t(nseg, torch.int32), t(nu, torch.float64)
    hs = (handle(monkeypatch, "diff", N, B, 3), handle(monkeypatch, "diff", N, B, 0))
    traj_exp = discretize(S, NS, NU, 1 / 40, N + 1, False)
    for tick in range(3):
        res = []
        for h in hs:
            o_ = dict(u0=torch.zeros(2, B, device=DEV), cmd=torch.zeros(3, B, device=DEV),
                      status=torch.full((B,), -7, dtype=torch.int32, device=DEV),
                      it=torch.zeros(B, dtype=torch.int32, device=DEV), traj=torch.zeros(N + 1, 3, B, device=DEV))
            h.run_path(P, V, S, NS, NU, 1 / 40, False, traj_out=o_["traj"], cmd=o_["cmd"], u0=o_["u0"],
                       status=o_["status"], qp_iter=o_["it"])
            res.append(o_)
        torch.cuda.synchronize()
        a, b = res
        assert (a["status"] == 0).all() and (b["status"] == 0).all(), tick
        assert int((b["it"] >= 3).sum()) > 0, tick
        assert close(a["u0"], b["u0"]) <= TOL, (tick, close(a["u0"], b["u0"]))
        assert close(a["cmd"], b["cmd"]) <= TOL, tick
        assert torch.equal(a["traj"], traj_exp) and torch.equal(b["traj"], traj_exp), tick


def test_handoff_list_is_cleared(built, monkeypatch):
    """Consecutive launches on one handle (the list and its counters are reset by the tail's last block): a launch
    in which nothing is handed off still returns every robot's result, and repeated identical launches agree."""
    model, N, B = "diff", 40, 300
    o, rec = oracle_closed_loop(model, N, B, 1)
    h = handle(monkeypatch, model, N, B, 2)
    x0 = t(np.stack([r[0] for r in rec]).T)
    yref = t(np.stack([r[1] for r in rec]).transpose(1, 2, 0))
    saved = h.save_state()
    outs = []
    for rep in range(3):
        h.restore_state(saved)
        u0 = torch.zeros(2, B, device=DEV)
        st = torch.full((B,), -7, dtype=torch.int32, device=DEV)
        it = torch.zeros(B, dtype=torch.int32, device=DEV)
        h.solve(x0, yref, u0=u0, status=st, qp_iter=it)
        torch.cuda.synchronize()
        assert (st == 0).all() and int((it >= 2).sum()) > 0, rep
        outs.append(u0)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])
