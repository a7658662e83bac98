"""Split launches (KArgs::split, small batches: one 256-lane block per robot, P0's integrations spread over the
block's 16 rows (4 waves, stages row, row + 16, ..., joined by a block barrier), the serial initial-iterate pass
reading its stage inputs from LDS) against the unsplit team launch of the
same inputs (NMPC_AMD_SPLIT_MAX=0 at handle creation), in every kernel mode: solve (the capsule ABI's path,
NMPCNavControlDiff.cpp:142), run with caller poses, and run_path (getNextNPoses in the launch). Both launches run
the same fp32 IPM from the same linearisation, so they agree to fp32 rounding (the RK4 code is the same function
inlined in two places); every launch is also checked against the fp64 oracle by the parity tests, which run at
split batch sizes."""
import numpy as np
import pytest
import torch

from helpers import oracle_closed_loop

from nmpc_nav_control_amd._lib import default_params
from nmpc_nav_control_amd.batch import BatchSolver
from nmpc_nav_control_amd.path import discretize
from oracle.oracle import path_discretize
from tests.path_cases import random_paths

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 1e-5


def t(a, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device=DEV, dtype=dtype)


def handle(monkeypatch, model, N, cap, layout=None, **env):
    """A handle created under the launch-choice overrides `env` (read at creation), with the team kernel's record
    layout `layout` (None: the model's own choice)."""
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    h = BatchSolver(model, N, cap, params=default_params(model, N), record_layout=layout)
    for k in env:
        monkeypatch.delenv(k)
    return h


LAYOUTS = {"diff": ("wide", "split"), "omni4": ("wide",), "tric": ("split",)}  # the team kernel's record layouts


def pair(monkeypatch, model, N, cap):
    """(split, unsplit) team-kernel handles of the same model and horizon (the row-parallel kernel, which takes
    these batch sizes by default, switched off)."""
    return (handle(monkeypatch, model, N, cap, NMPC_AMD_ROWPAR_MAX=0),
            handle(monkeypatch, model, N, cap, NMPC_AMD_ROWPAR_MAX=0, NMPC_AMD_SPLIT_MAX=0))


def close(u, v):
    return float((u.float() - v.float()).abs().max()) if u.numel() else 0.0


@pytest.mark.parametrize("model", ["diff", "omni4", "tric"])
@pytest.mark.parametrize("N,B", [(80, 13), (40, 1), (2, 5)])
def test_split_solve_equals_unsplit(built, monkeypatch, model, N, B):
    o, rec = oracle_closed_loop(model, N, B, 2)
    nx, nu = o.nx, o.nu
    sp, un = pair(monkeypatch, model, N, 64)
    x0 = t(np.stack([r[0] for r in rec]).T)
    yref = t(np.stack([r[1] for r in rec]).transpose(1, 2, 0))
    We = t(np.stack([r[2] for r in rec]).T)
    for s in (sp, un):
        xv, uv, _ = s.state()
        X, U = xv.to_tensor(), uv.to_tensor()
        X[:, :B] = t(np.stack([r[3] for r in rec]).reshape(B, -1).T)
        U[:, :B] = t(np.stack([r[4] for r in rec]).reshape(B, -1).T)
        xv.copy_from(X)
        uv.copy_from(U)
    for tick in range(3):  # a cold tick, then warm-started multipliers
        outs = []
        for s in (sp, un):
            o_ = dict(u0=torch.zeros(nu, B, device=DEV), xtraj=torch.zeros((N + 1) * nx, B, device=DEV),
                      status=torch.full((B,), -7, dtype=torch.int32, device=DEV),
                      qp_iter=torch.zeros(B, dtype=torch.int32, device=DEV))
            s.solve(x0, yref, We=We, u0=o_["u0"], xtraj=o_["xtraj"], status=o_["status"], qp_iter=o_["qp_iter"])
            outs.append(o_)
        torch.cuda.synchronize()
        assert (outs[0]["status"] == 0).all() and torch.equal(outs[0]["status"], outs[1]["status"]), tick
        assert close(outs[0]["u0"], outs[1]["u0"]) <= TOL, tick
        assert close(outs[0]["xtraj"], outs[1]["xtraj"]) <= TOL, tick
        assert (outs[0]["qp_iter"] - outs[1]["qp_iter"]).abs().max() <= 1, tick


@pytest.mark.parametrize("holo", [False, True])
def test_split_run_and_run_path_equal_unsplit(built, monkeypatch, holo):
    """run (caller poses, traj_len shorter than the horizon for some robots) and run_path, split against
    unsplit, over three warm-started ticks; run_path's poses come out of the launch bit-identical."""
    N, B = 40, 24
    rng = np.random.default_rng(9)
    segs, nseg, nu = random_paths(B, seed=9, max_segs=4, reverse_frac=0.2)
    nu[:] = rng.uniform(0, 0.3, B)
    exp_traj, _ = path_discretize(segs, nseg, nu, 1 / 40, N + 1, holo)
    pose = exp_traj[:, 0, :].copy()
    pose[:, :2] += rng.uniform(-0.1, 0.1, (B, 2))
    pose[:, 2] += rng.uniform(-0.2, 0.2, B)
    vel = np.zeros((B, 3))
    vel[:, 0] = rng.uniform(0.0, 0.5, B)
    P, V = t(pose.T), t(vel.T)
    S, NS, NU = t(segs, torch.float64), t(nseg, torch.int32), t(nu, torch.float64)
    tlen = t(np.where(np.arange(B) % 3 == 0, N // 2, N + 1), torch.int32)
    handles = {"run": pair(monkeypatch, "diff", N, B), "path": pair(monkeypatch, "diff", N, B)}
    for tick in range(3):
        traj = discretize(S, NS, NU, 1 / 40, N + 1, holo)
        res = {}
        for kind, hs in handles.items():
            res[kind] = []
            for h in hs:
                o_ = dict(u0=torch.zeros(2, B, device=DEV), cmd=torch.zeros(3, B, device=DEV),
                          status=torch.full((B,), -7, dtype=torch.int32, device=DEV),
                          traj=torch.zeros(N + 1, 3, B, device=DEV))
                if kind == "run":
                    h.run(P, V, traj, traj_len=tlen, cmd=o_["cmd"], u0=o_["u0"], status=o_["status"])
                else:
                    h.run_path(P, V, S, NS, NU, 1 / 40, holo, traj_out=o_["traj"], cmd=o_["cmd"], u0=o_["u0"],
                               status=o_["status"])
                res[kind].append(o_)
        torch.cuda.synchronize()
        for kind, (a, b) in res.items():
            assert (a["status"] == 0).all() and torch.equal(a["status"], b["status"]), (tick, kind)
            assert close(a["u0"], b["u0"]) <= TOL, (tick, kind)
            assert close(a["cmd"], b["cmd"]) <= TOL, (tick, kind)
        assert torch.equal(res["path"][0]["traj"], traj) and torch.equal(res["path"][1]["traj"], traj), tick


# ---- the row-parallel kernel (k_sqp_rti_rowpar, the default for batches up to 1024 robots) against the team
# kernel: the same IPM and stopping rule, with sums over stages in another order (4 rows), so the two agree to
# fp32 rounding amplified by the IPM's exit (an iteration more or less); both are checked against the oracle by
# the parity tests
TOL_RP = 3e-4


@pytest.mark.parametrize("layout", ["wide", "split"])
@pytest.mark.parametrize("model", ["diff", "omni4", "tric"])
@pytest.mark.parametrize("N,B", [(80, 13), (40, 64), (2, 5), (1, 3)])
def test_rowpar_solve_matches_team(built, monkeypatch, model, N, B, layout):
    """The row-parallel kernel (wide records) against the team kernel in each record layout the model has (diff:
    both, ADVICE r04: the split planes are the mixed fleet's default for diff)."""
    if layout not in LAYOUTS[model]:
        pytest.skip(f"{model}'s team kernel has no {layout} records")
    o, rec = oracle_closed_loop(model, N, B, 2)
    nx, nu = o.nx, o.nu
    rp = handle(monkeypatch, model, N, 64)
    tm = handle(monkeypatch, model, N, 64, layout=layout, NMPC_AMD_ROWPAR_MAX=0, NMPC_AMD_SPLIT_MAX=0)
    assert tm.plan_ex(B)["kernel"] == "team" and tm.plan_ex(B)["record_layout"] == layout
    assert rp.plan_ex(B)["kernel"] == "rowpar" or N == 1
    x0 = t(np.stack([r[0] for r in rec]).T)
    yref = t(np.stack([r[1] for r in rec]).transpose(1, 2, 0))
    We = t(np.stack([r[2] for r in rec]).T)
    for s in (rp, tm):
        xv, uv, _ = s.state()
        X, U = xv.to_tensor(), uv.to_tensor()
        X[:, :B] = t(np.stack([r[3] for r in rec]).reshape(B, -1).T)
        U[:, :B] = t(np.stack([r[4] for r in rec]).reshape(B, -1).T)
        xv.copy_from(X)
        uv.copy_from(U)
    for tick in range(3):
        outs = []
        for s in (rp, tm):
            o_ = dict(u0=torch.zeros(nu, B, device=DEV), xtraj=torch.zeros((N + 1) * nx, B, device=DEV),
                      status=torch.full((B,), -7, dtype=torch.int32, device=DEV),
                      qp_iter=torch.zeros(B, dtype=torch.int32, device=DEV))
            s.solve(x0, yref, We=We, u0=o_["u0"], xtraj=o_["xtraj"], status=o_["status"], qp_iter=o_["qp_iter"])
            outs.append(o_)
        torch.cuda.synchronize()
        assert (outs[0]["status"] == 0).all() and (outs[1]["status"] == 0).all(), tick
        assert close(outs[0]["u0"], outs[1]["u0"]) <= TOL_RP, (tick, close(outs[0]["u0"], outs[1]["u0"]))
        assert close(outs[0]["xtraj"], outs[1]["xtraj"]) <= TOL_RP, tick
        assert (outs[0]["qp_iter"] - outs[1]["qp_iter"]).abs().max() <= 3, tick


def test_rowpar_run_matches_team(built, monkeypatch):
    """run mode (pose / velocity packing, reference unwrap and padding with traj_len shorter than the horizon, the
    diff terminal-weight hack, carry and command) over warm-started ticks: row-parallel against the team kernel in
    both of diff's record layouts (wide, and the split planes the mixed fleet takes)."""
    N, B = 40, 24
    rng = np.random.default_rng(11)
    segs, nseg, nu = random_paths(B, seed=11, max_segs=4, reverse_frac=0.2)
    nu[:] = rng.uniform(0, 0.3, B)
    exp_traj, _ = path_discretize(segs, nseg, nu, 1 / 40, N + 1, False)
    pose = exp_traj[:, 0, :].copy()
    pose[:, :2] += rng.uniform(-0.1, 0.1, (B, 2))
    vel = np.zeros((B, 3))
    vel[:, 0] = rng.uniform(0.0, 0.5, B)
    P, V = t(pose.T), t(vel.T)
    S, NS, NU = t(segs, torch.float64), t(nseg, torch.int32), t(nu, torch.float64)
    tlen = t(np.where(np.arange(B) % 3 == 0, 1, np.where(np.arange(B) % 3 == 1, N // 2, N + 1)), torch.int32)
    hs = (handle(monkeypatch, "diff", N, B), handle(monkeypatch, "diff", N, B, "wide", NMPC_AMD_ROWPAR_MAX=0),
          handle(monkeypatch, "diff", N, B, "split", NMPC_AMD_ROWPAR_MAX=0))
    assert [h.plan_ex(B, "run")["record_layout"] for h in hs[1:]] == ["wide", "split"]
    for tick in range(4):
        traj = discretize(S, NS, NU, 1 / 40, N + 1, False)
        res = []
        for h in hs:
            o_ = dict(u0=torch.zeros(2, B, device=DEV), cmd=torch.zeros(3, B, device=DEV),
                      status=torch.full((B,), -7, dtype=torch.int32, device=DEV))
            h.run(P, V, traj, traj_len=tlen, cmd=o_["cmd"], u0=o_["u0"], status=o_["status"])
            res.append(o_)
        torch.cuda.synchronize()
        a = res[0]
        for j, b in enumerate(res[1:]):
            assert (a["status"] == 0).all() and (b["status"] == 0).all(), (tick, j)
            assert close(a["u0"], b["u0"]) <= TOL_RP, (tick, j, close(a["u0"], b["u0"]))
            assert close(a["cmd"], b["cmd"]) <= TOL_RP, (tick, j)
            ca, cb = hs[0].state()[2].to_tensor(), hs[1 + j].state()[2].to_tensor()
            assert close(ca[:, :B], cb[:, :B]) <= TOL_RP, (tick, j)
        # the two team layouts: the same arithmetic on differently placed records, bit for bit
        assert torch.equal(res[1]["u0"], res[2]["u0"]) and torch.equal(res[1]["cmd"], res[2]["cmd"]), tick


# ---- the column-form M block's per-launch constant rows ------------------------------------------------
# gconst_load (team_common.hpp) takes the state-independent rows of [B A] (rows >= NGV: the theta, wheel and
# reference rows, functions of dt and the model parameters only, which are per launch: KParams) from the lanes of
# each wave's FIRST team and uses them for all four teams of the wave. The checker build lib/mrow/ (Makefile: the row
# form for every model, every row read from the robot's own lanes) solves the same fleet; robots in different
# states in every wave must give the product's results to fp32 rounding.

@pytest.mark.parametrize("model", ["diff", "omni4", "tric"])
def test_constant_rows_per_launch(built, tmp_path, model):
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mrow = os.path.join(root, "nmpc_nav_control_amd", "lib", "mrow", "libnmpc_amd.so")
    assert os.path.exists(mrow), "lib/mrow/libnmpc_amd.so is built by the csrc Makefile (all)"
    N, B = 40, 64
    layout = "split" if model == "tric" else "wide"
    outs = {}
    for name, lib in (("product", None), ("mrow", mrow)):
        env = dict(os.environ)
        env.pop("NMPC_AMD_LIB", None)
        if lib:
            env["NMPC_AMD_LIB"] = lib
        out = str(tmp_path / f"{name}.npz")
        r = subprocess.run([sys.executable, os.path.join(root, "tests", "team_probe.py"), model, str(N), str(B), "6",
                            layout, out], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        outs[name] = np.load(out)
    a, b = outs["product"], outs["mrow"]
    assert str(b["lib"]).endswith("mrow/libnmpc_amd.so")
    assert (a["status"] == 0).all() and (b["status"] == 0).all()
    # robots in different states share each wave (the oracle closed loop's fleet after 6 ticks)
    x0 = a["xtraj"][:3]
    assert np.unique(np.round(x0, 3), axis=1).shape[1] == B
    du = float(np.abs(a["utraj"] - b["utraj"]).max())
    dx = float(np.abs(a["xtraj"] - b["xtraj"]).max())
    print(f"{model}: column form vs row form: u {du:.2e} x {dx:.2e}")
    assert du <= 3e-4 and dx <= 3e-4, (du, dx)
