"""The committed golden fixtures in front of the device: the kernels' bar is the data in
tests/golden/*.npz, not the live oracle, so a change to oracle/nmpc_oracle.c cannot move it unnoticed.

Each fixture holds one closed-loop tick of B robots (tests/golden/make_golden.py): the solve inputs x0, yref, W_e,
the warm iterate (xbar, ubar) and the fp64 oracle's SQP-RTI result (xbar_new, ubar_new, status). The test loads them
onto the device, runs one batched solve with every kernel a launch of that size can take (the row-parallel kernel,
the default at these batch sizes, and the team kernel with its split launch off), both IPM direction rules, and
compares with the committed result: u0 and the predicted states within 1e-3, the later inputs (warm-start data,
flat cost in u mid-horizon) within 5e-3, the tolerances of tests/test_gpu_parity.py. test_oracle.py holds the same
fixtures against the oracle on the CPU, so oracle, fixtures and device are pinned to each other.
"""
import glob
import os

import numpy as np
import pytest
import torch

from nmpc_nav_control_amd._lib import default_params
from nmpc_nav_control_amd.batch import BatchSolver

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "*_N*.npz")))
TOL_U, TOL_X, TOL_UTRAJ = 1e-3, 1e-3, 5e-3
DEV = torch.device("cuda:0")
IPMS = {"single": 1, "mehrotra": 0}


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device=DEV, dtype=torch.float32)


@pytest.mark.parametrize("kernel", ["default", "team"])
@pytest.mark.parametrize("ipm", sorted(IPMS))
@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p)[:-4] for p in FIXTURES])
def test_device_solve_matches_committed_fixture(built, monkeypatch, path, ipm, kernel):
    d = np.load(path)
    model, N = str(d["meta"][0]), int(d["meta"][1])
    B = d["x0"].shape[0]
    assert (d["status"] == 0).all()
    if kernel == "team":  # the team kernel at this size: neither the row-parallel kernel nor the split launch
        monkeypatch.setenv("NMPC_AMD_ROWPAR_MAX", "0")
        monkeypatch.setenv("NMPC_AMD_SPLIT_MAX", "0")
    prm = default_params(model, N)
    prm.qp_ipm = IPMS[ipm]
    s = BatchSolver(model, N, 64, params=prm)
    plan = s.plan_ex(B)
    if kernel == "team":
        assert plan["kernel"] == "team"
    elif ipm == "single":  # the row-parallel kernel covers the single-direction rule (Mehrotra: the split launch)
        assert plan["kernel"] == "rowpar"
    nx, nu = s.nx, s.nu
    xv, uv, _ = s.state()
    X, U = xv.to_tensor(), uv.to_tensor()
    X[:, :B] = t(d["xbar"].reshape(B, -1).T)
    U[:, :B] = t(d["ubar"].reshape(B, -1).T)
    xv.copy_from(X)
    uv.copy_from(U)
    xtraj = torch.zeros((N + 1) * nx, B, device=DEV)
    utraj = torch.zeros(N * nu, B, device=DEV)
    status = torch.full((B,), -7, dtype=torch.int32, device=DEV)
    s.solve(t(d["x0"].T), t(d["yref"].transpose(1, 2, 0)), We=t(d["We"].T), xtraj=xtraj, utraj=utraj, status=status)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    xg = xtraj.cpu().numpy().T.reshape(B, N + 1, nx)
    ug = utraj.cpu().numpy().T.reshape(B, N, nu)
    eu0 = np.abs(ug[:, 0] - d["ubar_new"][:, 0]).max()
    ex = np.abs(xg - d["xbar_new"]).max()
    eu = np.abs(ug - d["ubar_new"]).max()
    print(f"{os.path.basename(path)} {ipm} {kernel}: u0 {eu0:.2e} x {ex:.2e} u {eu:.2e}")
    assert eu0 <= TOL_U and ex <= TOL_X and eu <= TOL_UTRAJ, (eu0, ex, eu)
