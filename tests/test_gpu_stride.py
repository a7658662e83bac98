"""nmpc_batch_solve_iterate with a caller leading dimension ld != the handle's capacity: the
scratch planes (DZ plane, the row-parallel kernel's dummy blocks) follow the handle's allocation, so a solve of
robots [0, B) with any ld >= B leaves every other robot's records, DZ entries and warm-start flag untouched, and
gives the same result as nmpc_batch_solve on the handle's own iterate. The capsule shim calls with ld = n and a
power-of-two capacity (acados_shim.cpp), which is the ld < capacity case."""
import numpy as np
import pytest
import torch

from helpers import oracle_closed_loop

from nmpc_nav_control_amd._lib import default_params
from nmpc_nav_control_amd.batch import BatchSolver

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
CAP = 64


def t(a, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device=DEV, dtype=dtype)


def make(monkeypatch, model, N, kernel):
    env = {} if kernel == "rowpar" else {"NMPC_AMD_ROWPAR_MAX": 0, "NMPC_AMD_SPLIT_MAX": 0}
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    h = BatchSolver(model, N, CAP, params=default_params(model, N))
    for k in env:
        monkeypatch.delenv(k)
    return h


@pytest.mark.parametrize("kernel", ["rowpar", "team"])
@pytest.mark.parametrize("ld", [3, 5, 200])
def test_solve_iterate_ld_leaves_other_slots(built, monkeypatch, kernel, ld):
    model, N, B = "diff", 20, 3
    o, rec = oracle_closed_loop(model, N, CAP, 2)
    nx, nu = o.nx, o.nu
    x0 = t(np.stack([r[0] for r in rec]).T)
    yref = t(np.stack([r[1] for r in rec]).transpose(1, 2, 0))
    We = t(np.stack([r[2] for r in rec]).T)
    X0 = t(np.stack([r[3] for r in rec]).reshape(CAP, -1).T)
    U0 = t(np.stack([r[4] for r in rec]).reshape(CAP, -1).T)
    h, ref = make(monkeypatch, model, N, kernel), make(monkeypatch, model, N, kernel)
    for s in (h, ref):
        xv, uv, _ = s.state()
        xv.copy_from(X0)
        uv.copy_from(U0)
        s.solve(x0, yref, We=We)  # every slot warm: records and flags written for all CAP robots
    torch.cuda.synchronize()
    warm_v, scr_v = h.warm_state()
    warm_before, scr_before = warm_v.to_tensor().clone(), scr_v.to_tensor().clone()
    assert int(warm_before[0, B:].sum()) > 0  # the check below covers warm slots

    # robots [0, B) through the caller-held iterate with leading dimension ld
    xv, uv, _ = h.state()
    xb = torch.zeros((N + 1) * nx, ld, device=DEV)
    ub = torch.zeros(N * nu, ld, device=DEV)
    xb[:, :B] = xv.to_tensor()[:, :B]
    ub[:, :B] = uv.to_tensor()[:, :B]
    st = torch.full((B,), -7, dtype=torch.int32, device=DEV)
    h.solve_iterate(x0[:, :B].contiguous(), yref[:, :, :B].contiguous(), xb, ub, We=We[:, :B].contiguous(),
                    status=st)
    # the twin handle: the same solve on its own iterate
    u0 = torch.zeros(nu, B, device=DEV)
    xt = torch.zeros((N + 1) * nx, B, device=DEV)
    st_ref = torch.full((B,), -7, dtype=torch.int32, device=DEV)
    ref.solve(x0[:, :B].contiguous(), yref[:, :, :B].contiguous(), We=We[:, :B].contiguous(), u0=u0, xtraj=xt,
              status=st_ref)
    torch.cuda.synchronize()
    assert (st == 0).all() and (st_ref == 0).all()
    assert torch.equal(ub[:nu, :B], u0) and torch.equal(xb[:, :B], xt)
    assert not ub[:, B:].any() and not xb[:, B:].any()  # nothing written past the B columns of the caller's block

    warm_after, scr_after = warm_v.to_tensor(), scr_v.to_tensor()
    assert torch.equal(warm_after[0, B:], warm_before[0, B:])
    # scratch: the lane records [robot][stage][16][RS], then the DZ plane [robot][stage][16]
    rec_floats = scr_before.shape[1]
    per_stage_dz = 16
    dz_floats = CAP * (N + 1) * per_stage_dz
    # RS from the layout (team_scratch_floats): CAP (N+1) 16 (RS + 1) + 256 x 4 x 16 (RS + 1) + 64
    rs = (rec_floats - 64) // (CAP * (N + 1) * 16 + 256 * 4 * 16) - 1
    assert (rs + 1) * (CAP * (N + 1) * 16 + 256 * 4 * 16) + 64 == rec_floats
    rec_end = CAP * (N + 1) * 16 * rs
    per_robot = (N + 1) * 16 * rs
    assert rec_end + dz_floats <= rec_floats
    sb, sa = scr_before[0], scr_after[0]
    assert torch.equal(sa[B * per_robot:rec_end], sb[B * per_robot:rec_end]), "another robot's records changed"
    dz0 = rec_end + B * (N + 1) * per_stage_dz
    assert torch.equal(sa[dz0:rec_end + dz_floats], sb[dz0:rec_end + dz_floats]), "another robot's DZ plane changed"


def test_warm_rule_reports_the_effective_parameters(built, monkeypatch):
    """nmpc_batch_warm_rule gives the rule the kernels apply, env overrides included (the capsule shim
    mirrored the flags from its own parameter copy, which the overrides do not change)."""
    import ctypes

    from nmpc_nav_control_amd._lib import lib

    def rule(h):
        w, wm, im = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        assert lib().nmpc_batch_warm_rule(h._h, ctypes.byref(w), ctypes.byref(wm), ctypes.byref(im)) == 0
        return w.value, wm.value, im.value

    assert rule(BatchSolver("diff", 20, 8)) == (1, 12, 50)
    assert rule(BatchSolver("omni4", 20, 8)) == (1, 50, 50)  # qp_warm_iter_max 0: any converged solve
    monkeypatch.setenv("NMPC_AMD_WARM_ITER_MAX", "5")
    monkeypatch.setenv("NMPC_AMD_WARM", "0")
    h = BatchSolver("diff", 20, 8)
    monkeypatch.delenv("NMPC_AMD_WARM_ITER_MAX")
    monkeypatch.delenv("NMPC_AMD_WARM")
    assert rule(h) == (0, 5, 50)
