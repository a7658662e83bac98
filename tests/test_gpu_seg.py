"""The segmented row-parallel kernel (k_sqp_rti_rowpar SEG: the horizon's Riccati sweeps split over S segments that
run at the same time, joined by a master recursion over the segment boundaries; DESIGN.md "Segmented Riccati").

The segmented direction equals the serial one up to rounding (tools/seg_emu.py), so every segment count S that
divides N must give the serial row-parallel kernel's result (NMPC_AMD_SEG=0) to fp32 rounding amplified by the IPM's
exit, and both must match the fp64 oracle within the parity tolerance. S = 1 runs the segmented code with one
segment (absolute-form rhs, the stopping rule's separate adjoint pass, no master)."""
import numpy as np
import pytest
import torch

from helpers import oracle_closed_loop

from nmpc_nav_control_amd._lib import default_params
from nmpc_nav_control_amd.batch import BatchSolver

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL_SEG = 3e-4  # against the serial kernel (as tests/test_gpu_split.py's row-parallel vs team tolerance)
TOL = 1e-3      # against the oracle


def t(a, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device=DEV, dtype=dtype)


def handle(monkeypatch, model, N, cap, seg, rowpar_max=None):
    monkeypatch.setenv("NMPC_AMD_SEG", str(seg))
    if rowpar_max is not None:
        monkeypatch.setenv("NMPC_AMD_ROWPAR_MAX", str(rowpar_max))
    h = BatchSolver(model, N, cap, params=default_params(model, N))
    monkeypatch.delenv("NMPC_AMD_SEG")
    if rowpar_max is not None:
        monkeypatch.delenv("NMPC_AMD_ROWPAR_MAX")
    return h


def close(u, v):
    return float((u.float() - v.float()).abs().max()) if u.numel() else 0.0


def run_pair(monkeypatch, model, N, B, seg, ticks=3, cap=64, rowpar_max=None):
    """Solve the same oracle closed-loop inputs with the segmented and the serial row-parallel kernel for `ticks`
    ticks (the first cold, then warm-started); returns per tick (seg outputs, serial outputs) and the oracle's u0."""
    o, rec = oracle_closed_loop(model, N, B, 2)
    nx, nu = o.nx, o.nu
    hs = [handle(monkeypatch, model, N, cap, seg, rowpar_max), handle(monkeypatch, model, N, cap, 0, rowpar_max)]
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
    # the oracle's solution of the first tick (same inputs and iterate)
    u0_o = np.stack([o.sqp_rti(r[3], r[4], r[0], r[1], r[2])[3][0] for r in rec])
    out = []
    for _ in range(ticks):
        res = []
        for s in hs:
            d = dict(u0=torch.zeros(nu, B, device=DEV), xtraj=torch.zeros((N + 1) * nx, B, device=DEV),
                     status=torch.full((B,), -7, dtype=torch.int32, device=DEV),
                     qp_iter=torch.zeros(B, dtype=torch.int32, device=DEV),
                     qp_res=torch.zeros(3, B, device=DEV))
            s.solve(x0, yref, We=We, u0=d["u0"], xtraj=d["xtraj"], status=d["status"], qp_iter=d["qp_iter"],
                    qp_res=d["qp_res"])
            res.append(d)
        torch.cuda.synchronize()
        out.append(res)
    return out, u0_o


@pytest.mark.parametrize("model", ["diff", "omni4", "tric"])
# (S <= 8 on four waves: the sensitivities on waves 2-3 beside the factorisation; S = 10, 16: on the factorisation's
# own rows, DESIGN.md "Segmented Riccati")
@pytest.mark.parametrize("N,seg", [(80, 5), (80, 8), (80, 2), (80, 10), (80, 16), (40, 4), (40, 1), (20, 4), (2, 2),
                                   (1, 1)])
def test_seg_matches_serial_and_oracle(built, monkeypatch, model, N, seg):
    B = 9
    out, u0_o = run_pair(monkeypatch, model, N, B, seg)
    for tick, (sg, se) in enumerate(out):
        assert (sg["status"] == 0).all() and (se["status"] == 0).all(), (tick, sg["status"], se["status"])
        assert close(sg["u0"], se["u0"]) <= TOL_SEG, (tick, close(sg["u0"], se["u0"]))
        assert close(sg["xtraj"], se["xtraj"]) <= TOL_SEG, tick
        assert (sg["qp_iter"] - se["qp_iter"]).abs().max() <= 3, (tick, sg["qp_iter"], se["qp_iter"])
        # reported exit residuals: the stationarity residual comes from the separate adjoint pass
        assert (sg["qp_res"][0] >= 0).all() and (sg["qp_res"][0] <= 1e-3).all(), sg["qp_res"][0]
    err = float(np.abs(out[0][0]["u0"].cpu().numpy().T - u0_o).max())
    assert err <= TOL, err


@pytest.mark.parametrize("model", ["diff", "tric"])
def test_seg_one_wave_per_robot(built, monkeypatch, model):
    """Batches above 256 robots run two waves (segments on the first wave's 4 rows) per robot: 300 robots at N = 40,
    4 segments against the serial phases (one wave per robot)."""
    out, u0_o = run_pair(monkeypatch, model, 40, 300, 4, ticks=2, cap=300, rowpar_max=1024)
    for tick, (sg, se) in enumerate(out):
        assert (sg["status"] == 0).all() and (se["status"] == 0).all(), tick
        assert close(sg["u0"], se["u0"]) <= TOL_SEG, (tick, close(sg["u0"], se["u0"]))
    assert float(np.abs(out[0][0]["u0"].cpu().numpy().T - u0_o).max()) <= TOL


@pytest.mark.parametrize("model", ["diff", "tric"])
def test_hybrid_launch_matches_plain(built, monkeypatch, model):
    """NMPC_AMD_HYBRID=H: in a team-kernel launch the robots whose last IPM count was >= H run the segmented kernel
    on a second stream while the team kernel takes the rest (DESIGN.md "Hybrid launch"). Every robot's result equals
    the plain team launch's to the row-parallel kernel's tolerance, over ticks whose split changes with the counts.
    The hybrid launch is an A/B build only (-DNMPC_HYBRID: `make -C nmpc_nav_control_amd/csrc variant VARNAME=hybrid
    VARIANT_FLAGS=-DNMPC_HYBRID`, run with NMPC_AMD_LIB pointing at it); the product library leaves it out."""
    from nmpc_nav_control_amd._lib import lib
    if b"hybrid" not in lib().nmpc_version():
        pytest.skip("A/B build only: the product library has no hybrid launch")
    N, B = 40, 600
    o, rec = oracle_closed_loop(model, N, B, 2)
    nx, nu = o.nx, o.nu
    monkeypatch.setenv("NMPC_AMD_HYBRID", "8")
    monkeypatch.setenv("NMPC_AMD_SPLIT_MAX", "0")
    monkeypatch.setenv("NMPC_AMD_ROWPAR_MAX", "0")  # the team kernel (600 robots would run the segmented kernel)
    hy = BatchSolver(model, N, B, params=default_params(model, N))
    monkeypatch.delenv("NMPC_AMD_HYBRID")
    pl = BatchSolver(model, N, B, params=default_params(model, N))
    monkeypatch.delenv("NMPC_AMD_SPLIT_MAX")
    monkeypatch.delenv("NMPC_AMD_ROWPAR_MAX")
    x0 = t(np.stack([r[0] for r in rec]).T)
    yref = t(np.stack([r[1] for r in rec]).transpose(1, 2, 0))
    We = t(np.stack([r[2] for r in rec]).T)
    for s in (hy, pl):
        xv, uv, _ = s.state()
        xv.copy_from(t(np.stack([r[3] for r in rec]).reshape(B, -1).T))
        uv.copy_from(t(np.stack([r[4] for r in rec]).reshape(B, -1).T))
    u0_o = np.stack([o.sqp_rti(r[3], r[4], r[0], r[1], r[2])[3][0] for r in rec])
    for tick in range(3):
        res = []
        for s in (hy, pl):
            d = dict(u0=torch.zeros(nu, B, device=DEV), status=torch.full((B,), -7, dtype=torch.int32, device=DEV),
                     qp_iter=torch.zeros(B, dtype=torch.int32, device=DEV))
            s.solve(x0, yref, We=We, u0=d["u0"], status=d["status"], qp_iter=d["qp_iter"])
            res.append(d)
        torch.cuda.synchronize()
        a, b = res
        assert (a["status"] == 0).all() and (b["status"] == 0).all(), tick
        assert close(a["u0"], b["u0"]) <= TOL_SEG, (tick, close(a["u0"], b["u0"]))
        if tick == 0:
            assert float(np.abs(a["u0"].cpu().numpy().T - u0_o).max()) <= TOL
            assert int((b["qp_iter"] >= 8).sum()) > 0  # the next ticks split the batch


def test_plan_defaults(built):
    """nmpc_batch_plan: the kernel each launch size takes by default -- one capsule (N = 80) on four waves with 8
    horizon segments, up to 1024 robots (N = 40) the segmented kernel on two waves each (4 segments, all on the
    first wave), larger batches the team kernel."""
    h1 = BatchSolver("diff", 80, 1, params=default_params("diff", 80))
    assert h1.plan(1) == ("rowpar", 4, 8)
    h = BatchSolver("diff", 40, 4096, params=default_params("diff", 40))
    assert h.plan(256) == ("rowpar", 4, 5)
    assert h.plan(1024) == ("rowpar", 2, 4)
    assert h.plan(1025)[0] == "team" and h.plan(4096)[0] == "team"
    ht = BatchSolver("tric", 60, 64, params=default_params("tric", 60))
    assert ht.plan(64) == ("rowpar", 4, 6)
    ho = BatchSolver("omni4", 40, 512, params=default_params("omni4", 40))
    assert ho.plan(256)[0] == "rowpar" and ho.plan(300)[0] == "team"  # 357 registers: one wave per SIMD
