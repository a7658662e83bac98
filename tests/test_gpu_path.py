"""GPU parity of the batched path discretizer (nmpc_path_discretize, csrc/path_discretizer.hip) against the
fp64 oracle (oracle/path_oracle.c, PathDiscretizer.cpp:14-63) on the same segments.

Bar: x, y and every emit decision bit-exact (both sides run IEEE fp64 in the same operation order without
fused multiply-adds); theta within 1e-12 rad (the device and host atan2 may round the last ulp differently);
the fp32 output equals the fp64 output rounded. Then a path-following tick that never leaves the device
(discretize -> BatchSolver.run) against the oracle chain, with the SQP tolerance of test_gpu_parity.py.
"""
import math

import numpy as np
import pytest
import torch

from nmpc_nav_control_amd._lib import lib
from nmpc_nav_control_amd.batch import BatchSolver
from nmpc_nav_control_amd.path import PathDiscretizer, PathSegment, discretize, pack_paths
from oracle.oracle import Oracle, path_discretize
from tests.path_cases import edge_paths, random_paths

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def gpu_run(segs, nseg, nu, period, num_poses, holo):
    B = len(nseg)
    t64 = torch.empty((num_poses, 3, B), dtype=torch.float64, device=DEV)
    t32 = discretize(torch.from_numpy(np.ascontiguousarray(segs)).to(DEV), torch.from_numpy(nseg).to(DEV),
                     torch.from_numpy(nu).to(DEV), period, num_poses, holo, traj64=t64)
    torch.cuda.synchronize()
    return t64.permute(2, 0, 1).cpu().numpy(), t32.permute(2, 0, 1).cpu().numpy()


def check_parity(got, exp, names=None):
    for i in range(len(exp)):
        msg = names[i] if names else f"robot {i}"
        np.testing.assert_array_equal(got[i, :, :2], exp[i, :, :2], err_msg=msg)
        d = np.abs(np.angle(np.exp(1j * (got[i, :, 2] - exp[i, :, 2]))))
        assert d.max() <= 1e-12, (msg, d.max())


@pytest.mark.parametrize("holo", [False, True])
@pytest.mark.parametrize("period,num_poses", [(0.025, 41), (0.025, 61), (1.0, 8)])
def test_discretize_matches_oracle(built, period, num_poses, holo):
    segs, nseg, nu = random_paths(2000, seed=11 + num_poses)
    exp, _ = path_discretize(segs, nseg, nu, period, num_poses, holo)
    got, got32 = gpu_run(segs, nseg, nu, period, num_poses, holo)
    check_parity(got, exp)
    np.testing.assert_array_equal(got32, got.astype(np.float32))


def test_discretize_edge_cases(built):
    segs, nseg, nu, names = edge_paths()
    for holo in (False, True):
        exp, _ = path_discretize(segs, nseg, nu, 0.025, 41, holo)
        got, _ = gpu_run(segs, nseg, nu, 0.025, 41, holo)
        check_parity(got, exp, names)


def test_discretize_large_batch_properties(built):
    """65536 robots (the mixed-fleet size): finite output, oracle parity on a strided sample."""
    segs, nseg, nu = random_paths(65536 // 64, seed=5)
    segs, nseg, nu = np.tile(segs, (64, 1, 1)), np.tile(nseg, 64), np.tile(nu, 64)
    got, _ = gpu_run(segs, nseg, nu, 0.025, 41, False)
    assert np.isfinite(got).all()
    idx = np.arange(0, len(nseg), 997)
    exp, _ = path_discretize(segs[idx], nseg[idx], nu[idx], 0.025, 41, False)
    check_parity(got[idx], exp)
    # tiled robots are identical instances
    np.testing.assert_array_equal(got[: len(nseg) // 64], got[len(nseg) // 64: 2 * len(nseg) // 64])


def test_reference_mirror_getNextNPoses(built):
    pd = PathDiscretizer(0.025, 41)
    path = [PathSegment.line((0, 0), (1, 0), 0.5), PathSegment.arc(1, 0.5, 0.5, -math.pi / 2, 0.0, 0.5)]
    poses = pd.getNextNPoses(path, 0.2)
    assert len(poses) == 41
    segs, nseg = pack_paths([path])
    exp, _ = path_discretize(segs, nseg, np.array([0.2]), 0.025, 41, False)
    np.testing.assert_array_equal([[p.x, p.y] for p in poses], exp[0, :, :2])


def test_argument_errors(built):
    z = torch.zeros((4, 2, 16), dtype=torch.float64, device=DEV)
    n = torch.ones(4, dtype=torch.int32, device=DEV)
    u = torch.zeros(4, dtype=torch.float64, device=DEV)
    with pytest.raises(RuntimeError, match="num_poses"):
        discretize(z, n, u, 0.025, 0)
    with pytest.raises(RuntimeError, match="sample_period"):
        discretize(z, n, u, float("nan"), 4)
    assert lib().nmpc_path_discretize(0, None, 1, None, None, 0.025, 4, 0, None, None, None) == 0


def test_follow_path_tick_on_device_matches_oracle(built):
    """discretize -> BatchSolver.run (diff, N=40) on the device vs oracle discretize -> prepare -> sqp_rti."""
    N, B = 40, 256
    rng = np.random.default_rng(99)
    segs, nseg, nu = random_paths(B, seed=99, max_segs=4, reverse_frac=0.0)
    nu[:] = rng.uniform(0, 0.3, B)
    exp_traj, _ = path_discretize(segs, nseg, nu, 1 / 40, N + 1, False)
    # robots near their path start, heading along it
    pose = exp_traj[:, 0, :].copy()
    pose[:, :2] += rng.uniform(-0.1, 0.1, (B, 2))
    pose[:, 2] += rng.uniform(-0.2, 0.2, B)
    vel = np.zeros((B, 3))
    vel[:, 0] = rng.uniform(0.0, 0.5, B)
    pose32, vel32 = pose.astype(np.float32), vel.astype(np.float32)
    solver = BatchSolver("diff", N, B, device=DEV)
    traj = discretize(torch.from_numpy(segs).to(DEV), torch.from_numpy(nseg).to(DEV), torch.from_numpy(nu).to(DEV),
                      1 / 40, N + 1)
    u0 = torch.zeros((2, B), dtype=torch.float32, device=DEV)
    status = torch.zeros(B, dtype=torch.int32, device=DEV)
    solver.run(torch.from_numpy(pose32.T.copy()).to(DEV), torch.from_numpy(vel32.T.copy()).to(DEV), traj, u0=u0,
               status=status)
    torch.cuda.synchronize()
    u0 = u0.cpu().numpy().T
    assert (status.cpu().numpy() == 0).all()
    o = Oracle("diff", N, rule="batched")
    xb0, ub0 = o.iterate_create()
    err = 0.0
    for i in range(B):
        x0, yref, We = o.prepare(pose32[i].astype(np.float64), vel32[i].astype(np.float64), 0.0,
                                 exp_traj[i].astype(np.float32).astype(np.float64), np.zeros(o.nbx))
        st, _, xb, ub = o.sqp_rti(xb0, ub0, x0, yref, We)
        assert st == 0
        err = max(err, np.abs(u0[i] - ub[0]).max())
    assert err <= 1e-3, err


@pytest.mark.parametrize("holo", [False, True])
def test_run_path_one_launch_equals_two_launches(built, monkeypatch, holo):
    """nmpc_batch_run_path (getNextNPoses in the solve kernel: a path-following tick in one launch,
    NMPCNavControlROS.cpp:666-668 -> :713) against nmpc_path_discretize followed by nmpc_batch_run: the poses
    are bit-identical (both fp64 marches without contraction, path_march.hpp) and so is every output of the
    solve; over three ticks of warm-started solves (team kernel both ways)."""
    N, B = 40, 1000
    rng = np.random.default_rng(5)
    segs, nseg, nu = random_paths(B, seed=5, max_segs=4, reverse_frac=0.2)
    nu[:] = rng.uniform(0, 0.3, B)
    exp_traj, _ = path_discretize(segs, nseg, nu, 1 / 40, N + 1, holo)
    pose = exp_traj[:, 0, :].copy()
    pose[:, :2] += rng.uniform(-0.1, 0.1, (B, 2))
    pose[:, 2] += rng.uniform(-0.2, 0.2, B)
    vel = np.zeros((B, 3))
    vel[:, 0] = rng.uniform(0.0, 0.5, B)
    d = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).to(DEV, dt)  # noqa: E731
    P, V = d(pose.T), d(vel.T)
    S, NS, NU = d(segs, torch.float64), d(nseg, torch.int32), d(nu, torch.float64)
    # the same (team) kernel both ways: run_path always runs it, run would take the row-parallel kernel at this size
    monkeypatch.setenv("NMPC_AMD_ROWPAR_MAX", "0")
    two, one = BatchSolver("diff", N, B, device=DEV), BatchSolver("diff", N, B, device=DEV)
    monkeypatch.delenv("NMPC_AMD_ROWPAR_MAX")
    out = {k: [torch.zeros(r, B, device=DEV) for _ in range(2)] for k, r in (("u0", 2), ("cmd", 3))}
    st = [torch.zeros(B, dtype=torch.int32, device=DEV) for _ in range(2)]
    it = [torch.zeros(B, dtype=torch.int32, device=DEV) for _ in range(2)]
    traj_out = torch.zeros(N + 1, 3, B, device=DEV)
    for tick in range(3):
        traj = discretize(S, NS, NU, 1 / 40, N + 1, holo)
        two.run(P, V, traj, cmd=out["cmd"][0], u0=out["u0"][0], status=st[0], qp_iter=it[0])
        one.run_path(P, V, S, NS, NU, 1 / 40, holo, traj_out=traj_out, cmd=out["cmd"][1], u0=out["u0"][1],
                     status=st[1], qp_iter=it[1])
        torch.cuda.synchronize()
        assert torch.equal(traj_out, traj), tick
        for k in ("u0", "cmd"):
            assert torch.equal(out[k][0], out[k][1]), (tick, k)
        assert torch.equal(st[0], st[1]) and torch.equal(it[0], it[1]) and (st[0] == 0).all(), tick
