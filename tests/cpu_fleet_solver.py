"""CPU stand-in for BatchSolver, for the multi-process tests (TEST INFRASTRUCTURE: it runs the fp64 oracle).

It has the methods nmpc_nav_control_amd.fleet.Fleet calls (nu, state, run, fleet_sim_step, set_schedule) on
CPU torch tensors in the same [field][B] layouts, so the world-size-2 gloo tests drive the shipping
Fleet / FleetNode / CommandGather loop of bench.py with only the solver swapped:
  run            -> oracle batch_tick (prepare, SQP-RTI, post: NMPCNavControl*::run);
  fleet_sim_step -> the harness plant / reference step of fleet_sim.hip, restated in numpy (fp64 math on the
                    stored fp32 values; the CPU tests compare runs of this same code, never with the GPU).
"""
import numpy as np
import torch

from helpers import plant_measure
from nmpc_nav_control_amd.scenario import arc_pose, renew_step
from oracle.oracle import Oracle


class _View:
    def __init__(self, arr):
        self.arr = arr  # float64 numpy [rows][B]

    def to_tensor(self):
        return torch.from_numpy(self.arr.astype(np.float32))

    def copy_from(self, t):
        self.arr[...] = t.detach().cpu().numpy().astype(np.float64).reshape(self.arr.shape)


class OracleFleetSolver:
    kernel = "oracle"

    def __init__(self, model, N, capacity, device="cpu"):
        self.model, self.N, self.B = model, N, capacity
        self.o = Oracle(model, N, rule="batched")
        self.nu, self.nx = self.o.nu, self.o.nx
        xb, ub = self.o.iterate_create()
        self.xbar = np.repeat(xb[None], capacity, axis=0)
        self.ubar = np.repeat(ub[None], capacity, axis=0)
        self.carried = np.zeros((capacity, self.o.nbx))

    def set_schedule(self, mode):
        pass

    def state(self):
        B = self.B
        return (_View(self.xbar.reshape(B, -1).T.copy()), _View(self.ubar.reshape(B, -1).T.copy()),
                _CarriedView(self))

    def run(self, pose, vel, traj, steer=None, traj_len=None, reset=None, cmd=None, u0=None, status=None,
            qp_iter=None, qp_res=None, stream=None):
        h = lambda t: np.ascontiguousarray(t.numpy().T, np.float64)  # noqa: E731
        B = pose.shape[1]
        tl = traj_len.numpy().astype(np.int32) if traj_len is not None else np.full(B, self.N + 1, np.int32)
        st = np.ascontiguousarray(steer.numpy(), np.float64) if steer is not None else None
        rs = reset.numpy() if reset is not None else None
        nf, cmd_o, u0_o, st_o, it_o = self.o.batch_tick(
            h(pose), h(vel), st, np.ascontiguousarray(traj.numpy().transpose(2, 0, 1), np.float64), tl, rs,
            self.carried[:B], self.xbar[:B], self.ubar[:B], nthreads=1)
        if cmd is not None:
            cmd.copy_(torch.from_numpy(np.where((st_o == 0)[:, None], cmd_o, 0.0).T.astype(np.float32)))
        if u0 is not None:
            u0.copy_(torch.from_numpy(u0_o.T.astype(np.float32)))
        if status is not None:
            status.copy_(torch.from_numpy(st_o.astype(np.int32)))
        if qp_iter is not None:
            qp_iter.copy_(torch.from_numpy(it_o.astype(np.int32)))

    def fleet_sim_step_renew(self, path, s, pose, vel, steer, u0, status, traj, traj_len, ev, ttl, reset, seed, start,
                             renew, stream=None):
        """k_fleet_sim with its renewal record (scenario.renew_step after the plant step)."""
        self.fleet_sim_step(path, s, pose, vel, steer, u0, status, traj, traj_len, advance=True,
                            renew=(ev, ttl, reset, seed, start, renew))

    def fleet_sim_step(self, path, s, pose, vel, steer, u0, status, traj, traj_len, advance=True, stream=None,
                       renew=None):
        """numpy restatement of k_fleet_sim (fleet_sim.hip): plant RK4 step with the applied u0, measurement,
        goal / path renewal (optional), reference regeneration (arc path or goal pose)."""
        o, N = self.o, self.N
        P = path.numpy().astype(np.float64)
        B = pose.shape[1]
        ps, vs = pose.numpy(), vel.numpy()
        for i in range(B):
            if advance and (status is None or int(status[i]) == 0):
                x0, _, _ = o.prepare(ps[:, i].astype(np.float64), vs[:, i].astype(np.float64),
                                     float(steer[i]) if steer is not None else 0.0,
                                     np.zeros((1, 3)), self.carried[i])
                u = u0[:, i].numpy().astype(np.float64)
                for j in range(o.nbx):
                    x0[self._idxbx(j)] = self.carried[i, j] - u[j] * o.prm.dt_ctrl
                xn, _, _ = o.rk4(x0, u, o.prm.dt_ctrl)
                v3, stn = plant_measure(self.model, xn, o.prm.p)
                ps[:, i] = xn[:3]
                vs[:, i] = v3
                if steer is not None:
                    steer[i] = stn
            if renew is not None:
                ev, ttl, reset, seed, start, rn = renew
                Pn, sn, evn, ttln = P, s.numpy(), ev.numpy(), ttl.numpy()
                reset[i] = renew_step(self.model, Pn, sn, ps[:, i].astype(np.float64), evn, ttln, seed, start, i,
                                      renew={k: rn[k] for k in ("ttl_min", "ttl_max", "goal_r_lo", "goal_r_hi",
                                                                 "len_lo", "len_hi", "pos_tol", "ang_tol")},
                                      speed=rn["speed"])
                path[:, i] = torch.from_numpy(P[:, i].astype(np.float32))
                P[:, i] = path[:, i].numpy().astype(np.float64)
            if P[5, i] < 0:
                traj[0, :, i] = torch.from_numpy(P[:3, i].astype(np.float32))
                if traj_len is not None:
                    traj_len[i] = 1
                continue
            sc = float(s[i])
            for _ in range(3):
                q = arc_pose(P, i, sc)
                sc += (ps[0, i] - q[0]) * np.cos(q[2]) + (ps[1, i] - q[1]) * np.sin(q[2])
                sc = min(max(sc, 0.0), P[5, i])
            sc = max(sc, float(s[i]))
            s[i] = sc
            spacing = abs(P[4, i]) * o.prm.dt_ctrl
            for k in range(N + 1):
                traj[k, :, i] = torch.from_numpy(arc_pose(P, i, min(sc + (k + 1) * spacing, P[5, i]))
                                                 .astype(np.float32))
            if traj_len is not None:
                traj_len[i] = N + 1

    def _idxbx(self, j):
        return list(self.o.prm.idxbx)[j]


class _CarriedView:
    def __init__(self, solver):
        self.s = solver

    def to_tensor(self):
        return torch.from_numpy(self.s.carried.T.astype(np.float32).copy())

    def copy_from(self, t):
        self.s.carried[...] = t.detach().cpu().numpy().astype(np.float64).T
