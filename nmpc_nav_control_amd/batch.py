"""Batched solve path on the device: a thin Python owner of an ``nmpc_batch`` handle (libnmpc_amd.so).

Device memory and streams come from PyTorch (plumbing only); every array is an fp32 torch CUDA tensor in
the instance-minor ``[field][B]`` layout of include/nmpc_amd/nmpc_batch.h. All compute runs in the HIP
kernels of the library; there is no Python or CPU fallback.
"""
import ctypes

import torch

from ._lib import (KERNELS, MODEL_IDS, PLAN_MODES, REC_LAYOUTS, SCHEDULES, FleetRenew, FleetStats, LaunchPlan,
                   ModelParams, check, default_params, lib, model_dims)


def _ptr(t, dtype=None, shape=None, name="argument"):
    """Device pointer of a contiguous CUDA tensor, checked against the dtype and shape the kernel reads (a
    wrong dtype would be reinterpreted silently by the C ABI)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a device tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous tensor")
    if dtype is not None and t.dtype not in (dtype if isinstance(dtype, tuple) else (dtype,)):
        raise TypeError(f"{name}: expected dtype {dtype}, got {t.dtype}")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")
    return ctypes.c_void_p(t.data_ptr())


F32, I32, I64, U8 = torch.float32, torch.int32, torch.int64, (torch.uint8, torch.bool)


def _stream(stream):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class BatchSolver:
    """B independent OCP instances of one model, solved in lockstep on one GPU.

    ``solve`` is the batched ``{name}_acados_solve`` on caller-packed x0 / yref; ``run`` is the batched
    ``NMPCNavControl{Diff,Omni4,Tric}::run`` (pre-solve, SQP-RTI, post-solve) with the warm-start
    iterate and carried vel-ref states resident on the device between ticks.
    """

    fused_stats = True  # fleet_sim_step_renew accumulates the solve statistics in its own launch (nmpc_fleet_stats)

    def __init__(self, model, N, capacity, params=None, device="cuda", kernel=None, record_layout=None):
        self.model = model
        self.N = int(N)
        self.capacity = int(capacity)
        self.device = torch.device(device)
        self.params = params if params is not None else default_params(model, N)
        self.params.model = MODEL_IDS[model]
        self.params.N = self.N
        d = model_dims(model)
        self.nx, self.nu, self.ny, self.nbx, self.nbu = d["nx"], d["nu"], d["ny"], d["nbx"], d["nbu"]
        self._h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().nmpc_batch_create(ctypes.byref(self.params), self.capacity, ctypes.byref(self._h)),
                  "nmpc_batch_create")
        self.kernel = "team"
        if kernel is not None:
            self.set_kernel(kernel)
        if record_layout is not None:
            self.set_record_layout(record_layout)

    def set_record_layout(self, layout):
        """The team kernel's scratch record layout of this handle: 'auto' (the model's choice from this handle
        alone, fixed at create), 'wide' or 'split' (nmpc_batch_set_record_layout; diff has both, tric only split,
        omni4 only wide). Robots whose multipliers sit in the other layout start their next IPM cold."""
        check(lib().nmpc_batch_set_record_layout(self._h, REC_LAYOUTS[layout]), "nmpc_batch_set_record_layout")

    def plan_ex(self, B, mode="solve"):
        """The launch a call of B robots makes (nmpc_batch_plan_ex): dict with kernel ('team' / 'rowpar'),
        waves_per_robot, segments, record_layout ('wide' / 'split'), warm_tag and record_bytes. mode: 'solve',
        'run' or 'run_path'."""
        p = LaunchPlan()
        check(lib().nmpc_batch_plan_ex(self._h, int(B), PLAN_MODES[mode], ctypes.byref(p)), "nmpc_batch_plan_ex")
        return dict(kernel="rowpar" if p.kernel else "team", waves_per_robot=p.waves_per_robot, segments=p.segments,
                    record_layout="split" if p.record_layout else "wide", warm_tag=p.warm_tag,
                    record_bytes=p.record_bytes)

    def set_kernel(self, kernel):
        """'team' (16-lane team per robot): the only kernel."""
        check(lib().nmpc_batch_set_kernel(self._h, KERNELS[kernel]), "nmpc_batch_set_kernel")
        self.kernel = kernel

    def plan(self, B):
        """The kernel a solve / run launch of B robots takes (nmpc_batch_plan): (name, waves per robot, segments),
        name 'team' (k_sqp_rti_team) or 'rowpar' (k_sqp_rti_rowpar; segments 0 = its serial phases)."""
        k, w, sg = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().nmpc_batch_plan(self._h, int(B), ctypes.byref(k), ctypes.byref(w), ctypes.byref(sg)),
              "nmpc_batch_plan")
        return ("rowpar" if k.value else "team"), w.value, sg.value

    def set_schedule(self, mode):
        """Team placement of the team kernel: 'auto' (default), 'off', 'sorted' or 'interleaved'
        (include/nmpc_amd/nmpc_batch.h; no effect on any result)."""
        check(lib().nmpc_batch_set_schedule(self._h, SCHEDULES[mode]), "nmpc_batch_set_schedule")

    def close(self):
        if self._h:
            lib().nmpc_batch_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_params(self, params):
        check(lib().nmpc_batch_set_params(self._h, ctypes.byref(params)), "nmpc_batch_set_params")
        self.params = params

    def init_iterate(self, B=None, mode=0, stream=None):
        """mode 0: {name}_acados_create semantics (carried refs zeroed); mode 1: {name}_acados_reset (iterate
        zeroed, carried refs kept, as the per-robot reset mask)."""
        B = self.capacity if B is None else int(B)
        check(lib().nmpc_batch_init_iterate(self._h, B, int(mode), _stream(stream)), "nmpc_batch_init_iterate")

    def state(self):
        """Views of the resident device state: xbar [(N+1)*NX][cap], ubar [N*NU][cap], carried [NBX][cap]."""
        xb, ub, cr = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        stride = ctypes.c_int()
        check(lib().nmpc_batch_state(self._h, ctypes.byref(xb), ctypes.byref(ub), ctypes.byref(cr),
                                     ctypes.byref(stride)), "nmpc_batch_state")
        S = stride.value
        return (_DeviceView(xb.value, ((self.N + 1) * self.nx, S), self.device),
                _DeviceView(ub.value, (self.N * self.nu, S), self.device),
                _DeviceView(cr.value, (self.nbx, S), self.device))

    def warm_state(self):
        """Views of the IPM warm-start state (nmpc_batch_warm_state): per-robot flags [cap] (uint8) and the
        scratch records (bytes); with state() everything a solve reads from the handle."""
        w, sc, nb = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_size_t()
        check(lib().nmpc_batch_warm_state(self._h, ctypes.byref(w), ctypes.byref(sc), ctypes.byref(nb)),
              "nmpc_batch_warm_state")
        return (_DeviceView(w.value, (1, self.capacity), self.device, torch.uint8),
                _DeviceView(sc.value, (1, nb.value // 4), self.device))

    def forget_warm(self, mask=None, B=None, stream=None):
        """Cold IPM start at the next solve for the robots where mask != 0 (None: all of them); the iterate stays
        (nmpc_batch_forget_warm)."""
        B = self.capacity if B is None else int(B)
        check(lib().nmpc_batch_forget_warm(self._h, B, _ptr(mask, U8, (B,), "mask"), _stream(stream)),
              "nmpc_batch_forget_warm")

    def save_state(self):
        """Device copies of everything a solve reads from the handle (iterate, carried refs, warm start)."""
        return [v.to_tensor() for v in self.state() + self.warm_state()]

    def restore_state(self, saved):
        for v, t in zip(self.state() + self.warm_state(), saved):
            v.copy_from(t)

    def empty(self, *shape, dtype=torch.float32):
        return torch.empty(*shape, dtype=dtype, device=self.device)

    def solve(self, x0, yref, We=None, reset=None, u0=None, x1=None, xtraj=None, utraj=None, status=None,
              qp_iter=None, qp_res=None, stream=None):
        B = x0.shape[1]
        if not 0 <= B <= self.capacity:
            raise ValueError(f"batch {B} exceeds the capacity {self.capacity}")
        ny_in = yref.shape[1]
        N, nx, nu = self.N, self.nx, self.nu
        check(lib().nmpc_batch_solve(
            self._h, B, _ptr(x0, F32, (nx, B), "x0"), _ptr(yref, F32, (N + 1, ny_in, B), "yref"), ny_in,
            _ptr(We, F32, (nx, B), "We"), _ptr(reset, U8, (B,), "reset"), _ptr(u0, F32, (nu, B), "u0"),
            _ptr(x1, F32, (nx, B), "x1"), _ptr(xtraj, F32, ((N + 1) * nx, B), "xtraj"),
            _ptr(utraj, F32, (N * nu, B), "utraj"), _ptr(status, I32, (B,), "status"),
            _ptr(qp_iter, I32, (B,), "qp_iter"), _ptr(qp_res, F32, (3, B), "qp_res"), _stream(stream)),
            "nmpc_batch_solve")

    def solve_iterate(self, x0, yref, xbar, ubar, We=None, reset=None, status=None, qp_iter=None, qp_res=None,
                      stream=None):
        """nmpc_batch_solve with a caller-held iterate: xbar [(N+1)*NX][ld], ubar [N*NU][ld] are read and overwritten
        with the new iterate in place (nmpc_batch_solve_iterate). The IPM warm start still comes from the handle's
        slot i: keep instance i in slot i across calls, or call forget_warm after reordering."""
        B = x0.shape[1]
        if not 0 <= B <= self.capacity:
            raise ValueError(f"batch {B} exceeds the capacity {self.capacity}")
        ld = xbar.shape[1]
        if ubar.shape[1] != ld:
            raise ValueError("xbar and ubar need the same leading dimension")
        ny_in = yref.shape[1]
        N, nx, nu = self.N, self.nx, self.nu
        check(lib().nmpc_batch_solve_iterate(
            self._h, B, _ptr(x0, F32, (nx, B), "x0"), _ptr(yref, F32, (N + 1, ny_in, B), "yref"), ny_in,
            _ptr(We, F32, (nx, B), "We"), _ptr(reset, U8, (B,), "reset"), _ptr(xbar, F32, ((N + 1) * nx, ld), "xbar"),
            _ptr(ubar, F32, (N * nu, ld), "ubar"), ld, _ptr(status, I32, (B,), "status"),
            _ptr(qp_iter, I32, (B,), "qp_iter"), _ptr(qp_res, F32, (3, B), "qp_res"), _stream(stream)),
            "nmpc_batch_solve_iterate")

    def run(self, pose, vel, traj, steer=None, traj_len=None, reset=None, cmd=None, u0=None, status=None,
            qp_iter=None, qp_res=None, stream=None):
        B = pose.shape[1]
        if not 0 <= B <= self.capacity:
            raise ValueError(f"batch {B} exceeds the capacity {self.capacity}")
        check(lib().nmpc_batch_run(
            self._h, B, _ptr(pose, F32, (3, B), "pose"), _ptr(vel, F32, (3, B), "vel"),
            _ptr(steer, F32, (B,), "steer"), _ptr(traj, F32, (self.N + 1, 3, B), "traj"),
            _ptr(traj_len, I32, (B,), "traj_len"), _ptr(reset, U8, (B,), "reset"), _ptr(cmd, F32, (3, B), "cmd"),
            _ptr(u0, F32, (self.nu, B), "u0"), _ptr(status, I32, (B,), "status"),
            _ptr(qp_iter, I32, (B,), "qp_iter"), _ptr(qp_res, F32, (3, B), "qp_res"), _stream(stream)),
            "nmpc_batch_run")

    def run_path(self, pose, vel, segs, nseg, nearest_u, sample_period, is_holonomic=False, steer=None, reset=None,
                 traj_out=None, cmd=None, u0=None, status=None, qp_iter=None, qp_res=None, stream=None):
        """processFollowPath's getNextNPoses + run for B robots in one launch (nmpc_batch_run_path): segs
        float64 [B][S][16] (the nmpc_path_segment layout, nmpc_nav_control_amd.path.pack_paths), nseg int32
        [B], nearest_u float64 [B]; traj_out [N+1][3][B] receives the poses."""
        B = pose.shape[1]
        if not 0 <= B <= self.capacity:
            raise ValueError(f"batch {B} exceeds the capacity {self.capacity}")
        if segs.dim() != 3 or segs.shape[0] != B or segs.shape[2] != 16:
            raise ValueError(f"segs: expected shape ({B}, S, 16), got {tuple(segs.shape)}")
        check(lib().nmpc_batch_run_path(
            self._h, B, _ptr(pose, F32, (3, B), "pose"), _ptr(vel, F32, (3, B), "vel"),
            _ptr(steer, F32, (B,), "steer"), _ptr(segs, torch.float64, None, "segs"), segs.shape[1],
            _ptr(nseg, I32, (B,), "nseg"), _ptr(nearest_u, torch.float64, (B,), "nearest_u"), float(sample_period),
            1 if is_holonomic else 0, _ptr(reset, U8, (B,), "reset"),
            _ptr(traj_out, F32, (self.N + 1, 3, B), "traj_out"), _ptr(cmd, F32, (3, B), "cmd"),
            _ptr(u0, F32, (self.nu, B), "u0"), _ptr(status, I32, (B,), "status"),
            _ptr(qp_iter, I32, (B,), "qp_iter"), _ptr(qp_res, F32, (3, B), "qp_res"), _stream(stream)),
            "nmpc_batch_run_path")

    def fleet_sim_step(self, path, s, pose, vel, steer, u0, status, traj, traj_len, advance=True, stream=None):
        B = pose.shape[1]
        if not 0 <= B <= self.capacity:
            raise ValueError(f"batch {B} exceeds the capacity {self.capacity}")
        check(lib().nmpc_fleet_sim_step(
            self._h, B, _ptr(path, F32, (6, B), "path"), _ptr(s, F32, (B,), "s"), _ptr(pose, F32, (3, B), "pose"),
            _ptr(vel, F32, (3, B), "vel"), _ptr(steer, F32, (B,), "steer"), _ptr(u0, F32, (self.nu, B), "u0"),
            _ptr(status, I32, (B,), "status"), _ptr(traj, F32, (self.N + 1, 3, B), "traj"),
            _ptr(traj_len, I32, (B,), "traj_len"), int(bool(advance)), _stream(stream)), "nmpc_fleet_sim_step")


    def fleet_sim_step_renew(self, path, s, pose, vel, steer, u0, status, traj, traj_len, ev, ttl, reset, seed, start,
                             renew, stream=None, stats=None):
        """fleet_sim_step (advance) followed by the stationary loop's goal / path renewal (nmpc_fleet_sim_step_renew):
        ev, ttl int32 [B] in/out, reset uint8 [B] in (the flags the last solve ran with) / out (the next run's reset
        mask); renew: scenario.RENEW keys + kappa_max, speed (lo, hi). stats (optional): dict of device tensors the
        same launch accumulates the last solve's statistics into (nmpc_fleet_stats): qp_iter int32 [B] (in),
        iters_sum int64 [B], iters_max int32 [B], fail_cnt int64 [B], hist int64 [64], cold_cnt / cold_iters
        int64 [B]."""
        B = pose.shape[1]
        if not 0 <= B <= self.capacity:
            raise ValueError(f"batch {B} exceeds the capacity {self.capacity}")
        S = None
        if stats is not None:
            S = FleetStats(qp_iter=_ptr(stats["qp_iter"], I32, (B,), "qp_iter"),
                           iters_sum=_ptr(stats["iters_sum"], I64, (B,), "iters_sum"),
                           iters_max=_ptr(stats["iters_max"], I32, (B,), "iters_max"),
                           fail_cnt=_ptr(stats["fail_cnt"], I64, (B,), "fail_cnt"),
                           hist=_ptr(stats["hist"], I64, (64,), "hist"),
                           cold_cnt=_ptr(stats["cold_cnt"], I64, (B,), "cold_cnt"),
                           cold_iters=_ptr(stats["cold_iters"], I64, (B,), "cold_iters"))
        R = FleetRenew(seed=int(seed) & 0xFFFFFFFF, start=int(start), ttl_min=int(renew["ttl_min"]),
                       ttl_max=int(renew["ttl_max"]), goal_r_lo=renew["goal_r_lo"], goal_r_hi=renew["goal_r_hi"],
                       kappa_max=renew["kappa_max"], speed_lo=renew["speed"][0], speed_hi=renew["speed"][1],
                       len_lo=renew["len_lo"], len_hi=renew["len_hi"], pos_tol=renew["pos_tol"],
                       ang_tol=renew["ang_tol"], ev=_ptr(ev, I32, (B,), "ev"), ttl=_ptr(ttl, I32, (B,), "ttl"),
                       reset=_ptr(reset, U8, (B,), "reset"),
                       stats=ctypes.cast(ctypes.pointer(S), ctypes.c_void_p) if S is not None else None)
        check(lib().nmpc_fleet_sim_step_renew(
            self._h, B, _ptr(path, F32, (6, B), "path"), _ptr(s, F32, (B,), "s"), _ptr(pose, F32, (3, B), "pose"),
            _ptr(vel, F32, (3, B), "vel"), _ptr(steer, F32, (B,), "steer"), _ptr(u0, F32, (self.nu, B), "u0"),
            _ptr(status, I32, (B,), "status"), _ptr(traj, F32, (self.N + 1, 3, B), "traj"),
            _ptr(traj_len, I32, (B,), "traj_len"), ctypes.byref(R), _stream(stream)), "nmpc_fleet_sim_step_renew")


class _DeviceView:
    """Copy helpers for device memory owned by the library (no torch tensor aliases it)."""

    def __init__(self, addr, shape, device, dtype=torch.float32):
        self.addr, self.shape, self.device, self.dtype = addr, shape, device, dtype
        self.itemsize = torch.empty(0, dtype=dtype).element_size()

    def to_tensor(self):
        rows, S = self.shape
        out = torch.empty(rows, S, dtype=self.dtype, device=self.device)
        _memcpy(out.data_ptr(), self.addr, rows * S * self.itemsize)
        return out

    def copy_from(self, t):
        rows, S = self.shape
        t = t.to(device=self.device, dtype=self.dtype).contiguous()
        assert t.numel() == rows * S
        _memcpy(self.addr, t.data_ptr(), rows * S * self.itemsize)


def _memcpy(dst, src, nbytes):
    torch.cuda.synchronize()
    hip = _hip()
    rc = hip.hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), ctypes.c_size_t(nbytes), 3)  # DeviceToDevice
    if rc != 0:
        raise RuntimeError(f"hipMemcpy failed ({rc})")


_hip_lib = None


def _hip():
    global _hip_lib
    if _hip_lib is None:
        lib()  # libnmpc_amd pulls in libamdhip64
        _hip_lib = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
        _hip_lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return _hip_lib


__all__ = ["BatchSolver", "ModelParams", "default_params"]
