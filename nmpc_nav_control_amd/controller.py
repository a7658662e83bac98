"""Per-robot controllers mirroring the reference's L3 wrappers over the acados-compatible C ABI.

NMPCNavControl{Diff,Omni4,Tric} here follow include/nmpc_nav_control/NMPCNavControl{,Diff,Omni4,Tric}.h and
src/nmpc_nav_control/NMPCNavControl{,Diff,Omni4,Tric}.cpp call for call: the constructor creates the capsule
and sets parameters, bounds and weights through ``ocp_nlp_*`` (e.g. NMPCNavControlDiff.cpp:6-74); ``run``
packs x0 / yref, applies the diff terminal-weight hack, calls ``{name}_acados_solve`` and post-processes
(:82-175); ``reset_mpc`` calls ``{name}_acados_reset(capsule, 1)`` (:177-181). The solve itself runs on the
GPU through libnmpc_amd.so. Error behaviour matches processCreateStatus / processAcadosStatus
(NMPCNavControl.cpp:5-23): a non-zero status raises RuntimeError.
"""
import ctypes
import math
from dataclasses import dataclass

import numpy as np

from ._lib import MODEL_IDS, MODEL_NAMES, CodegenDesc, lib, model_dims, solver_lib


@dataclass
class Pose:
    x: float = 0.0
    y: float = 0.0
    theta: float = 0.0


@dataclass
class Vel:
    v: float = 0.0
    vn: float = 0.0
    w: float = 0.0


@dataclass
class CmdVelDiff:
    v: float = 0.0
    w: float = 0.0


@dataclass
class CmdVelOmni4:
    v: float = 0.0
    vn: float = 0.0
    w: float = 0.0


@dataclass
class CmdVelTric:
    v: float = 0.0
    alpha: float = 0.0


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class NMPCNavControl:
    """Base class (NMPCNavControl.h:21-59)."""

    model = None

    def __init__(self, dt, N=None):
        self.dt_ = float(dt)
        d = model_dims(self.model)
        self.nx, self.nu, self.ny, self.nbx, self.nbu, self.np = (d[k] for k in ("nx", "nu", "ny", "nbx", "nbu",
                                                                                   "np"))
        self._name = MODEL_NAMES[self.model]
        L = lib()
        self._L = L
        self._S = S = solver_lib(self._name)  # the generated per-model ABI
        self._capsule = getattr(S, f"{self._name}_acados_create_capsule")()
        if N is None:
            status = getattr(S, f"{self._name}_acados_create")(self._capsule)
        else:
            # a horizon other than the baked one needs its time steps (acados create_with_discretization):
            # uniform steps of the codegen length
            steps = (ctypes.c_double * int(N))(*([self._codegen_dt()] * int(N)))
            status = getattr(S, f"{self._name}_acados_create_with_discretization")(self._capsule, int(N), steps)
        self.processCreateStatus(status)
        self.N = self._dims_N()
        c = self._capsule.contents
        self._cfg, self._dims, self._in, self._out, self._solver = (c.nlp_config, c.nlp_dims, c.nlp_in,
                                                                    ctypes.cast(c.nlp_out, ctypes.c_void_p),
                                                                    c.nlp_solver)
        self.x0 = np.zeros(self.nx)
        self.yref = np.zeros((self.N + 1, self.ny))
        self.u0 = np.zeros(self.nu)
        self.status = 0
        self.kkt_res = 0.0
        self.cpu_time = 0.0

    def _codegen_dt(self):
        """Step of the shipped codegen configuration (tf / N = 1 / freq, scripts/diff/common.py:6-9)."""
        d = CodegenDesc()
        self._L.nmpc_codegen_default(MODEL_IDS[self.model], ctypes.byref(d))
        return d.tf / d.N

    def _dims_N(self):
        class Dims(ctypes.Structure):
            _fields_ = [("impl", ctypes.c_void_p), ("N", ctypes.c_int)]
        return ctypes.cast(self._capsule.contents.nlp_dims, ctypes.POINTER(Dims)).contents.N

    def __del__(self):
        try:
            getattr(self._S, f"{self._name}_acados_free")(self._capsule)
            getattr(self._S, f"{self._name}_acados_free_capsule")(self._capsule)
        except Exception:
            pass

    # NMPCNavControl.h:40-41
    def getHorizon(self):
        return self.N

    def getDeltaTime(self):
        return self.dt_

    # NMPCNavControl.cpp:5-23
    @staticmethod
    def processCreateStatus(create_status):
        if create_status != 0:
            raise RuntimeError(f"acados_create() returned status {create_status}.")

    @staticmethod
    def processAcadosStatus(acados_status):
        if acados_status != 0:
            raise RuntimeError(f"acados_solve() returned status {acados_status}.")
        return True

    # NMPCNavControl.cpp:25-31
    @staticmethod
    def unwrapAngle(current, previous):
        delta = current - previous
        if delta > math.pi:
            current -= 2 * math.pi
        elif delta < -math.pi:
            current += 2 * math.pi
        return current

    # ---- acados C interface helpers ---------------------------------------------------------------------
    def _cset(self, stage, field, arr):
        a = np.ascontiguousarray(arr, np.float64)
        rc = self._L.ocp_nlp_constraints_model_set(self._cfg, self._dims, self._in, self._out, stage,
                                                   field.encode(), a.ctypes.data_as(ctypes.c_void_p))
        if rc != 0:
            raise RuntimeError(f"ocp_nlp_constraints_model_set({stage}, {field}) failed")

    def _wset(self, stage, field, arr):
        a = np.ascontiguousarray(arr, np.float64)
        rc = self._L.ocp_nlp_cost_model_set(self._cfg, self._dims, self._in, stage, field.encode(),
                                            a.ctypes.data_as(ctypes.c_void_p))
        if rc != 0:
            raise RuntimeError(f"ocp_nlp_cost_model_set({stage}, {field}) failed")

    def _out_get(self, stage, field, n):
        a = np.zeros(n)
        self._L.ocp_nlp_out_get(self._cfg, self._dims, self._out, stage, field.encode(),
                                a.ctypes.data_as(ctypes.c_void_p))
        return a

    def out_set(self, stage, field, arr):
        a = np.ascontiguousarray(arr, np.float64)
        self._L.ocp_nlp_out_set(self._cfg, self._dims, self._out, stage, field.encode(),
                                a.ctypes.data_as(ctypes.c_void_p))

    def solver_opts_set(self, field, value):
        """ocp_nlp_solver_opts_set(config, capsule->nlp_opts, field, &value) for the int fields "qp_warm_start"
        (0: HPIPM's cold start every solve, the reference's generated default; 1, acados' primal-only warm start,
        starts cold too; 2: the capsule's multiplier warm start) and "qp_iter_max"."""
        v = ctypes.c_int(int(value))
        self._L.ocp_nlp_solver_opts_set(self._cfg, self._capsule.contents.nlp_opts, field.encode(), ctypes.byref(v))

    def qp_iter(self):
        """IPM iterations of the last solve (ocp_nlp_get "qp_iter")."""
        n = ctypes.c_int()
        self._L.ocp_nlp_get(self._solver, b"qp_iter", ctypes.byref(n))
        return n.value

    def iterate(self):
        xs = np.stack([self._out_get(k, "x", self.nx) for k in range(self.N + 1)])
        us = np.stack([self._out_get(k, "u", self.nu) for k in range(self.N)])
        return xs, us

    def _setup(self, p, x_min, x_max, u_min, u_max, W_diag):
        """Constructor body shared by the three wrappers (NMPCNavControlDiff.cpp:14-73)."""
        self.p = np.asarray(p, np.float64)
        self.W = np.diag(np.asarray(W_diag[: self.ny], np.float64))
        self.W_e = np.diag(np.asarray(W_diag[: self.nx], np.float64))
        for i in range(self.N):
            rc = getattr(self._S, f"{self._name}_acados_update_params")(self._capsule, i, _dp(self.p), self.np)
            if rc != 0:
                raise RuntimeError("update_params failed")
        for i in range(1, self.N + 1):
            self._cset(i, "lbx", x_min)
            self._cset(i, "ubx", x_max)
        for i in range(self.N):
            self._cset(i, "lbu", u_min)
            self._cset(i, "ubu", u_max)
        for i in range(self.N):
            self._wset(i, "W", self.W.flatten(order="F"))
        self._wset(self.N, "W", self.W_e.flatten(order="F"))

    def _pack_refs(self, robot_pose, traj_ref):
        """Unwrap and pad the reference (NMPCNavControlDiff.cpp:104-124)."""
        previous_theta = robot_pose.theta
        it = iter(traj_ref)
        for i in range(self.N + 1):
            nxt = next(it, None)
            if nxt is not None:
                self.yref[i, 0] = nxt.x
                self.yref[i, 1] = nxt.y
                self.yref[i, 2] = self.unwrapAngle(nxt.theta, previous_theta)
                previous_theta = self.yref[i, 2]
            else:
                self.yref[i, :3] = self.yref[i - 1, :3]
        for i in range(self.N + 1):
            self._wset(i, "yref", self.yref[i, : (self.nx if i == self.N else self.ny)])

    def _solve(self):
        status = getattr(self._S, f"{self._name}_acados_solve")(self._capsule)
        self.processAcadosStatus(status)
        self.status = status
        self.kkt_res = self._capsule.contents.nlp_out.contents.inf_norm_res
        t = ctypes.c_double()
        self._L.ocp_nlp_get(self._solver, b"time_tot", ctypes.byref(t))
        self.cpu_time = t.value * 1000.0
        self.u0 = self._out_get(0, "u", self.nu)
        return self.cpu_time

    def reset_mpc(self):
        getattr(self._S, f"{self._name}_acados_reset")(self._capsule, 1)
        return True


class NMPCNavControlDiff(NMPCNavControl):
    """NMPCNavControlDiff.h / .cpp"""

    model = "diff"

    def __init__(self, dt, dist_b, tau_v, v_max, a_max, W_diag, N=None):
        super().__init__(dt, N)
        self._setup([dist_b, tau_v], [-v_max] * 2, [v_max] * 2, [-a_max] * 2, [a_max] * 2, W_diag)

    def directKinematrics(self, v, w):
        return v - 0.5 * self.p[0] * w, v + 0.5 * self.p[0] * w

    def inverseKinematrics(self, vl, vr):
        return (vr + vl) / 2.0, (vr - vl) / self.p[0]

    def run(self, robot_pose, robot_vel, traj_ref, robot_vel_ref):
        """NMPCNavControlDiff.cpp:82-175. Returns (True, cpu_time_ms); fills robot_vel_ref."""
        if not isinstance(robot_vel_ref, CmdVelDiff):
            raise RuntimeError("Invalid command velocity type passed to run method.")
        self.x0[0:3] = (robot_pose.x, robot_pose.y, robot_pose.theta)
        self.x0[3], self.x0[4] = self.directKinematrics(robot_vel.v, robot_vel.w)
        self._cset(0, "lbx", self.x0)
        self._cset(0, "ubx", self.x0)
        self._pack_refs(robot_pose, traj_ref)
        N = self.N
        hack = np.array_equal(self.yref[N, :3], self.yref[N - 1, :3])
        for j in range(3):
            self.W_e[j, j] = (100.0 if hack else 1.0) * self.W[j, j]
        self._wset(N, "W", self.W_e.flatten(order="F"))
        cpu_time = self._solve()
        new_vl_ref = self.x0[5] + self.u0[0] * self.dt_
        new_vr_ref = self.x0[6] + self.u0[1] * self.dt_
        robot_vel_ref.v, robot_vel_ref.w = self.inverseKinematrics(new_vl_ref, new_vr_ref)
        self.x0 = self._out_get(1, "x", self.nx)
        self.x0[5], self.x0[6] = new_vl_ref, new_vr_ref
        return True, cpu_time


class NMPCNavControlOmni4(NMPCNavControl):
    """NMPCNavControlOmni4.h / .cpp (no terminal-weight hack)."""

    model = "omni4"

    def __init__(self, dt, l1_plus_l2, tau_v, v_max, a_max, W_diag, N=None):
        super().__init__(dt, N)
        self._setup([l1_plus_l2, tau_v], [-v_max] * 4, [v_max] * 4, [-a_max] * 4, [a_max] * 4, W_diag)

    def directKinematrics(self, v, vn, w):
        h = 0.5 * self.p[0] * w
        return v - vn - h, -v - vn - h, v + vn - h, -v + vn - h

    def inverseKinematrics(self, v1, v2, v3, v4):
        return ((v1 - v2 + v3 - v4) / 4.0, (-v1 - v2 + v3 + v4) / 4.0, (-v1 - v2 - v3 - v4) / (2.0 * self.p[0]))

    def run(self, robot_pose, robot_vel, traj_ref, robot_vel_ref):
        """NMPCNavControlOmni4.cpp:91-177."""
        if not isinstance(robot_vel_ref, CmdVelOmni4):
            raise RuntimeError("Invalid command velocity type passed to run method.")
        self.x0[0:3] = (robot_pose.x, robot_pose.y, robot_pose.theta)
        self.x0[3:7] = self.directKinematrics(robot_vel.v, robot_vel.vn, robot_vel.w)
        self._cset(0, "lbx", self.x0)
        self._cset(0, "ubx", self.x0)
        self._pack_refs(robot_pose, traj_ref)
        cpu_time = self._solve()
        new_ref = self.x0[7:11] + self.u0 * self.dt_
        robot_vel_ref.v, robot_vel_ref.vn, robot_vel_ref.w = self.inverseKinematrics(*new_ref)
        self.x0 = self._out_get(1, "x", self.nx)
        self.x0[7:11] = new_ref
        return True, cpu_time


class NMPCNavControlTric(NMPCNavControl):
    """NMPCNavControlTric.h / .cpp (terminal hack commented out in the reference, :130-143)."""

    model = "tric"

    def __init__(self, dt, dist_d, tau_v, tau_a, v_max, a_max, alpha_min, alpha_max, dalpha_max, W_diag, N=None):
        super().__init__(dt, N)
        self.robot_steering_wheel_angle_ = 0.0
        self._setup([dist_d, tau_v, tau_a], [-v_max, alpha_min], [v_max, alpha_max], [-a_max, -dalpha_max],
                    [a_max, dalpha_max], W_diag)

    def setSteeringWheelAngle(self, a):
        self.robot_steering_wheel_angle_ = float(a)

    def run(self, robot_pose, robot_vel, traj_ref, robot_vel_ref):
        """NMPCNavControlTric.cpp:88-178."""
        if not isinstance(robot_vel_ref, CmdVelTric):
            raise RuntimeError("Invalid command velocity type passed to run method.")
        self.x0[0:3] = (robot_pose.x, robot_pose.y, robot_pose.theta)
        self.x0[3] = robot_vel.v
        self.x0[4] = self.robot_steering_wheel_angle_
        self._cset(0, "lbx", self.x0)
        self._cset(0, "ubx", self.x0)
        self._pack_refs(robot_pose, traj_ref)
        cpu_time = self._solve()
        new_v_ref = self.x0[5] + self.u0[0] * self.dt_
        new_alpha_ref = self.x0[6] + self.u0[1] * self.dt_
        robot_vel_ref.v, robot_vel_ref.alpha = new_v_ref, new_alpha_ref
        self.x0 = self._out_get(1, "x", self.nx)
        self.x0[5], self.x0[6] = new_v_ref, new_alpha_ref
        return True, cpu_time


def batch_solve(controllers):
    """Solve many capsules of one model in one device launch ({name}_acados_batch_solve)."""
    if not controllers:
        return np.zeros(0, np.int32)
    name = controllers[0]._name
    arr_t = ctypes.POINTER(type(controllers[0]._capsule.contents)) * len(controllers)
    arr = arr_t(*[c._capsule for c in controllers])
    status = np.zeros(len(controllers), np.int32)
    solve = getattr(solver_lib(name), f"{name}_acados_batch_solve")
    solve(arr, status.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), len(controllers))
    return status
