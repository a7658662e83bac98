"""ctypes binding of the fp64 CPU oracle (oracle/nmpc_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker / CPU baseline, never by the product package.
Parity with acados is UNPINNED (see nmpc_oracle.h).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

OC_DIFF, OC_OMNI4, OC_TRIC = 0, 1, 2
MODEL_IDS = {"diff": OC_DIFF, "omni4": OC_OMNI4, "tric": OC_TRIC}
NBMAX = 8
# IPM exit rules of the oracle (nmpc_oracle.h infeas_lambda): "acados" (the default) has no infeasibility exit, as
# HPIPM (a hard QP runs to iter_max; the capsule ABI's semantics); "batched" restates the batched device API's
# default early exit (status 4 once the bound multipliers pass 1e5 x the weight scale with the bound residual open,
# nmpc_model_params_default qp_infeas_lambda). A comparison against the batched API states rule="batched".
RULES = {"acados": 0.0, "batched": 1e5}


class OcParams(ctypes.Structure):
    _fields_ = [
        ("model", ctypes.c_int), ("N", ctypes.c_int),
        ("nx", ctypes.c_int), ("nu", ctypes.c_int), ("nbx", ctypes.c_int), ("nbu", ctypes.c_int),
        ("np", ctypes.c_int), ("ny", ctypes.c_int), ("nyn", ctypes.c_int),
        ("idxbx", ctypes.c_int * 4), ("idxbu", ctypes.c_int * 4),
        ("dt", ctypes.c_double), ("dt_ctrl", ctypes.c_double),
        ("p", ctypes.c_double * 3),
        ("lbx", ctypes.c_double * 4), ("ubx", ctypes.c_double * 4),
        ("lbu", ctypes.c_double * 4), ("ubu", ctypes.c_double * 4),
        ("W", ctypes.c_double * 15), ("W_e", ctypes.c_double * 11),
        ("terminal_hack", ctypes.c_int), ("tric_sin_bug", ctypes.c_int),
        ("iter_max", ctypes.c_int),
        ("tol_stat", ctypes.c_double), ("tol_ineq", ctypes.c_double), ("tol_comp", ctypes.c_double),
        ("mu0", ctypes.c_double), ("thr0", ctypes.c_double), ("tau", ctypes.c_double),
        ("infeas_lambda", ctypes.c_double),
    ]


class OcStats(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int), ("qp_iter", ctypes.c_int),
                ("res_stat", ctypes.c_double), ("res_ineq", ctypes.c_double), ("mu", ctypes.c_double)]


class OcQpSol(ctypes.Structure):
    _fields_ = [(n, ctypes.POINTER(ctypes.c_double))
                for n in ("du", "dx", "pi", "lam_lb", "lam_ub", "t_lb", "t_ub")]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        P = ctypes.POINTER(OcParams)
        _lib.oc_params_default.argtypes = [ctypes.c_int, ctypes.c_int, P]
        _lib.oc_params_set_limits.argtypes = [P] + [ctypes.c_double] * 5
        _lib.oc_model_f.argtypes = [P, dp, dp, dp]
        _lib.oc_model_jac.argtypes = [P, dp, dp, dp, dp]
        _lib.oc_rk4.argtypes = [P, dp, dp, ctypes.c_double, dp, dp, dp]
        _lib.oc_build_qp.argtypes = [P] + [dp] * 5 + [dp] * 12
        _lib.oc_sqp_rti_ex.argtypes = [P, dp, dp, dp, dp, dp, ctypes.POINTER(OcStats), ctypes.POINTER(OcQpSol)]
        _lib.oc_sqp_rti_ex.restype = ctypes.c_int
        _lib.oc_iterate_create.argtypes = [P, dp, dp]
        _lib.oc_iterate_reset.argtypes = [P, dp, dp]
        _lib.oc_prepare.argtypes = [P, dp, dp, ctypes.c_double, dp, ctypes.c_int, dp, dp, dp, dp]
        _lib.oc_post.argtypes = [P, dp, dp, dp, dp]
        _lib.oc_batch_tick.argtypes = [P, ctypes.c_int, dp, dp, dp, dp, ctypes.POINTER(ctypes.c_int),
                                       ctypes.POINTER(ctypes.c_ubyte), dp, dp, dp, dp, dp,
                                       ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        _lib.oc_batch_tick.restype = ctypes.c_int
        _lib.oc_path_discretize.argtypes = [ctypes.c_int, dp, ctypes.c_int, ctypes.POINTER(ctypes.c_int), dp,
                                            ctypes.c_double, ctypes.c_int, ctypes.c_int, dp,
                                            ctypes.POINTER(ctypes.c_int)]
    return _lib


def _p(a):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"], (a.dtype, a.flags)
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _ip(a):
    if a is None:
        return None
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


class Oracle:
    """One model configuration of the CPU oracle. `rule` is the IPM exit rule (RULES): "acados" by default, "batched"
    for comparisons against the batched device API's default parameters."""

    def __init__(self, model, N, rule="acados", **overrides):
        if rule not in RULES:
            raise ValueError(f"rule must be one of {sorted(RULES)}")
        self.model = model
        self.prm = OcParams()
        lib().oc_params_default(MODEL_IDS[model], N, ctypes.byref(self.prm))
        self.prm.infeas_lambda = RULES[rule]
        self.rule = rule if "infeas_lambda" not in overrides else f"infeas_lambda={overrides['infeas_lambda']:g}"
        for k, v in overrides.items():
            cur = getattr(self.prm, k)
            if isinstance(cur, ctypes.Array):
                for i, x in enumerate(v):
                    cur[i] = x
            else:
                setattr(self.prm, k, v)

    # dims
    @property
    def N(self):
        return self.prm.N

    @property
    def nx(self):
        return self.prm.nx

    @property
    def nu(self):
        return self.prm.nu

    @property
    def ny(self):
        return self.prm.ny

    @property
    def nbx(self):
        return self.prm.nbx

    @property
    def nbu(self):
        return self.prm.nbu

    def set_limits(self, v_max, a_max, alpha_min=-np.pi / 4, alpha_max=np.pi / 4, dalpha_max=np.pi / 12):
        lib().oc_params_set_limits(ctypes.byref(self.prm), v_max, a_max, alpha_min, alpha_max, dalpha_max)

    def f(self, x, u):
        out = np.zeros(self.nx)
        lib().oc_model_f(ctypes.byref(self.prm), _p(np.ascontiguousarray(x, np.float64)),
                         _p(np.ascontiguousarray(u, np.float64)), _p(out))
        return out

    def jac(self, x, u):
        Jx = np.zeros((self.nx, self.nx))
        Ju = np.zeros((self.nx, self.nu))
        lib().oc_model_jac(ctypes.byref(self.prm), _p(np.ascontiguousarray(x, np.float64)),
                           _p(np.ascontiguousarray(u, np.float64)), _p(Jx), _p(Ju))
        return Jx, Ju

    def rk4(self, x, u, h=None):
        h = self.prm.dt if h is None else h
        xn = np.zeros(self.nx)
        A = np.zeros((self.nx, self.nx))
        B = np.zeros((self.nx, self.nu))
        lib().oc_rk4(ctypes.byref(self.prm), _p(np.ascontiguousarray(x, np.float64)),
                     _p(np.ascontiguousarray(u, np.float64)), h, _p(xn), _p(A), _p(B))
        return xn, A, B

    def iterate_create(self):
        xb = np.zeros((self.N + 1, self.nx))
        ub = np.zeros((self.N, self.nu))
        lib().oc_iterate_create(ctypes.byref(self.prm), _p(xb), _p(ub))
        return xb, ub

    def build_qp(self, xbar, ubar, x0, yref, We):
        N, nx, nu, nbx, nbu = self.N, self.nx, self.nu, self.nbx, self.nbu
        q = dict(A=np.zeros((N, nx, nx)), B=np.zeros((N, nx, nu)), b=np.zeros((N, nx)),
                 Hx=np.zeros((N + 1, nx)), Hu=np.zeros((N, nu)), gx=np.zeros((N + 1, nx)), gu=np.zeros((N, nu)),
                 lbx=np.zeros((N + 1, nbx)), ubx=np.zeros((N + 1, nbx)), lbu=np.zeros((N, nbu)),
                 ubu=np.zeros((N, nbu)), dx0=np.zeros(nx))
        lib().oc_build_qp(ctypes.byref(self.prm), _p(np.ascontiguousarray(xbar, np.float64)),
                          _p(np.ascontiguousarray(ubar, np.float64)), _p(np.ascontiguousarray(x0, np.float64)),
                          _p(np.ascontiguousarray(yref, np.float64)), _p(np.ascontiguousarray(We, np.float64)),
                          *[_p(q[k]) for k in ("A", "B", "b", "Hx", "Hu", "gx", "gu", "lbx", "ubx", "lbu", "ubu",
                                               "dx0")])
        return q

    def sqp_rti(self, xbar, ubar, x0, yref, We, return_sol=False):
        """One SQP-RTI iteration; returns (status, stats dict, xbar_new, ubar_new[, sol])."""
        N, nx, nu = self.N, self.nx, self.nu
        xb = np.array(xbar, np.float64, order="C").reshape(N + 1, nx).copy()
        ub = np.array(ubar, np.float64, order="C").reshape(N, nu).copy()
        st = OcStats()
        arrs = dict(du=np.zeros((N, nu)), dx=np.zeros((N + 1, nx)), pi=np.zeros((N + 1, nx)),
                    lam_lb=np.zeros((N + 1, NBMAX)), lam_ub=np.zeros((N + 1, NBMAX)),
                    t_lb=np.zeros((N + 1, NBMAX)), t_ub=np.zeros((N + 1, NBMAX)))
        sol = OcQpSol(*[_p(arrs[k]) for k in ("du", "dx", "pi", "lam_lb", "lam_ub", "t_lb", "t_ub")])
        s = lib().oc_sqp_rti_ex(ctypes.byref(self.prm), _p(xb), _p(ub), _p(np.ascontiguousarray(x0, np.float64)),
                                _p(np.ascontiguousarray(yref, np.float64)), _p(np.ascontiguousarray(We, np.float64)),
                                ctypes.byref(st), ctypes.byref(sol))
        stats = dict(status=st.status, qp_iter=st.qp_iter, res_stat=st.res_stat, res_ineq=st.res_ineq, mu=st.mu)
        if return_sol:
            return s, stats, xb, ub, arrs
        return s, stats, xb, ub

    def prepare(self, pose, vel, steer, traj, carried):
        traj = np.ascontiguousarray(traj, np.float64).reshape(-1, 3)
        x0 = np.zeros(self.nx)
        yref = np.zeros((self.N + 1, self.ny))
        We = np.zeros(self.nx)
        lib().oc_prepare(ctypes.byref(self.prm), _p(np.ascontiguousarray(pose, np.float64)),
                         _p(np.ascontiguousarray(vel, np.float64)), float(steer), _p(traj), traj.shape[0],
                         _p(np.ascontiguousarray(carried, np.float64)), _p(x0), _p(yref), _p(We))
        return x0, yref, We

    def post(self, x0, u0):
        cmd = np.zeros(3)
        carried = np.zeros(self.nbx)
        lib().oc_post(ctypes.byref(self.prm), _p(np.ascontiguousarray(x0, np.float64)),
                      _p(np.ascontiguousarray(u0, np.float64)), _p(cmd), _p(carried))
        return cmd, carried

    def batch_tick(self, pose, vel, steer, traj, ntraj, reset, carried, xbar, ubar, nthreads=0):
        """AoS batch tick (the timed CPU baseline). carried/xbar/ubar updated in place."""
        B = pose.shape[0]
        cmd = np.zeros((B, 3))
        u0 = np.zeros((B, self.nu))
        status = np.zeros(B, np.int32)
        qp_iter = np.zeros(B, np.int32)
        rp = None
        if reset is not None:
            reset = np.ascontiguousarray(reset, np.uint8)
            rp = reset.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte))
        nf = lib().oc_batch_tick(ctypes.byref(self.prm), B, _p(pose), _p(vel), _p(steer), _p(traj), _ip(ntraj), rp,
                                 _p(carried), _p(xbar), _p(ubar), _p(cmd), _p(u0), _ip(status), _ip(qp_iter),
                                 int(nthreads))
        return nf, cmd, u0, status, qp_iter


def path_discretize(segs, nseg, nearest_u, sample_period, num_poses, is_holonomic=False):
    """PathDiscretizer::getNextNPoses (oracle/path_oracle.c) for B robots: segs float64 [B][S][16] (the
    nmpc_path_segment layout), nseg int32 [B], nearest_u [B]. Returns (poses [B][num_poses][3], steps [B])."""
    segs = np.ascontiguousarray(segs, np.float64)
    nseg = np.ascontiguousarray(nseg, np.int32)
    nearest_u = np.ascontiguousarray(nearest_u, np.float64)
    B, S = segs.shape[0], segs.shape[1]
    out = np.zeros((B, num_poses, 3))
    steps = np.zeros(B, np.int32)
    lib().oc_path_discretize(B, _p(segs), S, _ip(nseg), _p(nearest_u), float(sample_period), int(num_poses),
                             1 if is_holonomic else 0, _p(out), _ip(steps))
    return out, steps
