"""ctypes binding of libnmpc_amd.so (the HIP solve path). Fails loudly when the library is missing:
there is no CPU fallback in the product package."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
LIB_PATH = os.environ.get("NMPC_AMD_LIB") or os.path.join(LIB_DIR, "libnmpc_amd.so")

MODEL_IDS = {"diff": 0, "omni4": 1, "tric": 2}
MODEL_NAMES = {"diff": "diff2amr", "omni4": "omni4amr", "tric": "tric3amr"}

c_int_p = ctypes.POINTER(ctypes.c_int)
c_double_p = ctypes.POINTER(ctypes.c_double)
c_void_p = ctypes.c_void_p


class ModelParams(ctypes.Structure):
    """Mirror of nmpc_model_params (include/nmpc_amd/nmpc_batch.h)."""
    _fields_ = [
        ("model", ctypes.c_int), ("N", ctypes.c_int),
        ("dt", ctypes.c_double), ("dt_ctrl", ctypes.c_double),
        ("p", ctypes.c_double * 3),
        ("lbx", ctypes.c_double * 4), ("ubx", ctypes.c_double * 4),
        ("lbu", ctypes.c_double * 4), ("ubu", ctypes.c_double * 4),
        ("W", ctypes.c_double * 15), ("W_e", ctypes.c_double * 11),
        ("terminal_hack", ctypes.c_int), ("tric_sin_bug", ctypes.c_int),
        ("qp_iter_max", ctypes.c_int),
        ("qp_tol_stat", ctypes.c_double), ("qp_tol_ineq", ctypes.c_double), ("qp_tol_comp", ctypes.c_double),
        ("qp_mu0", ctypes.c_double), ("qp_thr0", ctypes.c_double), ("qp_tau", ctypes.c_double),
        ("qp_ipm", ctypes.c_int), ("qp_sigma_lo", ctypes.c_double), ("qp_sigma_hi", ctypes.c_double),
        ("qp_warm_start", ctypes.c_int), ("qp_warm_kappa", ctypes.c_double), ("qp_warm_iter_max", ctypes.c_int),
        ("qp_infeas_lambda", ctypes.c_double),
    ]


class FleetStats(ctypes.Structure):
    """Mirror of nmpc_fleet_stats (include/nmpc_amd/nmpc_batch.h): per-tick solve statistics accumulated by the
    renewal launch."""
    _fields_ = [("qp_iter", c_void_p), ("iters_sum", c_void_p), ("iters_max", c_void_p), ("fail_cnt", c_void_p),
                ("hist", c_void_p), ("cold_cnt", c_void_p), ("cold_iters", c_void_p)]


class FleetRenew(ctypes.Structure):
    """Mirror of nmpc_fleet_renew (include/nmpc_amd/nmpc_batch.h): the harness's stationary goal / path renewal."""
    _fields_ = [("seed", ctypes.c_uint), ("start", ctypes.c_int), ("ttl_min", ctypes.c_int), ("ttl_max", ctypes.c_int),
                ("goal_r_lo", ctypes.c_float), ("goal_r_hi", ctypes.c_float), ("kappa_max", ctypes.c_float),
                ("speed_lo", ctypes.c_float), ("speed_hi", ctypes.c_float), ("len_lo", ctypes.c_float),
                ("len_hi", ctypes.c_float), ("pos_tol", ctypes.c_float), ("ang_tol", ctypes.c_float),
                ("ev", c_void_p), ("ttl", c_void_p), ("reset", c_void_p), ("stats", c_void_p)]


class LaunchPlan(ctypes.Structure):
    """Mirror of nmpc_launch_plan (include/nmpc_amd/nmpc_batch.h)."""
    _fields_ = [("kernel", ctypes.c_int), ("waves_per_robot", ctypes.c_int), ("segments", ctypes.c_int),
                ("record_layout", ctypes.c_int), ("warm_tag", ctypes.c_int), ("record_bytes", ctypes.c_size_t)]


class CodegenDesc(ctypes.Structure):
    """Mirror of nmpc_codegen_desc (include/nmpc_amd/nmpc_capsule.h)."""
    _fields_ = [("model", ctypes.c_int), ("N", ctypes.c_int), ("tf", ctypes.c_double),
                ("p", ctypes.c_double * 3), ("lbx", ctypes.c_double * 4), ("ubx", ctypes.c_double * 4),
                ("lbu", ctypes.c_double * 4), ("ubu", ctypes.c_double * 4), ("W", ctypes.c_double * 15),
                ("W_e", ctypes.c_double * 11)]


class NlpOut(ctypes.Structure):
    """Mirror of the ocp_nlp_out handle (include/acados_c/ocp_nlp_interface.h)."""
    _fields_ = [("impl", c_void_p), ("inf_norm_res", ctypes.c_double), ("total_cost", ctypes.c_double),
                ("sqp_iter", ctypes.c_int)]


class SolverCapsule(ctypes.Structure):
    """Mirror of {name}_solver_capsule (include/acados_solver_{name}.h)."""
    _fields_ = [("nlp_config", c_void_p), ("nlp_dims", c_void_p), ("nlp_in", c_void_p),
                ("nlp_out", ctypes.POINTER(NlpOut)), ("nlp_solver", c_void_p), ("nlp_opts", c_void_p),
                ("impl", c_void_p)]


# every symbol the public headers declare (checked by tests/test_abi_symbols.py)
BATCH_SYMBOLS = [
    "nmpc_model_dims", "nmpc_model_params_default", "nmpc_model_params_set_limits", "nmpc_batch_create",
    "nmpc_batch_destroy", "nmpc_batch_set_params", "nmpc_batch_get_params", "nmpc_batch_init_iterate",
    "nmpc_batch_solve", "nmpc_batch_solve_iterate", "nmpc_batch_run", "nmpc_batch_run_path", "nmpc_batch_state", "nmpc_batch_warm_state", "nmpc_batch_warm_rule", "nmpc_batch_plan", "nmpc_batch_plan_ex", "nmpc_batch_set_record_layout", "nmpc_batch_forget_warm", "nmpc_batch_set_kernel", "nmpc_batch_set_schedule",
    "nmpc_fleet_sim_step", "nmpc_fleet_sim_step_renew", "nmpc_fleet_hash",
    "nmpc_last_error", "nmpc_version", "nmpc_path_discretize", "nmpc_codegen_default", "nmpc_capsule_new",
    "nmpc_capsule_delete", "nmpc_capsule_create", "nmpc_capsule_reset", "nmpc_capsule_update_params",
    "nmpc_capsule_solve", "nmpc_capsule_batch_solve", "nmpc_capsule_free", "nmpc_capsule_print_stats",
]
KERNELS = {"team": 0}
REC_LAYOUTS = {"auto": -1, "wide": 0, "split": 1}
PLAN_MODES = {"solve": 0, "run": 1, "run_path": 2}
WARM_TAGS = {1: "wide", 2: "split", 3: "mehrotra"}
SCHEDULES = {"off": 0, "auto": 1, "sorted": 2, "interleaved": 3, "spread": 4}
NLP_SYMBOLS = ["ocp_nlp_constraints_model_set", "ocp_nlp_cost_model_set", "ocp_nlp_constraints_model_get",
               "ocp_nlp_cost_model_get", "ocp_nlp_out_get", "ocp_nlp_out_set", "ocp_nlp_get", "ocp_nlp_solver_opts_set",
               "ocp_nlp_dims_get_from_attr"]
CAPSULE_SUFFIXES = ["create_capsule", "free_capsule", "create", "create_with_discretization", "reset",
                    "update_params", "solve", "batch_solve", "free", "print_stats", "get_nlp_in", "get_nlp_out",
                    "get_nlp_solver", "get_nlp_config", "get_nlp_opts", "get_nlp_dims"]


def capsule_symbols():
    return [f"{n}_acados_{s}" for n in MODEL_NAMES.values() for s in CAPSULE_SUFFIXES]


_lib = None


def lib():
    """Load libnmpc_amd.so (raises if it was not built: run __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libnmpc_amd.so not found at {LIB_PATH}: build it with "
                           "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    P = ctypes.POINTER(ModelParams)
    i, vp = ctypes.c_int, c_void_p
    L.nmpc_model_dims.argtypes = [i] + [c_int_p] * 6
    L.nmpc_model_params_default.argtypes = [i, i, P]
    L.nmpc_model_params_set_limits.argtypes = [P] + [ctypes.c_double] * 5
    L.nmpc_batch_create.argtypes = [P, i, ctypes.POINTER(vp)]
    L.nmpc_batch_destroy.argtypes = [vp]
    L.nmpc_batch_set_params.argtypes = [vp, P]
    L.nmpc_batch_get_params.argtypes = [vp, P]
    L.nmpc_batch_init_iterate.argtypes = [vp, i, i, vp]
    L.nmpc_batch_solve.argtypes = [vp, i, vp, vp, i, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.nmpc_batch_solve_iterate.argtypes = [vp, i, vp, vp, i, vp, vp, vp, vp, i, vp, vp, vp, vp]
    L.nmpc_batch_run.argtypes = [vp, i, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.nmpc_batch_run_path.argtypes = [vp, i, vp, vp, vp, vp, i, vp, vp, ctypes.c_double, i, vp, vp, vp, vp, vp, vp,
                                      vp, vp]
    L.nmpc_batch_set_kernel.argtypes = [vp, i]
    L.nmpc_batch_set_schedule.argtypes = [vp, i]
    L.nmpc_batch_state.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp), c_int_p]
    L.nmpc_batch_forget_warm.argtypes = [vp, i, vp, vp]
    L.nmpc_batch_warm_state.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_size_t)]
    L.nmpc_batch_warm_rule.argtypes = [vp, c_int_p, c_int_p, c_int_p]
    L.nmpc_batch_plan.argtypes = [vp, ctypes.c_int, c_int_p, c_int_p, c_int_p]
    L.nmpc_batch_plan_ex.argtypes = [vp, i, i, ctypes.POINTER(LaunchPlan)]
    L.nmpc_batch_set_record_layout.argtypes = [vp, i]
    L.nmpc_fleet_sim_step.argtypes = [vp, i, vp, vp, vp, vp, vp, vp, vp, vp, vp, i, vp]
    L.nmpc_fleet_sim_step_renew.argtypes = [vp, i, vp, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.POINTER(FleetRenew), vp]
    L.nmpc_fleet_hash.argtypes = [ctypes.c_uint, ctypes.c_uint, ctypes.c_uint]
    L.nmpc_fleet_hash.restype = ctypes.c_uint
    L.nmpc_path_discretize.argtypes = [i, vp, i, vp, vp, ctypes.c_double, i, i, vp, vp, vp]
    L.nmpc_codegen_default.argtypes = [i, ctypes.POINTER(CodegenDesc)]
    L.nmpc_last_error.restype = ctypes.c_char_p
    L.nmpc_version.restype = ctypes.c_char_p
    cp = ctypes.POINTER(SolverCapsule)
    L.nmpc_capsule_new.restype = cp
    L.nmpc_capsule_new.argtypes = [i]
    L.ocp_nlp_constraints_model_set.argtypes = [vp, vp, vp, vp, i, ctypes.c_char_p, vp]
    L.ocp_nlp_cost_model_set.argtypes = [vp, vp, vp, i, ctypes.c_char_p, vp]
    L.ocp_nlp_out_get.argtypes = [vp, vp, vp, i, ctypes.c_char_p, vp]
    L.ocp_nlp_out_set.argtypes = [vp, vp, vp, i, ctypes.c_char_p, vp]
    L.ocp_nlp_get.argtypes = [vp, ctypes.c_char_p, vp]
    L.ocp_nlp_solver_opts_set.argtypes = [vp, vp, ctypes.c_char_p, vp]
    _lib = L
    return L


_solver_libs = {}


def solver_lib(name):
    """libacados_ocp_solver_{name}.so: the generated per-model ABI (tools/generate_solver_libs.py) that
    forwards to libnmpc_amd.so with the codegen configuration baked in."""
    if name in _solver_libs:
        return _solver_libs[name]
    lib()  # libnmpc_amd.so first (RTLD_GLOBAL): the solver library resolves to the same instance
    path = os.path.join(os.path.dirname(LIB_PATH), f"libacados_ocp_solver_{name}.so")
    if not os.path.exists(path):
        path = os.path.join(LIB_DIR, f"libacados_ocp_solver_{name}.so")
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not found: build it with `make -C nmpc_nav_control_amd/csrc`")
    S = ctypes.CDLL(path)
    cp = ctypes.POINTER(SolverCapsule)
    i = ctypes.c_int
    getattr(S, f"{name}_acados_create_capsule").restype = cp
    getattr(S, f"{name}_acados_free_capsule").argtypes = [cp]
    getattr(S, f"{name}_acados_create").argtypes = [cp]
    getattr(S, f"{name}_acados_create_with_discretization").argtypes = [cp, i, c_double_p]
    getattr(S, f"{name}_acados_reset").argtypes = [cp, i]
    getattr(S, f"{name}_acados_update_params").argtypes = [cp, i, c_double_p, i]
    getattr(S, f"{name}_acados_solve").argtypes = [cp]
    getattr(S, f"{name}_acados_batch_solve").argtypes = [ctypes.POINTER(cp), c_int_p, i]
    getattr(S, f"{name}_acados_free").argtypes = [cp]
    _solver_libs[name] = S
    return S


def check(rc, what="nmpc call"):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {lib().nmpc_last_error().decode()}")
    return rc


def default_params(model, N):
    prm = ModelParams()
    check(lib().nmpc_model_params_default(MODEL_IDS[model], int(N), ctypes.byref(prm)), "params_default")
    return prm


def model_dims(model):
    vals = [ctypes.c_int() for _ in range(6)]
    check(lib().nmpc_model_dims(MODEL_IDS[model], *[ctypes.byref(v) for v in vals]), "model_dims")
    return dict(zip(("nx", "nu", "ny", "nbx", "nbu", "np"), (v.value for v in vals)))
