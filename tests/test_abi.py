"""CPU tests of the drop-in boundary: libnmpc_amd.so plus the generated libacados_ocp_solver_{name}.so export
every function include/*.h declares, the model-descriptor codegen (tools/generate_solver_libs.py), the
host-side calls that need no GPU (dims, default parameters, limits, version), and the parameter loaders
(nmpc_nav_control.yaml / acados_models.yaml surfaces, NMPCNavControlROS::readParam)."""
import glob
import math
import os
import re
import subprocess

import pytest

from nmpc_nav_control_amd import _lib
from nmpc_nav_control_amd.config import from_ros_params, horizon_from_codegen, load_yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = sorted(glob.glob(os.path.join(ROOT, "include", "**", "*.h"), recursive=True))
DECL = re.compile(r"^[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", re.M)


def declared_functions():
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        text = "\n".join(l for l in text.splitlines() if not l.lstrip().startswith("#"))
        for m in DECL.finditer(text):
            if not m.group(0).lstrip().startswith(("typedef", "return")):
                names.add(m.group(1))
    return names


def exported_symbols(path=None):
    out = subprocess.run(["nm", "-D", "--defined-only", path or _lib.LIB_PATH], capture_output=True, text=True,
                         check=True)
    return {l.split()[-1] for l in out.stdout.splitlines() if " T " in l}


def solver_lib_path(name):
    return os.path.join(_lib.LIB_DIR, f"libacados_ocp_solver_{name}.so")


def test_headers_declare_the_reference_abi(built):
    decl = declared_functions()
    for s in _lib.BATCH_SYMBOLS + _lib.NLP_SYMBOLS + _lib.capsule_symbols():
        assert s in decl, s


def test_library_exports_every_declared_function(built):
    """libnmpc_amd.so (the libacados part: ocp_nlp_*, nmpc_*) + the three generated solver libraries."""
    exported = exported_symbols()
    for name in _lib.MODEL_NAMES.values():
        exported |= exported_symbols(solver_lib_path(name))
    missing = declared_functions() - exported
    assert not missing, sorted(missing)


def test_solver_libraries_follow_the_acados_split(built):
    """libacados_ocp_solver_<name>.so (the link names of CMakeLists.txt:112-114) holds exactly the model's
    {name}_acados_* ABI and loads libnmpc_amd.so; libnmpc_amd.so holds no per-model symbol, so a process that
    links all three solver libraries (as the reference does) resolves each model to its own generated code."""
    core = exported_symbols()
    for name in _lib.MODEL_NAMES.values():
        p = solver_lib_path(name)
        syms = exported_symbols(p)
        assert syms == {f"{name}_acados_{s}" for s in _lib.CAPSULE_SUFFIXES}, sorted(syms)
        assert not any(s.startswith(f"{name}_") for s in core)
        dyn = subprocess.run(["readelf", "-d", p], capture_output=True, text=True, check=True).stdout
        assert "[libnmpc_amd.so]" in dyn and "$ORIGIN" in dyn


@pytest.mark.parametrize("model,dims", [
    ("diff", dict(nx=7, nu=2, ny=9, nbx=2, nbu=2, np=2)),
    ("omni4", dict(nx=11, nu=4, ny=15, nbx=4, nbu=4, np=2)),
    ("tric", dict(nx=7, nu=2, ny=9, nbx=2, nbu=2, np=3)),
])
def test_model_dims_match_generated_headers(built, model, dims):
    assert _lib.model_dims(model) == dims
    hdr = open(os.path.join(ROOT, "include", f"acados_solver_{_lib.MODEL_NAMES[model]}.h")).read()
    pre = _lib.MODEL_NAMES[model].upper()
    for k, v in (("NX", dims["nx"]), ("NU", dims["nu"]), ("NY", dims["ny"]), ("NYN", dims["nx"]),
                 ("NBX", dims["nbx"]), ("NBU", dims["nbu"]), ("NBX0", dims["nx"]),
                 ("NBXN", dims["nbx"]), ("NP", dims["np"])):
        assert re.search(rf"#define {pre}_{k}\s+{v}\b", hdr), (k, v)


def test_default_params_follow_codegen(built):
    """scripts/*/generate_c_code.py defaults: Q/R diagonals, v_max 1, a_max 1, dt = 1/40."""
    prm = _lib.default_params("diff", 80)
    assert prm.N == 80 and math.isclose(prm.dt, 1 / 40) and math.isclose(prm.dt_ctrl, 1 / 40)
    assert list(prm.W[:9]) == [10, 10, 5, 0, 0, 0, 0, 1, 1]
    assert list(prm.lbu[:2]) == [-1, -1] and list(prm.ubu[:2]) == [1, 1]
    assert list(prm.lbx[:2]) == [-1, -1] and list(prm.ubx[:2]) == [1, 1]
    assert prm.terminal_hack == 1
    t = _lib.default_params("tric", 80)
    assert t.terminal_hack == 0 and t.tric_sin_bug == 1  # tric_amr_model.py:45 reproduced by default
    assert math.isclose(t.p[0], 0.270) and math.isclose(t.p[2], 0.5)
    o = _lib.default_params("omni4", 80)
    assert math.isclose(o.p[0], 0.535) and o.terminal_hack == 0


def test_set_limits_tric_angles(built):
    prm = _lib.default_params("tric", 40)
    _lib.check(_lib.lib().nmpc_model_params_set_limits(prm, 0.8, 0.5, -1.2, 1.1, 0.3))
    assert list(prm.lbx[:2]) == pytest.approx([-0.8, -1.2]) and list(prm.ubx[:2]) == pytest.approx([0.8, 1.1])
    assert list(prm.lbu[:2]) == pytest.approx([-0.5, -0.3]) and list(prm.ubu[:2]) == pytest.approx([0.5, 0.3])


def test_invalid_model_is_an_argument_error(built):
    prm = _lib.ModelParams()
    rc = _lib.lib().nmpc_model_params_default(7, 40, prm)
    assert rc != 0 and b"model" in _lib.lib().nmpc_last_error()


def test_version_string(built):
    assert _lib.lib().nmpc_version().decode().startswith("nmpc_amd")


# ---- parameter surfaces ----------------------------------------------------------------------------------

@pytest.mark.parametrize("name,model", [("diff", "diff"), ("omni4", "omni4"), ("tric", "tric")])
def test_ros_yaml_loads(built, name, model):
    P = load_yaml(os.path.join(ROOT, "configs", f"{name}.yaml"))
    codegen = load_yaml(os.path.join(ROOT, "configs", "acados_models.yaml"))
    geom, prm = from_ros_params(P, codegen=codegen)
    assert geom == model
    N, dt = horizon_from_codegen(codegen[f"{model}_params"])
    assert prm.N == N and math.isclose(prm.dt, dt)
    nx = _lib.model_dims(model)["nx"]
    assert list(prm.W_e[:nx]) == P["cost_matrix_weights_state_diag"]


def test_ros_param_errors(built):
    with pytest.raises(RuntimeError, match="steering_geometry parameter"):
        from_ros_params({})
    with pytest.raises(RuntimeError, match="Invalid steering_geometry"):
        from_ros_params({"steering_geometry": "ackermann"})
    with pytest.raises(RuntimeError, match="requires the definition"):
        from_ros_params({"steering_geometry": "diff", "rob_dist_between_wh": 0.3})
    P = load_yaml(os.path.join(ROOT, "configs", "diff.yaml"))
    P["cost_matrix_weights_state_diag"] = [1, 2, 3]
    with pytest.raises(RuntimeError, match="array of 7 numeric values"):
        from_ros_params(P)


def test_codegen_horizon():
    """scripts/diff/common.py: N = ceil(tf_ini * freq); shipped config tf_ini 2.0, freq 40 -> N 80."""
    assert horizon_from_codegen({"tf_ini": 2.0, "freq": 40}) == (80, 1 / 40)
    assert horizon_from_codegen({"tf_ini": 1.0, "freq": 40})[0] == 40


def test_params_struct_layout_and_ipm_options(built):
    """The ctypes mirror of nmpc_model_params covers exactly what the library writes (a guard region past the
    mirror stays untouched), the IPM rule defaults to one direction per iteration, and a bad rule or sigma
    clamp is an argument error at nmpc_batch_create."""
    import ctypes
    L = _lib.lib()
    n = ctypes.sizeof(_lib.ModelParams)
    buf = (ctypes.c_ubyte * (n + 64))(*([0xAB] * (n + 64)))
    prm = _lib.ModelParams.from_buffer(buf)
    assert L.nmpc_model_params_default(0, 40, ctypes.byref(prm)) == 0
    assert bytes(buf[n:]) == b"\xab" * 64
    assert prm.qp_ipm == 1 and (prm.qp_sigma_lo, prm.qp_sigma_hi) == (0.01, 0.5)
    assert prm.qp_warm_start == 1 and prm.qp_warm_kappa == 0.2
    h = ctypes.c_void_p()
    for field, val in (("qp_ipm", 2), ("qp_sigma_lo", 0.0), ("qp_sigma_hi", 1.5), ("qp_warm_start", 3),
                       ("qp_warm_kappa", 0.0)):
        bad = _lib.ModelParams()
        assert L.nmpc_model_params_default(0, 20, ctypes.byref(bad)) == 0
        setattr(bad, field, val)
        assert L.nmpc_batch_create(ctypes.byref(bad), 8, ctypes.byref(h)) != 0, field
        assert b"qp_" in L.nmpc_last_error()


def test_null_handle_is_an_argument_error_everywhere(built):
    """Every batched entry point checks its handle before touching the device: NULL -> NMPC_ERR_ARG and a message
    (the reference's wrappers map any non-zero status to their exception path, NMPCNavControl.cpp:14-23)."""
    import ctypes
    L = _lib.lib()
    vp = ctypes.c_void_p
    calls = {
        "nmpc_batch_set_params": lambda: L.nmpc_batch_set_params(None, _lib.default_params("diff", 20)),
        "nmpc_batch_get_params": lambda: L.nmpc_batch_get_params(None, _lib.ModelParams()),
        "nmpc_batch_init_iterate": lambda: L.nmpc_batch_init_iterate(None, 1, 0, None),
        "nmpc_batch_solve": lambda: L.nmpc_batch_solve(None, 1, *([None] * 2), 9, *([None] * 11)),
        "nmpc_batch_solve_iterate": lambda: L.nmpc_batch_solve_iterate(None, 1, None, None, 9, *([None] * 4), 1,
                                                                        *([None] * 4)),
        "nmpc_batch_run": lambda: L.nmpc_batch_run(None, 1, *([None] * 12)),
        "nmpc_batch_set_kernel": lambda: L.nmpc_batch_set_kernel(None, 0),
        "nmpc_batch_set_schedule": lambda: L.nmpc_batch_set_schedule(None, 0),
        "nmpc_batch_state": lambda: L.nmpc_batch_state(None, None, None, None, None),
        "nmpc_batch_forget_warm": lambda: L.nmpc_batch_forget_warm(None, 1, None, None),
        "nmpc_batch_warm_state": lambda: L.nmpc_batch_warm_state(None, None, None, None),
        "nmpc_batch_warm_rule": lambda: L.nmpc_batch_warm_rule(None, None, None, None),
        "nmpc_batch_plan": lambda: L.nmpc_batch_plan(None, 1, None, None, None),
        "nmpc_fleet_sim_step": lambda: L.nmpc_fleet_sim_step(None, 1, *([None] * 9), 0, None),
    }
    for name, call in calls.items():
        assert call() == -1, name  # NMPC_ERR_ARG
        assert L.nmpc_last_error(), name
    assert L.nmpc_batch_destroy(vp()) == 0  # destroying NULL is a no-op, like free()


@pytest.mark.parametrize("field,val,code", [("N", 0, -1), ("N", 5000, -1), ("dt", 0.0, -1), ("dt_ctrl", -1.0, -1),
                                            ("qp_iter_max", 0, -1), ("qp_warm_iter_max", -1, -1)])
def test_params_validation_at_create(built, field, val, code):
    """nmpc_batch_create validates the parameter block before any device allocation (runs without a GPU)."""
    import ctypes
    L = _lib.lib()
    bad = _lib.default_params("diff", 20)
    setattr(bad, field, val)
    h = ctypes.c_void_p()
    assert L.nmpc_batch_create(ctypes.byref(bad), 8, ctypes.byref(h)) == code, field
    assert not h.value and L.nmpc_last_error()


def test_bounds_weights_and_capacity_validation(built):
    """Empty bound boxes and non-positive model parameters are argument errors; a zero input weight R is the one
    unsupported OCP (the input-block Cholesky needs R dt > 0, as the reference's yaml always gives); capacity < 1."""
    import ctypes
    L = _lib.lib()
    h = ctypes.c_void_p()
    for mutate, code in ((lambda p: p.lbx.__setitem__(0, p.ubx[0]), -1), (lambda p: p.lbu.__setitem__(1, 2.0), -1),
                         (lambda p: p.p.__setitem__(0, 0.0), -1), (lambda p: p.W.__setitem__(7, 0.0), -3)):
        prm = _lib.default_params("diff", 20)
        mutate(prm)
        assert L.nmpc_batch_create(ctypes.byref(prm), 8, ctypes.byref(h)) == code
        assert not h.value
    assert L.nmpc_batch_create(ctypes.byref(_lib.default_params("diff", 20)), 0, ctypes.byref(h)) == -1
    assert b"capacity" in L.nmpc_last_error()
