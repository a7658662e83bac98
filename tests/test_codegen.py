"""CPU tests of the model-descriptor codegen (tools/generate_solver_libs.py), the counterpart of the reference's
scripts/generate_acados_libs.py + scripts/<geometry>/generate_c_code.py: what a codegen yaml bakes
(scripts/<geometry>/common.py load_parameters), the generated c_generated_code/ layout, and a C program that
includes the generated header and links the generated library the way CMakeLists.txt:66-72,112-114 does."""
import json
import math
import os
import subprocess
import sys

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import generate_solver_libs as gen  # noqa: E402

from nmpc_nav_control_amd import _lib  # noqa: E402

SHIPPED = os.path.join(ROOT, "configs", "acados_models.yaml")


def test_shipped_descriptors():
    P = yaml.safe_load(open(SHIPPED))
    d = gen.load_parameters("diff", P["diff_params"])
    assert (d["N"], d["tf"]) == (80, 2.0)
    assert d["p"] == [0.270, 0.1] and d["lbu"] == [-2.0, -2.0] and d["ubx"] == [1.0, 1.0]
    assert d["W"] == [10, 10, 5, 0, 0, 0, 0, 1, 1] and d["W_e"] == [1000, 1000, 500, 0, 0, 0, 0]
    t = gen.load_parameters("tric", P["tric_params"])
    deg = math.pi / 180
    assert t["p"] == [0.270, 0.1, 0.5]
    assert t["lbx"] == [-1.0, -30 * deg] and t["ubx"] == [1.0, 30 * deg]
    assert t["lbu"] == [-1.0, -120 * deg] and t["ubu"] == [1.0, 120 * deg]
    o = gen.load_parameters("omni4", P["omni4_params"])
    assert o["p"] == [0.535, 0.1] and o["lbx"] == [-1.0] * 4 and len(o["W"]) == 15


def test_horizon_rounds_up():
    """N = ceil(tf_ini / (1/freq)) (scripts/diff/common.py:7-8), TF = N dt."""
    P = yaml.safe_load(open(SHIPPED))["diff_params"]
    d = gen.load_parameters("diff", dict(P, tf_ini=1.01, freq=20))
    assert d["N"] == 21 and d["tf"] == pytest.approx(21 / 20)


def test_library_descriptors_match_the_shipped_defaults(built):
    """The in-tree libraries are generated from configs/acados_models.yaml; nmpc_codegen_default holds the
    same values (used when a capsule is created without a descriptor)."""
    import ctypes
    Desc = _lib.CodegenDesc

    P = yaml.safe_load(open(SHIPPED))
    L = _lib.lib()
    for geom, model in (("diff", 0), ("omni4", 1), ("tric", 2)):
        exp = gen.load_parameters(geom, P[f"{geom}_params"])
        got = Desc()
        assert L.nmpc_codegen_default(model, ctypes.byref(got)) == 0
        assert (got.N, got.tf) == (exp["N"], exp["tf"])
        for k in ("p", "lbx", "ubx", "lbu", "ubu", "W", "W_e"):
            assert list(getattr(got, k))[:len(exp[k])] == pytest.approx(exp[k], abs=1e-15), (geom, k)
        gen_json = json.load(open(os.path.join(ROOT, "build", "generated", geom, f"acados_ocp_{exp['name']}.json")))
        assert gen_json["N"] == exp["N"] and gen_json["W"] == exp["W"]


PROGRAM = r"""
#include <stdio.h>
#include "acados_solver_diff2amr.h"
#include "acados_c/ocp_nlp_interface.h"
int main(void) {
    diff2amr_solver_capsule* c = diff2amr_acados_create_capsule();
    int st = diff2amr_acados_create(c);
    double x[DIFF2AMR_NX];
    ocp_nlp_out_get(c->nlp_config, c->nlp_dims, c->nlp_out, 0, "x", x);
    int nu = ocp_nlp_dims_get_from_attr(c->nlp_config, c->nlp_dims, c->nlp_out, DIFF2AMR_N - 1, "u");
    printf("%d %d %d %d %.6f\n", st, DIFF2AMR_N, c->nlp_dims->N, nu, x[2]);
    diff2amr_acados_free(c);
    diff2amr_acados_free_capsule(c);
    return 0;
}
"""


DISC_PROGRAM = r"""
#include <stdio.h>
#include "acados_solver_diff2amr.h"
#include "acados_c/ocp_nlp_interface.h"
int main(void) {
    diff2amr_solver_capsule* c = diff2amr_acados_create_capsule();
    int st_null = diff2amr_acados_create_with_discretization(c, 12, NULL);
    double steps[12];
    for (int k = 0; k < 12; k++) steps[k] = 0.05;
    int st = diff2amr_acados_create_with_discretization(c, 12, steps);
    double w[DIFF2AMR_NYN * DIFF2AMR_NYN] = {0};
    int st_w = ocp_nlp_cost_model_set(c->nlp_config, c->nlp_dims, c->nlp_in, 13, "W", w);  /* past N = 12 */
    int st_w12 = ocp_nlp_cost_model_set(c->nlp_config, c->nlp_dims, c->nlp_in, 12, "W", w);
    printf("%d %d %d %d %d\n", st_null, st, c->nlp_dims->N, st_w, st_w12);
    diff2amr_acados_free(c);
    diff2amr_acados_free_capsule(c);
    return 0;
}
"""


def test_generated_tree_links_like_the_reference(built, tmp_path):
    cfg = yaml.safe_load(open(SHIPPED))
    cfg["diff_params"].update(tf_ini=1.0, freq=20)  # N = 20
    del cfg["omni4_params"]
    yml = tmp_path / "models.yaml"
    yml.write_text(yaml.safe_dump(cfg))
    out = tmp_path / "scripts"
    rc = gen.main([str(yml), "--out", str(out)])
    assert rc == 0
    cg = out / "diff" / "c_generated_code"
    assert sorted(os.listdir(cg)) == ["acados_ocp_diff2amr.json", "acados_solver_diff2amr.h",
                                      "diff2amr_solver.c", "libacados_ocp_solver_diff2amr.so"]
    assert not (out / "omni4").exists() and (out / "tric" / "c_generated_code").exists()
    assert "#define DIFF2AMR_N      20" in (cg / "acados_solver_diff2amr.h").read_text()
    # CMakeLists.txt: include_directories(${ACADOS_INCLUDE_DIRS} ${diff2amr_model}), link ${ACADOS_LIBRARIES}
    # (= libnmpc_amd.so) and ${diff2amr_model}/libacados_ocp_solver_diff2amr.so
    (tmp_path / "main.c").write_text(PROGRAM)
    exe = tmp_path / "main"
    subprocess.run(["gcc", "-std=c11", "-I", str(cg), "-I", os.path.join(ROOT, "include"), str(tmp_path / "main.c"),
                    _lib.LIB_PATH, str(cg / "libacados_ocp_solver_diff2amr.so"), "-o", str(exe)], check=True)
    env = dict(os.environ)
    env.pop("NMPC_AMD_DIFF2AMR_N", None)
    res = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=120)
    assert res.returncode == 0, res.stderr
    st, n_macro, n_dims, nu, th = res.stdout.split()
    assert (int(st), int(n_macro), int(n_dims), int(nu)) == (0, 20, 20, 2)
    assert float(th) == pytest.approx(math.pi, abs=1e-6)  # create(): x = ocp.constraints.x0 = [0, 0, pi, ...]
    # another horizon needs its time steps, as in acados' create_with_discretization (a NULL vector with
    # n != the baked N fails and says why); with uniform steps the capsule takes the new N
    (tmp_path / "disc.c").write_text(DISC_PROGRAM)
    exe2 = tmp_path / "disc"
    subprocess.run(["gcc", "-std=c11", "-I", str(cg), "-I", os.path.join(ROOT, "include"), str(tmp_path / "disc.c"),
                    _lib.LIB_PATH, str(cg / "libacados_ocp_solver_diff2amr.so"), "-o", str(exe2)], check=True)
    res = subprocess.run([str(exe2)], capture_output=True, text=True, env=env, timeout=120)
    assert res.returncode == 0, res.stderr
    assert res.stdout.split() == ["1", "0", "12", "-1", "0"]
    assert "new_time_steps is NULL" in res.stderr and "stage 13 outside 0..12" in res.stderr


def test_generator_errors(tmp_path, caplog):
    assert gen.main([]) == 1
    assert "The path for the YAML file is required" in caplog.text
    bad = tmp_path / "bad.yaml"
    bad.write_text(yaml.safe_dump({"diff_params": {"tf_ini": 2.0, "freq": 40}}))
    assert gen.main([str(bad), "--out", str(tmp_path / "o")]) == 1
    assert "Failed to generate Acados solver libraries" in caplog.text
    empty = tmp_path / "empty.yaml"
    empty.write_text(yaml.safe_dump({"other": 1}))
    assert gen.main([str(empty), "--out", str(tmp_path / "o2")]) == 0
    assert "No parameters found in YAML file to generate the 'diff' libraries." in caplog.text


def test_descriptors_pinned_to_the_reference_loader():
    """tools/generate_solver_libs.load_parameters against the reference's own scripts/*/common.py
    load_parameters, evaluated on the shipped codegen yaml and variations of it (fixture made by
    tests/golden/make_codegen_descriptors.py): N, TF, parameters, bounds (tric angles in radians) and the
    W = blkdiag(Q, R), W_e = QN that generate_c_code.py bakes, bit for bit."""
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "codegen_descriptors.json")))
    assert len(fx["cases"]) == 16
    pkeys = {"diff": ["DIST_B", "TAU_V"], "omni4": ["L1_PLUS_L2", "TAU_V"], "tric": ["DIST_D", "TAU_V", "TAU_A"]}
    for case in fx["cases"]:
        g, ref = case["geometry"], case["load_parameters"]
        d = gen.load_parameters(g, case["params"])
        assert d["N"] == ref["N"] and d["tf"] == ref["TF"], (g, case["params"])
        assert d["p"] == [ref[k] for k in pkeys[g]]
        assert d["W"] == ref["Q_diag"] + ref["R_diag"] and d["W_e"] == ref["QN_diag"]
        nb = {"diff": 2, "omni4": 4, "tric": 1}[g]
        assert d["ubx"][:nb] == [ref["V_MAX"]] * nb and d["lbx"][:nb] == [-ref["V_MAX"]] * nb
        if g == "tric":
            assert (d["lbx"][1], d["ubx"][1]) == (ref["ALPHA_MIN"], ref["ALPHA_MAX"])
            assert (d["lbu"], d["ubu"]) == ([-ref["A_MAX"], -ref["DALPHA_MAX"]], [ref["A_MAX"], ref["DALPHA_MAX"]])
        else:
            assert d["lbu"] == [-ref["A_MAX"]] * nb and d["ubu"] == [ref["A_MAX"]] * nb


def test_team_asm_header_is_generated():
    """csrc/team_asm_gen.hpp is the output of tools/gen_team_asm.py, byte for byte (the kernels'
    fused-DPP asm blocks are edited in the generator, never in the header)."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("gen_team_asm", os.path.join(root, "tools", "gen_team_asm.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    with open(gen.OUT) as fh:
        assert fh.read() == gen.generate(), "team_asm_gen.hpp differs from tools/gen_team_asm.py: regenerate it"


# A/B-only build options (each decided by a same-box A/B run) keep compiling: the product library leaves
# them out, so nothing else would notice when a change of the shared blocks breaks one (the
# -DNMPC_ROWPAR_MCOL call of m_block had kept an old signature). Syntax and template instantiation only (-fsyntax-only,
# device and host), a few seconds each.
AB_VARIANTS = [("sqp_rti_rowpar.hip", "-DNMPC_ROWPAR_MCOL"), ("sqp_rti_rowpar.hip", "-DNMPC_SEQ_MASTER"),
               ("sqp_rti_rowpar.hip", "-DNMPC_STAMPS"), ("sqp_rti_team.hip", "-DNMPC_MROW"),
               ("sqp_rti_team.hip", "-DNMPC_MCOL_ALL"), ("sqp_rti_team.hip", "-DNMPC_SEQ_PIVOTS"),
               ("sqp_rti_team.hip", "-DNMPC_ROW_PIV2"), ("sqp_rti_team.hip", "-DNMPC_STAMPS"),
               ("sqp_rti_team.hip", "-DP1_MASKED_STORE"), ("sqp_rti_team.hip", "-DNMPC_REC_FULL"),
               ("sqp_rti_team.hip", "-DNMPC_RSS_FULL"), ("sqp_rti_team.hip", "-DNMPC_HYBRID"),
               ("sqp_rti_rowpar.hip", "-DNMPC_HYBRID"), ("nmpc_batch.cpp", "-DNMPC_HYBRID"),
               ("sqp_rti_team.hip", "-DNMPC_F32_FACTOR"), ("sqp_rti_rowpar.hip", "-DNMPC_P0_SERIAL"),
               ("sqp_rti_rowpar.hip", "-DNMPC_W4_BOUND2"), ("sqp_rti_rowpar.hip", "-DNMPC_P0_NO_OVERLAP"),
               ("sqp_rti_rowpar.hip", "-DNMPC_SENS_FUSED"), ("sqp_rti_rowpar.hip", "-DNMPC_D_SEPARATE"),
               ("sqp_rti_rowpar.hip", "-DNMPC_LR_IN_C")]


@pytest.mark.parametrize("src,flag", AB_VARIANTS, ids=[f"{s.split('.')[0]}{f[2:].lower()}" for s, f in AB_VARIANTS])
def test_ab_variant_compiles(src, flag):
    csrc = os.path.join(ROOT, "nmpc_nav_control_amd", "csrc")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only", "-Wno-unused-command-line-argument",
           "-I", os.path.join(ROOT, "include"), "-I", csrc, flag]
    if src.endswith(".cpp"):
        cmd += ["-x", "hip"]
    r = subprocess.run(cmd + [os.path.join(csrc, src)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
