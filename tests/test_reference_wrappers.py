"""The reference's own per-model wrappers against the drop-in boundary (CPU; skipped without /root/reference).

src/nmpc_nav_control/NMPCNavControl{,Diff,Omni4,Tric}.cpp are compiled IN PLACE (never copied into this
repository) with the include set of NMPCNavControl.h:10-17 resolved to include/ (acados-named headers of the
boundary) and `acados_solver_{name}.h` of NMPCNavControl{Diff,Omni4,Tric}.h:4, then linked like
CMakeLists.txt:112-114 (libacados_ocp_solver_{name}.so + the acados library, here libnmpc_amd.so) with
-Wl,--no-undefined, so every acados symbol the wrappers use must resolve in this build's libraries.

The only stand-ins are two EMPTY headers generated in a temp dir, itrci_nav/ParametricPath{,Set}.h: the
wrappers include them (NMPCNavControl.h:7-8) but use nothing from them (the un-vendored path library belongs
to the ROS node, out of scope), and the std headers ROS would have pulled in are force-included. The result
is not an oracle and is never run on the GPU: a small driver of our own constructs each wrapper with the
shipped ROS-yaml values (its constructor runs every capsule setter: update_params on stages 0..N-1, lbx/ubx
on 1..N, lbu/ubu on 0..N-1, W on 0..N-1 and W_e on N; NMPCNavControlDiff.cpp:6-74), calls reset_mpc() and
destroys it: host-only capsule code, so it runs here and must log no shim error.
"""
import os
import subprocess

import numpy as np
import pytest

from nmpc_nav_control_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
SRC = os.path.join(REF, "src", "nmpc_nav_control")
WRAPPERS = ["NMPCNavControl.cpp", "NMPCNavControlDiff.cpp", "NMPCNavControlOmni4.cpp", "NMPCNavControlTric.cpp"]
FORCE = ["list", "vector", "string", "cmath"]

pytestmark = pytest.mark.skipif(not os.path.isdir(SRC), reason="the reference tree is not present")

DRIVER = r"""
#include <cstdio>
#include <stdexcept>
#include "nmpc_nav_control/NMPCNavControlDiff.h"
#include "nmpc_nav_control/NMPCNavControlOmni4.h"
#include "nmpc_nav_control/NMPCNavControlTric.h"
using namespace nmpc_nav_control;
int main() {
    const double dt = 1.0 / 40.0;  /* config/nmpc_nav_control.yaml:4 */
    try {
        /* config/nmpc_nav_control.yaml:28-36, 16-25, 39-51 (the values NMPCNavControlROS.cpp:82-160 passes) */
        NMPCNavControlDiff diff(dt, 0.270, 0.1, 1.0, 1.0, {10, 10, 5, 0, 0, 0, 0, 1, 1});
        NMPCNavControlOmni4 omni(dt, 0.535, 0.1, 1.0, 1.0, {10, 10, 5, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1});
        NMPCNavControlTric tric(dt, 0.270, 0.1, 0.5, 1.0, 1.0, -0.785398, 0.785398, 0.261799,
                                {10, 10, 5, 0, 0, 0, 0, 1, 1});
        std::printf("%g %g %g %d %d %d\n", diff.getHorizon(), omni.getHorizon(), tric.getHorizon(),
                    (int)diff.reset_mpc(), (int)omni.reset_mpc(), (int)tric.reset_mpc());
    } catch (const std::exception& e) {
        std::printf("exception %s\n", e.what());
        return 1;
    }
    return 0;
}
"""


def _solver_lib(name):
    return os.path.join(_lib.LIB_DIR, f"libacados_ocp_solver_{name}.so")


def _stubs(tmp_path):
    inc = tmp_path / "stub_include" / "itrci_nav"
    inc.mkdir(parents=True)
    for h in ("ParametricPath.h", "ParametricPathSet.h"):
        (inc / h).write_text(f"/* empty: {h} is included by NMPCNavControl.h:7-8 and unused by the wrappers */\n"
                             "#pragma once\n")
    return str(tmp_path / "stub_include")


def _cxx(tmp_path):
    return ["g++", "-std=c++14", "-fPIC", "-Wall", "-Wno-unused-parameter", "-I", os.path.join(REF, "include"),
            "-I", os.path.join(ROOT, "include"), "-I", _stubs(tmp_path)] + sum((["-include", h] for h in FORCE), [])


def test_reference_constructor_signatures():
    """The driver below uses the constructors as the reference declares them."""
    for h, sig in (("NMPCNavControlDiff.h", "NMPCNavControlDiff(double dt, double dist_b, double tau_v, double v_max, "
                                             "double a_max, std::vector<double> W_diag)"),
                   ("NMPCNavControlTric.h", "NMPCNavControlTric(")):
        assert sig in open(os.path.join(REF, "include", "nmpc_nav_control", h)).read()


def test_reference_wrappers_compile_link_and_construct(built, tmp_path):
    cxx = _cxx(tmp_path)
    objs = []
    for src in WRAPPERS:
        obj = str(tmp_path / src.replace(".cpp", ".o"))
        r = subprocess.run(cxx + ["-c", os.path.join(SRC, src), "-o", obj], capture_output=True, text=True)
        assert r.returncode == 0, f"{src}:\n{r.stderr[-3000:]}"
        objs.append(obj)
    libs = [_lib.LIB_PATH] + [_solver_lib(n) for n in ("diff2amr", "omni4amr", "tric3amr")]
    rpath = f"-Wl,-rpath,{_lib.LIB_DIR}"
    so = str(tmp_path / "libnmpc_nav_control_wrappers.so")
    r = subprocess.run(["g++", "-shared", "-Wl,--no-undefined", "-o", so] + objs + libs + [rpath],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    (tmp_path / "driver.cpp").write_text(DRIVER)
    exe = str(tmp_path / "driver")
    r = subprocess.run(cxx + [str(tmp_path / "driver.cpp"), "-o", exe, so] + libs + [rpath, f"-Wl,-rpath,{tmp_path}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout, r.stderr)
    # the shipped codegen yaml bakes N = ceil(2.0 s * 40 Hz) = 80 for all three models (scripts/*/common.py:5-9)
    assert r.stdout.split() == ["80", "80", "80", "1", "1", "1"], r.stdout
    assert "[nmpc_amd]" not in r.stderr, r.stderr


# ---- the reference's run() executed: oracle/ref_driver.cpp ------------------------------------

@pytest.fixture(scope="module")
def ref_driver(built):
    """oracle/_ref/ref_wrappers_{oracle,device}: the reference's wrappers compiled in place (build() makes them)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    return True


@pytest.mark.parametrize("model", ["diff", "omni4", "tric"])
def test_reference_run_matches_the_oracle_restatement(ref_driver, model):
    """The reference's own run() (NMPCNavControl{Diff,Omni4,Tric}.cpp:82-175 / :96-174 / :93-178), with the fp64
    oracle as its solver, over closed-loop ticks and the edge cases of tests/ref_wrappers.py: everything it sets
    before the solve (x0, yref of every stage, W_e), the iterate the solve starts from, the solve, and the command and
    carried references after it equal the oracle's restatement (oc_prepare, oc_sqp_rti, oc_post) bit for bit."""
    import ref_wrappers as rw
    o = rw.oracle(model)
    robots = rw.closed_loop_robots(o, robots=3, ticks=12) + rw.edge_robots(o)
    recs, stderr = rw.run_driver("oracle", o, robots)
    assert "[nmpc_amd]" not in stderr, stderr
    for seq, rc in zip(robots, recs):
        rw.check_robot(o, seq, rc)
    # the branches were taken: padded lists, the diff hack both ways, +-pi unwraps
    We_scale = {rc["We"][0] / o.prm.W[0] for r in recs for rc in r}
    assert (We_scale == {1.0, 100.0}) if model == "diff" else (We_scale == {1.0}), We_scale
    th = np.concatenate([rc["yref"].reshape(rw.N + 1, o.ny)[:, 2] for r in recs for rc in r])
    assert th.max() > np.pi and th.min() < -np.pi, (th.min(), th.max())


def test_reference_run_detects_a_changed_restatement(ref_driver):
    """The bit-for-bit check is sharp: a one-ulp change of the oracle's control time step (oc_post's carry
    x_ref + u0 dt) is caught in the command."""
    import ref_wrappers as rw
    o = rw.oracle("diff")
    robots = rw.closed_loop_robots(o, robots=1, ticks=3)
    recs, _ = rw.run_driver("oracle", o, robots)
    o.prm.dt_ctrl = np.nextafter(o.prm.dt_ctrl, 1.0)
    with pytest.raises(AssertionError):
        rw.check_robot(o, robots[0], recs[0])
