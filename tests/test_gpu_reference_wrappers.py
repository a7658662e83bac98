"""The reference's own wrappers around the MI355X solve (-m gpu).

oracle/_ref/ref_wrappers_device is NMPCNavControl{,Diff,Omni4,Tric}.cpp compiled in place (on the build host, where
the reference tree is; the GPU box only runs the binary) and linked as the reference's CMakeLists.txt:112-114 links
them, against libacados_ocp_solver_{name}.so + libnmpc_amd.so: every acados call of the reference's run() reaches
this repository's drop-in, and each solve is one launch of the HIP kernel. Over closed-loop and edge-case ticks
(tests/ref_wrappers.py) the test checks:
  * what the reference's run() set (x0, yref of every stage, W_e) equals oc_prepare bit for bit;
  * its command equals oc_post on the u0 the device returned, bit for bit;
  * the device's u0 and x1 are the oracle's SQP-RTI step from the same iterate within the parity tolerance 1e-3
    (acados rule: cold QP start, no infeasibility exit, the capsule defaults).
"""
import os

import numpy as np
import pytest

import ref_wrappers as rw

pytestmark = pytest.mark.gpu
TOL = 1e-3


@pytest.mark.parametrize("model", ["diff", "omni4", "tric"])
def test_reference_run_on_the_device(model):
    assert os.path.exists(rw.EXE["device"]), "oracle/_ref/ref_wrappers_device is built by __graft_entry__.build()"
    o = rw.oracle(model)
    robots = rw.closed_loop_robots(o, robots=3, ticks=10) + rw.edge_robots(o)
    recs, stderr = rw.run_driver("device", o, robots)
    assert "[nmpc_amd]" not in stderr, stderr
    errs = []
    for seq, rc in zip(robots, recs):
        errs += rw.check_robot(o, seq, rc, solve_tol=TOL)
        assert all(r["status"] == 0 for r in rc)
    print(f"{model}: {len(errs)} ticks of the reference's run() on the device, u0 max-abs err {max(errs):.2e}")
