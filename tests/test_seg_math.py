"""The segmented Riccati's algebra on the CPU (tools/seg_emu.py, the numpy model of k_sqp_rti_rowpar SEG): the
segment sweeps with a free end costate plus the boundary master give the serial Riccati's Newton direction, with
the device's master form (Q = Y Y', Y = L R^-T from the factor of Phat, DESIGN.md "Segmented Riccati") as well as
with the pivoted solve of X it replaced, on synthetic QPs with barrier weights up to 1e12. Parity unpinned: the
reference holds no solve fixtures; the oracle's serial solve is the check."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import seg_emu  # noqa: E402
import seg_ipm_study  # noqa: E402

from oracle.oracle import Oracle  # noqa: E402


@pytest.mark.parametrize("model,N", [("diff", 40), ("tric", 20), ("omni4", 20)])
@pytest.mark.parametrize("S", [2, 4, 5])
@pytest.mark.parametrize("chol", [False, True])
def test_segmented_direction_equals_serial(model, N, S, chol):
    if N % S:
        pytest.skip("S must divide N")
    o = Oracle(model, N, rule="batched")
    rng = np.random.default_rng(11)
    for _ in range(3):
        G, H, g = seg_emu.make_qp(o, N, rng, 1e6)
        u_ref, x_ref = seg_emu.riccati_serial(G, H, g, o.nx, o.nu, N)
        u, x, gap, _ = seg_emu.riccati_segmented(G, H, g, o.nx, o.nu, N, S, np.float64, chol)
        scale = max(1.0, np.abs(u_ref).max())
        assert np.abs(u - u_ref).max() / scale <= 1e-6
        assert np.abs(x - x_ref).max() / max(1.0, np.abs(x_ref).max()) <= 1e-6
        assert gap <= 1e-6


def test_master_factor_drops_rounding_pivots():
    """The device Cholesky (team_common.hpp rowchol): a pivot at rounding level relative to its column's diagonal
    entry drops the column instead of scaling it by 1 / sqrt(noise)."""
    rng = np.random.default_rng(3)
    H = rng.normal(size=(7, 3))
    A = H @ H.T  # rank 3
    A = (A.astype(np.float32)).astype(np.float64)
    L = seg_emu.psd_chol(A, 0.0, rel=1e-13)
    assert np.abs(L @ L.T - A).max() <= 1e-5 * np.abs(A).max()
    assert np.isfinite(L).all()


def _batched_master(form):
    """seg_ipm_study's batched master forms on one robot: `bidir` (the device's since round 5: backward and dual
    sweeps joined at S / 2) and `scan` (the tree form, emulated only)."""
    def run(segs, nx):
        sb = [{k: np.asarray(sg[k], dtype=np.float64)[None] for k in ("P", "p", "Phi", "Gam", "t")} for sg in segs]
        S = len(sb)
        if form == "bidir":
            s, lam = seg_ipm_study.master_bidir(sb, S, nx, 1)
        else:
            s, lam = seg_ipm_study.master_scan(sb, S, nx, 1)
        return [None if v is None else v[0] for v in s], [None if v is None else v[0] for v in lam]
    return run


@pytest.mark.parametrize("model,N,S", [("diff", 40, 4), ("tric", 20, 4), ("tric", 40, 8), ("omni4", 20, 5),
                                       ("diff", 40, 2)])
@pytest.mark.parametrize("form", ["bidir", "scan"])
def test_bidirectional_and_tree_masters_equal_serial(model, N, S, form):
    """The round-5 master (two sweeps from both ends, joined at m = S / 2; DESIGN.md "Round 5") and the tree form
    give the serial Riccati's direction with fp64 segment sums (the device sums Gam in fp64)."""
    o = Oracle(model, N, rule="batched")
    rng = np.random.default_rng(5)
    for _ in range(3):
        G, H, g = seg_emu.make_qp(o, N, rng, 1e6)
        u_ref, x_ref = seg_emu.riccati_serial(G, H, g, o.nx, o.nu, N)
        u, x, gap, _ = seg_emu.riccati_segmented(G, H, g, o.nx, o.nu, N, S, np.float64,
                                                 master_fn=_batched_master(form))
        scale = max(1.0, np.abs(u_ref).max())
        assert np.abs(u - u_ref).max() / scale <= 1e-6
        assert gap <= 1e-6
