"""CPU tests of the path-discretizer oracle (oracle/path_oracle.c, PathDiscretizer.cpp:14-63).

The reference has no tests or fixtures for this path and its segment math lives in the un-vendored
parametric_trajectories_common, so the oracle is pinned by a line-by-line Python restatement
(tests/path_ref.py, bit-exact) and by geometric properties of PathDiscretizer's output; the committed fixture
tests/golden/path_cases.npz (tests/golden/make_golden_path.py) guards it against regressions.
"""
import math
import os

import numpy as np
import pytest

from oracle.oracle import path_discretize
from tests.path_cases import edge_paths, random_paths
from tests.path_ref import PathDiscretizer, TPath

HERE = os.path.dirname(os.path.abspath(__file__))


def ref_run(segs, nseg, nu, period, num_poses, holo):
    out, steps = [], []
    for i in range(len(nseg)):
        pd = PathDiscretizer(period, num_poses, holo)
        poses, st = pd.getNextNPoses([TPath(r) for r in segs[i, :nseg[i]]], float(nu[i]))
        out.append(poses)
        steps.append(st)
    return np.array(out), np.array(steps)


@pytest.mark.parametrize("holo", [False, True])
@pytest.mark.parametrize("period,num_poses", [(0.025, 41), (0.025, 21), (1.0, 5)])
def test_oracle_matches_line_by_line_restatement(period, num_poses, holo):
    segs, nseg, nu = random_paths(40, seed=7 + num_poses)
    got, st = path_discretize(segs, nseg, nu, period, num_poses, holo)
    exp, st_ref = ref_run(segs, nseg, nu, period, num_poses, holo)
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(st, st_ref)


def test_oracle_edge_cases_match_restatement():
    segs, nseg, nu, names = edge_paths()
    for holo in (False, True):
        got, st = path_discretize(segs, nseg, nu, 0.025, 41, holo)
        exp, st_ref = ref_run(segs, nseg, nu, 0.025, 41, holo)
        for i, n in enumerate(names):
            np.testing.assert_array_equal(got[i], exp[i], err_msg=n)
        np.testing.assert_array_equal(st, st_ref)


def test_spacing_is_speed_times_period_on_a_line():
    """Straight line at 0.5 m/s, T = 0.1 s: consecutive poses 5 cm apart within the 1 % threshold plus one
    sub-step (rel = goal / 10)."""
    segs, nseg, nu, names = edge_paths()
    i = names.index("straight")
    out, _ = path_discretize(segs[i:i + 1], nseg[i:i + 1], nu[i:i + 1], 0.1, 20, False)
    p = out[0]
    d = np.hypot(np.diff(p[:, 0]), np.diff(p[:, 1]))
    assert np.all(np.abs(d - 0.05) <= 0.05 * (0.01 + 0.1) + 1e-12)
    assert np.hypot(p[0, 0], p[0, 1]) == pytest.approx(0.05, abs=0.0055)
    np.testing.assert_array_equal(p[:, 2], 0.0)  # heading of the line


def test_padding_with_the_path_end():
    segs, nseg, nu, names = edge_paths()
    out, _ = path_discretize(segs, nseg, nu, 0.025, 41, False)
    for name in ("past_end", "beyond_end", "short_path"):
        p = out[names.index(name)]
        end = p[-1]
        k = np.argmax(np.all(p == end, axis=1))
        assert np.all(p[k:] == end), name
    np.testing.assert_allclose(out[names.index("past_end"), :, :2], [[2.0, 0.0]] * 41)


def test_reverse_segment_adds_pi_and_holonomic_uses_theta_h():
    segs, nseg, nu, names = edge_paths()
    i = names.index("reverse")
    nh, _ = path_discretize(segs[i:i + 1], nseg[i:i + 1], nu[i:i + 1], 0.025, 41, False)
    hol, _ = path_discretize(segs[i:i + 1], nseg[i:i + 1], nu[i:i + 1], 0.025, 41, True)
    np.testing.assert_allclose(nh[0, :, 2], math.atan2(0.5, -1.0) + math.pi)
    np.testing.assert_array_equal(hol[0, :, 2], 0.0)
    np.testing.assert_array_equal(nh[0, :, :2], hol[0, :, :2])


def test_zero_speed_repeats_the_nearest_point():
    segs, nseg, nu, names = edge_paths()
    i = names.index("zero_speed")
    out, steps = path_discretize(segs[i:i + 1], nseg[i:i + 1], nu[i:i + 1], 0.025, 41, False)
    np.testing.assert_allclose(out[0, :, :2], [[0.2, 0.2]] * 41)
    assert steps[0] == 41


def test_points_per_cycle_follow_the_period():
    """num_points_per_cycle = 20 when sample_period >= 1 (PathDiscretizer.cpp:9-10): about twice the steps."""
    segs, nseg, nu = random_paths(8, seed=3, speed=(0.02, 0.03))
    _, s_fast = path_discretize(segs, nseg, np.zeros(8), 0.99, 4, False)
    _, s_slow = path_discretize(segs, nseg, np.zeros(8), 1.0, 4, False)
    assert s_slow.sum() > 1.6 * s_fast.sum()


def test_golden_fixture():
    g = np.load(os.path.join(HERE, "golden", "path_cases.npz"))
    for holo in (0, 1):
        out, steps = path_discretize(g["segs"], g["nseg"], g["nearest_u"], float(g["period"]), int(g["num_poses"]),
                                     bool(holo))
        np.testing.assert_array_equal(out, g[f"poses_{holo}"])
        np.testing.assert_array_equal(steps, g[f"steps_{holo}"])
