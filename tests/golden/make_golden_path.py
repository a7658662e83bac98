"""Regenerate tests/golden/path_cases.npz: seeded path cases (tests/path_cases.py) and the oracle's
getNextNPoses output for them (oracle/path_oracle.c). Run from the repo root: python tests/golden/make_golden_path.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle.oracle import path_discretize  # noqa: E402
from tests.path_cases import edge_paths, random_paths  # noqa: E402

segs, nseg, nu = random_paths(24, seed=2024, max_segs=3)
es, en, eu, _ = edge_paths()
segs = np.concatenate([segs, es])
nseg = np.concatenate([nseg, en])
nu = np.concatenate([nu, eu])
period, num_poses = 0.025, 41
out = dict(segs=segs, nseg=nseg, nearest_u=nu, period=period, num_poses=num_poses)
for holo in (0, 1):
    out[f"poses_{holo}"], out[f"steps_{holo}"] = path_discretize(segs, nseg, nu, period, num_poses, bool(holo))
np.savez_compressed(os.path.join(ROOT, "tests", "golden", "path_cases.npz"), **out)
print("wrote", len(nseg), "cases")
