"""Print the launch plan of a diff N = 80 handle for forced segment counts (NMPC_AMD_SEG): which kernel, waves and
segments a launch of 9 robots takes (nmpc_batch_plan_ex)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nmpc_nav_control_amd._lib import default_params
from nmpc_nav_control_amd.batch import BatchSolver
for S in (8, 10, 16):
    os.environ["NMPC_AMD_SEG"] = str(S)
    h = BatchSolver("diff", 80, 64, params=default_params("diff", 80))
    print(S, h.plan_ex(9))
