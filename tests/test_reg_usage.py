"""Register budget of the segmented row-parallel kernel (tools/reg_usage.py, the compiler's resource remarks for the
product flags): above 256 robots it runs two waves per robot, two robots' waves per SIMD, which needs at most 256
arch + accumulation VGPRs per lane (the W = 1 and W = 2 instantiations; W = 4 runs one wave per SIMD). Round 4 lost a
third of diff1024's rate (1.65 -> 1.11 M it/s) when a change pushed the kernel to 256 + 4 AGPRs. omni4 (357) is
routed to the team kernel above 256 robots (nmpc_batch.cpp)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_segmented_kernels_fit_two_waves_per_simd():
    import reg_usage
    use = reg_usage.usage("sqp_rti_rowpar.hip")
    seg = {k: v for k, v in use.items() if "k_sqp_rti_rowpar" in k and "ELb1E" in k}
    assert len(seg) == 9, sorted(seg)  # 3 models x W in {1, 2, 4}
    for k, (v, a, _) in seg.items():
        if "Omni4" in k:
            continue
        if "ELi4ELb1E" in k:  # W = 4: launches of at most 256 robots, one block per CU (one wave per SIMD)
            assert v + a <= 512, (k, v, a)
            continue
        assert v + a <= 256, (k, v, a)
