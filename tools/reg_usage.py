#!/usr/bin/env python3
"""Register and scratch usage of the solve kernels (gfx950), from the compiler's kernel-resource-usage remarks.

A kernel's waves per SIMD are bounded by its arch + accumulation VGPRs (512 per lane on gfx950): at most 256 lets
two waves share a SIMD, which the segmented row-parallel kernel needs above 256 robots (two waves per robot,
DESIGN.md section 4). Prints one line per kernel instantiation: name, VGPRs, AGPRs, scratch bytes per lane.
usage: python tools/reg_usage.py [sqp_rti_rowpar.hip] [--filter Diff2]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "nmpc_nav_control_amd", "csrc")
# the product flags of csrc/Makefile for the solve kernels (CXXFLAGS + TEAM_FLAGS)
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", f"-I{ROOT}/include", f"-I{CSRC}",
         "-ffp-contract=fast", "-fno-math-errno", "-munsafe-fp-atomics", "-fno-slp-vectorize", "-mllvm",
         "-amdgpu-sched-strategy=max-ilp", "--cuda-device-only", "-c", "-o", os.devnull,
         "-Rpass-analysis=kernel-resource-usage"]


def usage(src="sqp_rti_rowpar.hip"):
    """{kernel mangled name: (vgprs, agprs, scratch bytes per lane)}"""
    res = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, os.path.join(CSRC, src)], capture_output=True, text=True,
                         check=True)
    out, name, cur = {}, None, {}
    for line in res.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name, cur = m.group(1), {}
            continue
        for key, pat in (("v", r"VGPRs: (\d+)"), ("a", r"AGPRs: (\d+)"), ("s", r"ScratchSize \[bytes/lane\]: (\d+)")):
            m = re.search(pat, line)
            if m and name:
                cur[key] = int(m.group(1))
        if name and len(cur) == 3:
            out[name] = (cur["v"], cur["a"], cur["s"])
            name = None
    return out


def main():
    src = next((a for a in sys.argv[1:] if a.endswith(".hip")), "sqp_rti_rowpar.hip")
    flt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else ""
    for k, (v, a, s) in sorted(usage(src).items()):
        if flt in k:
            print(f"{k:90s} vgpr {v:3d} agpr {a:3d} scratch {s:4d} B/lane  waves/SIMD {512 // max(1, (v + a + 7) // 8 * 8)}")


if __name__ == "__main__":
    main()
