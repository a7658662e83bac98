"""Memory-counter waits in the gfx950 ISA of the solve kernel, per loop (a development check for the sweep loops).

usage: python tools/isa_waits.py [--kernel Diff2ELb0ELb1ELi1] [--flags "-DFOO"] [--all]
Compiles csrc/sqp_rti_team.hip to device assembly with the product flags (+ --flags), takes one kernel
instantiation and prints, for every loop, its header label, depth, instruction count, the number of fp64 DPP
FMAs (the P1 factorisation loop is the one with ~120) and every s_waitcnt vmcnt in it with its line."""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "nmpc_nav_control_amd", "csrc")
FLAGS = ("--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast -fno-math-errno -munsafe-fp-atomics "
         "-fno-slp-vectorize -mllvm -amdgpu-sched-strategy=max-ilp --cuda-device-only -S").split()


def compile_asm(extra, out):
    cmd = ["/opt/rocm/bin/hipcc", *FLAGS, f"-I{ROOT}/include", f"-I{CSRC}", *extra,
           os.path.join(CSRC, "sqp_rti_team.hip"), "-o", out]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)


def kernel_lines(path, key):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and key in l.split(":")[0] and ":" in l)
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    return lines[start:end]


def loops(lines):
    """(header label, depth, first line, last line) of every loop: a loop spans the blocks annotated with its
    header (``in Loop: Header=...`` / ``Parent Loop ...``), up to the next block label after the last of them
    (the latch may sit above the header in a rotated loop)."""
    labels = [i for i, l in enumerate(lines) if re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", l)]
    out = []
    for i, l in enumerate(lines):
        m = re.match(r"^\.LBB(\d+_\d+):", l)
        nxt = lines[i + 1] if i + 1 < len(lines) else ""
        h = re.search(r"Loop Header: Depth=(\d+)", l + " " + nxt)
        if not (m and h):
            continue
        name = "BB" + m.group(1)
        member = [j for j in labels if re.search(r"(Header=|Parent Loop )" + name + r" ", lines[j]) or j == i]
        first, last = min(member), max(member)
        end = next((j for j in labels if j > last), len(lines)) - 1
        out.append((".LBB" + m.group(1), int(h.group(1)), first, end))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="Diff2ELb0ELb1ELi1")  # diff, not dense, single-direction, run mode
    ap.add_argument("--flags", default="")
    ap.add_argument("--all", action="store_true", help="every loop, not only those with vmcnt waits")
    ap.add_argument("--asm", default="/tmp/isa_waits.s")
    ap.add_argument("--no-compile", action="store_true", help="analyse an existing --asm file")
    a = ap.parse_args()
    if not a.no_compile:
        compile_asm(a.flags.split(), a.asm)
    lines = kernel_lines(a.asm, a.kernel)
    with open(a.asm + ".kernel.s", "w") as fh:  # the kernel alone; the printed line numbers index this file
        fh.write("\n".join(lines))
    for lab, depth, s, e in loops(lines):
        body = lines[s:e + 1]
        f64 = sum("v_fmac_f64_dpp" in l for l in body)
        waits = [(s + j, l.strip()) for j, l in enumerate(body) if "s_waitcnt" in l and "vmcnt" in l]
        insts = sum(1 for l in body if l.startswith("\t") and not l.strip().startswith((";", ".")))
        if waits or a.all:
            print(f"{lab} depth {depth} lines {s}-{e} insts {insts} f64dpp {f64}")
            for ln, w in waits:
                print(f"    {ln:6d} {w}")


if __name__ == "__main__":
    sys.exit(main())
