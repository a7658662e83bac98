"""Per-phase cycles of the row-parallel kernel (diag build, NMPC_STAMPS): P0a / P0b and per IPM iteration the
phases A (stage-parallel update), B (serial Riccati), C (serial forward), D (stage-parallel step).
usage (GPU box): python tools/phase_stamps_rowpar.py [model] [B] [N] [ticks]"""
import ctypes
import os
import sys

import numpy as np
import torch

root = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
os.environ["NMPC_AMD_LIB"] = os.environ.get("STAMPS_LIB") or os.path.join(root, "nmpc_nav_control_amd/lib/diag/libnmpc_amd.so")
sys.path.insert(0, root)
from nmpc_nav_control_amd._lib import lib  # noqa: E402
from nmpc_nav_control_amd.fleet import Fleet  # noqa: E402
from nmpc_nav_control_amd.scenario import DEFAULT_SEED  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "diff"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
N = int(sys.argv[3]) if len(sys.argv) > 3 else 80
T = int(sys.argv[4]) if len(sys.argv) > 4 else 30
f = Fleet(model, B, N, DEFAULT_SEED + 1, torch.device("cuda", 0))
for _ in range(T):
    f.tick()
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
f.solve()
ev1.record()
torch.cuda.synchronize()
W = 3 + 4 * 64
buf = (ctypes.c_ulonglong * (256 * W))()
L = lib()
L.nmpc_debug_stamps_rowpar.argtypes = [ctypes.c_void_p]
assert L.nmpc_debug_stamps_rowpar(buf) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(256, W).astype(np.int64)[:min(B, 256)]  # robots 0..255 stamped
it = f.qp_iter.cpu().numpy()[:min(B, 256)]
print("kernel ms", ev0.elapsed_time(ev1), "qp_iter", it.tolist())
# serial kernel: A, B (Riccati), C (forward), D; segmented (NMPC_AMD_SEG > 0): A, B (segment sweeps), M (master),
# C+D (segment forward + step); the segmented kernel decides to stop before its phase B
plan = f.solver.plan(B)  # (kernel, waves per robot, segments) of this launch
print("plan", plan)
seg = plan[2] > 0
names = ["A", "Bseg", "M", "CD"] if seg else ["A", "B", "C", "D"]
ph = {n: [] for n in names}
for b in range(min(B, 256)):
    for i in range(int(it[b]) + 1):
        base = 3 + 4 * i
        prev = st[b, 2] if i == 0 else st[b, base - 1]
        ph[names[0]].append(st[b, base] - prev)
        if not seg or i < it[b]:
            ph[names[1]].append(st[b, base + 1] - st[b, base])
        if i < it[b]:
            ph[names[2]].append(st[b, base + 2] - st[b, base + 1])
            ph[names[3]].append(st[b, base + 3] - st[b, base + 2])
print("P0a cycles", (st[:, 1] - st[:, 0]).tolist(), "P0b", (st[:, 2] - st[:, 1]).tolist())
for k, v in ph.items():
    v = np.array(v)
    print(k, "mean %.0f p50 %.0f max %.0f n %d per stage %.0f" % (v.mean(), np.median(v), v.max(), len(v), v.mean() / (N + 1)))

# the segment master's parts (diag builds with g_rp_mstamps): per iteration deltas
if seg and hasattr(L, "nmpc_debug_mstamps_rowpar"):
    mb = (ctypes.c_ulonglong * (256 * 64 * 8))()
    L.nmpc_debug_mstamps_rowpar.argtypes = [ctypes.c_void_p]
    if L.nmpc_debug_mstamps_rowpar(mb) == 0:
        ms = np.frombuffer(mb, dtype=np.uint64).reshape(256, 64, 8).astype(np.int64)[:min(B, 256)]
        parts = {"sweeps (rows 0 / 1)": (0, 1), "join": (1, 4), "propagations": (4, 5), "to the barrier": (5, 7),
                 "total": (0, 7)}
        for name, (a, b) in parts.items():
            v = np.array([ms[r, i, b] - ms[r, i, a] for r in range(ms.shape[0]) for i in range(int(it[r]))
                          if ms[r, i, a] > 0 and ms[r, i, b] > 0])
            if len(v):
                print("  master %-20s mean %7.0f p50 %7.0f n %d" % (name, v.mean(), np.median(v), len(v)))

# per boundary step of the backward sweep (diag builds with g_rp_sstamps): cycles between consecutive steps
if seg and hasattr(L, "nmpc_debug_sstamps_rowpar") and hasattr(L, "nmpc_debug_mstamps_rowpar"):
    sb = (ctypes.c_ulonglong * (256 * 64 * 16))()
    L.nmpc_debug_sstamps_rowpar.argtypes = [ctypes.c_void_p]
    if L.nmpc_debug_sstamps_rowpar(sb) == 0:
        ss = np.frombuffer(sb, dtype=np.uint64).reshape(256, 64, 16).astype(np.int64)[:min(B, 256)]
        S_ = plan[2]
        m_ = 0 if os.environ.get("SEQM") else S_ // 2
        steps = list(range(S_ - 2, m_ - 1, -1))  # the backward sweep's boundaries, in order
        rows = []
        for r in range(ss.shape[0]):
            for i in range(int(it[r])):
                t0 = ms[r, i, 0]
                prev, d = t0, []
                for b in steps:
                    d.append(ss[r, i, b] - prev)
                    prev = ss[r, i, b]
                rows.append(d)
        if rows:
            a = np.array(rows)
            print("  backward sweep per step (boundary order %s): mean %s" % (steps, np.round(a.mean(axis=0)).astype(int).tolist()))
