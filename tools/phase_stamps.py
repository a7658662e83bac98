"""Per-phase cycle stamps of the team kernel from the diagnostic build (make -C nmpc_nav_control_amd/csrc diag,
NMPC_STAMPS): P0 / P1 / F0 / C1F1 / safeguard cycles per IPM iteration and the P1 per-stage sub-phases.
usage (GPU box): python tools/phase_stamps.py [model] [B] [N]"""
import os, sys, ctypes, numpy as np, torch
root = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
os.environ["NMPC_AMD_LIB"] = os.environ.get("STAMPS_LIB") or os.path.join(root, "nmpc_nav_control_amd/lib/diag/libnmpc_amd.so")
sys.path.insert(0, root)
from nmpc_nav_control_amd.fleet import Fleet
from nmpc_nav_control_amd.scenario import DEFAULT_SEED
from nmpc_nav_control_amd._lib import lib
dev = torch.device("cuda", 0)
model = sys.argv[1] if len(sys.argv) > 1 else "diff"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
N = int(sys.argv[3]) if len(sys.argv) > 3 else 40
f = Fleet(model, B, N, DEFAULT_SEED + 1, dev)
for _ in range(int(os.environ.get("STAMP_WARM", "240"))):  # stationary closed loop (bench default)
    f.tick()
torch.cuda.synchronize()
W = 2 + 4 * 64
buf = (ctypes.c_ulonglong * (256 * W))()
L = lib()
L.nmpc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record(); f.solve(); ev1.record(); torch.cuda.synchronize()
print("kernel ms", ev0.elapsed_time(ev1))
if hasattr(L, "nmpc_debug_stamps_pa"):
    pa = (ctypes.c_ulonglong * 256)()
    L.nmpc_debug_stamps_pa.argtypes = [ctypes.c_void_p]
    assert L.nmpc_debug_stamps_pa(pa) == 0
assert L.nmpc_debug_stamps(buf, 256 * W) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(256, W).astype(np.int64)
if hasattr(L, "nmpc_debug_stamps_pa") and pa[0] > st[0, 0]:  # split launches only
    print("P0 stage-parallel part cycles", int(pa[0]) - st[0, 0], "serial pass", st[0, 1] - int(pa[0]))
it = f.qp_iter.cpu().numpy()[::4][:256]
itw = f.qp_iter.cpu().numpy().reshape(-1, 4).max(1)[:256]
ph = {"P1": [], "F0": [], "C1F1": [], "SG": []}
nw = min(256, B // 4)
st = st[:nw]
for w in range(nw):
    n = itw[w]
    for i in range(n):
        base = 2 + 4 * i
        prev = st[w, 1] if i == 0 else st[w, 5 + 4 * (i - 1)]
        ph["P1"].append(st[w, base] - prev)
        ph["F0"].append(st[w, base + 1] - st[w, base])
        ph["C1F1"].append(st[w, base + 2] - st[w, base + 1])
        ph["SG"].append(st[w, base + 3] - st[w, base + 2])
p0 = st[:, 1] - st[:, 0]
print("P0 cycles (mean/max)", p0.mean(), p0.max())
for k, v in ph.items():
    v = np.array(v)
    print(k, "mean %.0f  p50 %.0f  max %.0f  n %d" % (v.mean(), np.median(v), v.max(), len(v)))
tot = st[:, 0].min(), max(st[w, 2 + 4 * itw[w]] for w in range(nw))
print("wave max iters: mean %.1f max %d" % (itw.mean(), itw.max()))
print("total wave cycles (first->last stamp) max", tot[1] - tot[0])

buf2 = (ctypes.c_ulonglong * (256 * 8))()
L.nmpc_debug_stamps_p1.argtypes = [ctypes.c_void_p]
assert L.nmpc_debug_stamps_p1(buf2) == 0
s2 = np.frombuffer(buf2, dtype=np.uint64).reshape(256, 8).astype(np.int64)[:nw]
ok = (s2[:, 7] > s2[:, 0]) & (s2[:, 0] > 0)
d2 = np.diff(s2[ok], axis=1)
names = ["update+resid", "adjoint+terminal..Gd", "pg", "mrow", "cholesky", "rhs+LR+carry", "store"]
print("P1 stage sub-phases (cycles, median over waves):", {n: int(np.median(d2[:, i])) for i, n in enumerate(names)}, "total", int(np.median(s2[ok, 7] - s2[ok, 0])))

buf3 = (ctypes.c_ulonglong * (256 * 64))()
L.nmpc_debug_stamps_c1.argtypes = [ctypes.c_void_p]
assert L.nmpc_debug_stamps_c1(buf3) == 0
s3 = np.frombuffer(buf3, dtype=np.uint64).reshape(256, 64).astype(np.int64)[:nw]
c1, f1 = [], []
for w in range(nw):
    for i in range(min(itw[w], 64)):
        base = 2 + 4 * i
        if s3[w, i] > 0:
            c1.append(s3[w, i] - st[w, base + 1])
            f1.append(st[w, base + 2] - s3[w, i])
print("C1 mean %.0f p50 %.0f   F1 mean %.0f p50 %.0f" % (np.mean(c1), np.median(c1), np.mean(f1), np.median(f1)))
