"""Dump whole closed-loop ticks of a bench fleet for IPM studies on the CPU (tools/warm_study.py): per robot the
solve inputs (snapshot), the warm-start multipliers (LL / LU of the lane records), the warm flag and the GPU's
executed IPM iterations of that tick. usage (GPU box): python tools/tick_dump.py [config] [warm ticks] [dump ticks] [out]"""
import os
import sys

import numpy as np
import torch

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from bench import CONFIGS  # noqa: E402
from nmpc_nav_control_amd.fleet import Fleet  # noqa: E402
from nmpc_nav_control_amd.scenario import DEFAULT_SEED  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "metric"
    cfg = CONFIGS[name]
    warm_ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 260
    dump = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "gpurun_out", f"tick_dump_{name}.npz")
    (m, B), = cfg["models"]
    N = cfg["N"]
    f = Fleet(m, B, N, DEFAULT_SEED + cfg["idx"], torch.device("cuda", 0))
    nu = f.solver.nu
    nv = f.solver.nx + nu
    RS = 16 if (m != "tric" and nu == 2) else 20
    LL = 6 if nu == 2 else 10  # TeamRec<M, SD=true>: L2 layout (NU = 2) / Mehrotra order (NU = 4)
    for _ in range(warm_ticks):
        f.tick()
    wv, sv = f.solver.warm_state()
    keep = {}
    for t in range(dump):
        torch.cuda.synchronize()
        sn = f.snapshot()
        if f.solver.plan_ex(B)["record_layout"] == "wide":
            rec = sv.to_tensor()[0, :B * (N + 1) * 16 * RS].reshape(B, N + 1, 16, RS)
            keep[f"t{t}_lam"] = rec[:, :, :nv, LL:LL + 2].cpu().numpy()
            keep[f"t{t}_warm"] = wv.to_tensor()[0, :B].cpu().numpy()
        else:  # split record planes (tric): no multipliers dumped, every robot replayed cold
            keep[f"t{t}_lam"] = np.zeros((B, N + 1, nv, 2), np.float32)
            keep[f"t{t}_warm"] = np.zeros(B, np.uint8)
        f.solve()
        torch.cuda.synchronize()
        keep[f"t{t}_gpu_iter"] = f.qp_iter.cpu().numpy()
        keep[f"t{t}_gpu_status"] = f.status.cpu().numpy()
        for k, v in sn.items():
            if v is not None:
                keep[f"t{t}_{k}"] = np.asarray(v, np.float32 if v.dtype == np.float64 else v.dtype)
        f.advance()
    np.savez_compressed(out, **keep)
    print("dumped", out, {k: v.shape for k, v in list(keep.items())[:12]})


if __name__ == "__main__":
    main()
