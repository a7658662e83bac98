"""Find the robots of a bench fleet whose solve fails (status != 0) or runs long, and save their pre-tick state for
a CPU replay (oracle / emulator). usage (GPU box): python tools/fail_probe.py [config] [ticks] [min_iter] [out.npz]"""
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
    cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "metric"]
    ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    min_it = int(sys.argv[3]) if len(sys.argv) > 3 else 35
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "gpurun_out", "fail_probe.npz")
    (m, B), = cfg["models"]
    f = Fleet(m, B, cfg["N"], DEFAULT_SEED + cfg["idx"], torch.device("cuda", 0))
    res = torch.zeros(3, B, device="cuda")
    keep = {}
    wv, sv = f.solver.warm_state()
    nx, nu = f.solver.nx, f.solver.nu
    RS = 16 if (m != "tric" and nu == 2) else 20  # TeamRec<M, SD>::RS of the product layout
    for t in range(ticks):
        torch.cuda.synchronize()
        sn = f.snapshot()
        scratch = sv.to_tensor()  # the records before this solve (warm multipliers)
        warm = wv.to_tensor()
        f.solver.run(f.pose, f.vel, f.traj, steer=f.steer, traj_len=f.tlen, reset=f.reset, cmd=f.cmd, u0=f.u0,
                     status=f.status, qp_iter=f.qp_iter, qp_res=res, stream=f.stream)
        torch.cuda.synchronize()
        st, it = f.status.cpu().numpy(), f.qp_iter.cpu().numpy()
        bad = np.nonzero((st != 0) | (it >= min_it))[0]
        for i in bad:
            key = f"t{t}_r{i}"
            keep[key + "_status"] = np.array([st[i], it[i]])
            keep[key + "_res"] = res[:, i].cpu().numpy()
            for k, v in sn.items():
                if v is not None:
                    keep[key + "_" + k] = np.asarray(v[i])
            blk = (cfg["N"] + 1) * 16 * RS
            keep[key + "_records"] = scratch[0, i * blk:(i + 1) * blk].cpu().numpy().reshape(cfg["N"] + 1, 16, RS)
            keep[key + "_warm"] = np.array([int(warm[0, i])])
            print(f"tick {t} robot {i}: status {st[i]} qp_iter {it[i]} res {res[:, i].cpu().numpy()} "
                  f"reset {sn['reset'][i] if sn['reset'] is not None else None}", flush=True)
        f.advance()
    np.savez(out, **keep)


if __name__ == "__main__":
    main()
