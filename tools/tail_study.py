#!/usr/bin/env python3
"""IPM tail study on dumped stationary bench ticks (tools/tick_dump.py): which robots set the per-tick maximum of
IPM iterations (the launch time at one wave per SIMD), and whether the initial point of cold robots (slack floor
thr0, mu0) or of warm-started ones (their own slack floor) shortens it. Runs the device's single-direction IPM in
the fp64 emulator (tools/ipm_emu.py) with the device's warm rule (the dumped per-robot warm flags; resets cold).
usage: python tools/tail_study.py gpurun_out/tick_dump_metric.npz [--ticks 3] [--n 4096]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--model", default="diff")
    ap.add_argument("--N", type=int, default=40)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--ticks", type=int, default=3)
    ap.add_argument("--kappa", type=float, default=0.2)
    a = ap.parse_args()
    from ipm_emu import Emu
    from warm_study import build
    d = np.load(a.dump)
    single = lambda mu, al, it: np.clip((1 - al) ** 2, 0.01, 0.5)  # noqa: E731
    # (name, cold thr0, cold mu0, warm thr0)
    rules = [("device", 0.25, 1.0, 0.25), ("warm thr0 0.1", 0.25, 1.0, 0.1), ("warm thr0 0.05", 0.25, 1.0, 0.05),
             ("cold thr0 0.5", 0.5, 1.0, 0.25), ("cold thr0 1.0", 1.0, 1.0, 0.25), ("cold mu0 0.1", 0.25, 0.1, 0.25),
             ("cold mu0 10", 0.25, 10.0, 0.25), ("cold thr0 0.5 mu0 0.1", 0.5, 0.1, 0.25)]
    res = {r[0]: [] for r in rules}
    res["gpu"] = []
    for t in range(a.ticks):
        Q, lam, warm, gpu = build(d, t, a.model, a.N, a.n)
        reset = d[f"t{t}_reset"][:len(warm)] if f"t{t}_reset" in d else np.zeros(len(warm), np.int32)
        res["gpu"].append(gpu)
        wst = (np.nan_to_num(lam[..., 0]), np.nan_to_num(lam[..., 1]), a.kappa, 1e3)
        cache = {}
        for name, c_thr, c_mu, w_thr in rules:
            kc, kw = (c_thr, c_mu), w_thr
            if kc not in cache:
                cache[kc] = Emu(Q, thr0=c_thr, mu0=c_mu).solve(single=single)["iters"]
            if ("w", kw) not in cache:
                cache[("w", kw)] = Emu(Q, thr0=w_thr).solve(single=single, warm=wst)["iters"]
            it = np.where(warm, cache[("w", kw)], cache[kc])
            res[name].append(it)
        dev = res["device"][-1]
        top = np.argsort(-dev)[:12]
        print(f"tick {t}: gpu max {gpu.max()} emu max {dev.max()}; corr {np.corrcoef(gpu, dev)[0, 1]:.3f}; "
              f"resets {int(reset.sum())} warm {int(warm.sum())}")
        print("   top robots (emu iters, gpu iters, reset, warm):",
              [(int(dev[i]), int(gpu[i]), int(reset[i]), int(warm[i])) for i in top])
        for lab, m in (("reset", reset != 0), ("cold(no reset)", (~warm) & (reset == 0)), ("warm", warm)):
            if m.any():
                print(f"   {lab:16s} n={int(m.sum()):5d} mean {dev[m].mean():5.2f} max {dev[m].max():3d}")
    print(f"{'rule':24s} {'mean':>6s} {'p99':>5s} {'p99.9':>6s} {'max':>4s}  per-tick max  wave-max mean")
    for name, v in res.items():
        allv = np.concatenate(v)
        wm = np.mean([x[: len(x) // 4 * 4].reshape(-1, 4).max(1).mean() for x in v])
        print(f"{name:24s} {allv.mean():6.2f} {np.percentile(allv, 99):5.1f} {np.percentile(allv, 99.9):6.1f} "
              f"{allv.max():4d}  {[int(x.max()) for x in v]}  {wm:5.2f}")


if __name__ == "__main__":
    main()
