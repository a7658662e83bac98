#!/usr/bin/env python3
"""Copy one tools/profile_round.sh collection from gpurun_out/ into profiles/<round>/ (the files bench.py and the
docs cite), summarising the PMC passes with tools/pmc_summary.py.

usage: python tools/collect_round.py <tag> <round, e.g. r04> <source commit> [--configs "metric diff1024 ..."]
  <tag>_ubench.json          -> ubench_valu.json
  <tag>_mall_{64,2048}/      -> pmc/mall_calibration.json (tools/pmc_summary.py --mall)
  <tag>_capsule_c_<mode>.json -> capsule_latency_c_diff_N80_<mode>.json (mode warm / cold)
  <tag>_bench_<config>.json  -> configs/bench_<config>.json (metric also bench_metric.json)
  <tag>_prof/                -> bench_metric_kernel_stats.csv + bench_metric_kernel_trace_timed.json
  <tag>_<config>_pmc*/       -> pmc/pmc_<config key>.json (last 10 dispatches per kernel)"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
# bench.py's per-config PMC key (bench.py _pmc_key: models, N, batch per GPU, stream groups)
KEYS = {"metric": "diff_N40_B4096", "diff1024": "diff_N40_B1024", "omni4": "omni4_N40_B4096",
        "tric": "tric_N60_B8192_g2", "mixed": "diff_N40_B2731+omni4_N40_B2731+tric_N40_B2730"}


def timed_trace(prof_dir, steps=100):
    """Mean duration of the last `steps` solve-kernel launches of a kernel trace (the bench's timed region)."""
    path = next(iter(glob.glob(os.path.join(prof_dir, "**", "*kernel_trace.csv"), recursive=True)), None)
    if path is None:
        return None
    rows = [r for r in csv.DictReader(open(path)) if "k_sqp_rti" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = rows[-steps:]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in last]
    return {"kernel": last[0]["Kernel_Name"][:80] if last else None, "launches": len(durs),
            "mean_ms": sum(durs) / len(durs) if durs else None, "min_ms": min(durs, default=None),
            "max_ms": max(durs, default=None), "source": os.path.relpath(path, ROOT)}


def main():
    tag, rnd, commit = sys.argv[1:4]
    configs = (sys.argv[sys.argv.index("--configs") + 1].split() if "--configs" in sys.argv
               else ["metric", "diff1024", "omni4", "tric", "mixed"])
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(os.path.join(dst, "configs"), exist_ok=True)

    def cp(src, name):
        s = os.path.join(OUT, src)
        if os.path.exists(s):
            shutil.copy(s, os.path.join(dst, name))
            print("copied", src, "->", name)
        else:
            print("missing", src)

    cp(f"{tag}_ubench.json", "ubench_valu.json")
    for mode in ("warm", "cold"):
        cp(f"{tag}_capsule_c_{mode}.json", f"capsule_latency_c_diff_N80_{mode}.json")
    for c in configs:
        cp(f"{tag}_bench_{c}.json", f"configs/bench_{c}.json")
    cp(f"{tag}_bench_metric.json", "bench_metric.json")
    if os.path.isdir(os.path.join(OUT, f"{tag}_mall_64")):
        res = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), "--mall",
                              os.path.join(OUT, f"{tag}_mall")], capture_output=True, text=True, check=True)
        os.makedirs(os.path.join(dst, "pmc"), exist_ok=True)
        with open(os.path.join(dst, "pmc", "mall_calibration.json"), "w") as fh:
            fh.write(res.stdout)
        print("wrote pmc/mall_calibration.json")
    prof = os.path.join(OUT, f"{tag}_prof")
    stats = next(iter(glob.glob(os.path.join(prof, "**", "*kernel_stats.csv"), recursive=True)), None)
    if stats:
        shutil.copy(stats, os.path.join(dst, "bench_metric_kernel_stats.csv"))
        with open(os.path.join(dst, "bench_metric_kernel_trace_timed.json"), "w") as fh:
            json.dump(timed_trace(prof), fh, indent=1)
        print("wrote kernel stats + timed trace")
    for c in configs:
        if not glob.glob(os.path.join(OUT, f"{tag}_{c}_pmc*")):
            print("no pmc for", c)
            continue
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), os.path.join(OUT, f"{tag}_{c}"),
                        KEYS[c], "--round", rnd, "--last", "10", "--commit", commit, "--write"],
                       check=True, stdout=subprocess.DEVNULL)
        print("wrote pmc", KEYS[c])


if __name__ == "__main__":
    main()
