#!/bin/bash
# failure probe + stationary-window check (steps 20 vs 100) + stream groups
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03b
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/fail_probe.py metric 300 40 $OUT/fail_probe.npz > $OUT/fail_probe.txt 2>&1 || exit 1
B() { timeout -k 10 240 python bench.py "$@"; }
B --steps 20 --warmup 5 --no-cpu-baseline > $OUT/metric_s20.json 2>/dev/null || exit 1
B --steps 100 --warmup 10 --no-cpu-baseline > $OUT/metric_s100.json 2>/dev/null || exit 1
B --steps 20 --warmup 5 --no-cpu-baseline > $OUT/metric_s20_b.json 2>/dev/null || exit 1
B --steps 100 --warmup 10 --no-cpu-baseline --groups 2 > $OUT/metric_s100_g2.json 2>/dev/null || exit 1
python - <<PY
import json, glob
for f in sorted(glob.glob("$OUT/*.json")):
    d = json.load(open(f)); r = d.get("roofline") or {}
    print(f.split("/")[-1], d["value"], d["ms_per_step"], r.get("kernel_ms_mean"), d.get("qp_iter"), d["failed_solves"])
PY
tail -20 $OUT/fail_probe.txt
