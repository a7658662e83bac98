#!/bin/bash
# A/B of the product library against several variant libraries (make -C nmpc_nav_control_amd/csrc variant
# VARNAME=<name> VARIANT_FLAGS=...), interleaved reps, no CPU baseline.
# usage: gpurun -- 'bash tools/ab_multi.sh <tag> "<configs>" <variant names...>'
TAG=$1; CONFIGS=$2; shift 2
VARS="$@"
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; exit $rc; fi; }
for rep in 1 2; do for c in $CONFIGS; do
  timeout -k 10 200 python bench.py --config $c --steps 60 --no-cpu-baseline > $OUT/${TAG}_${c}_prod_$rep.json 2>/dev/null; ok $?
  for v in $VARS; do
    NMPC_AMD_LIB=$GRAFT_REPO_ROOT/nmpc_nav_control_amd/lib/$v/libnmpc_amd.so timeout -k 10 200 python bench.py --config $c --steps 60 --no-cpu-baseline > $OUT/${TAG}_${c}_${v}_$rep.json 2>/dev/null; ok $?
  done
done; done
python - <<PY
import json, glob
for f in sorted(glob.glob("$OUT/${TAG}_*_*_*.json")):
    d = json.load(open(f)); r = d.get("roofline") or {}
    print(f.split("/")[-1], d["value"], d["ms_per_step"], r.get("kernel_ms_mean"), d["qp_iter_mean"], d["qp_iter_max"], d["failed_solves"])
PY
