#!/bin/bash
# A/B of the product library against lib/variant (make -C nmpc_nav_control_amd/csrc variant VARIANT_FLAGS=...):
# parity tests on the product library, then alternating bench runs of both. usage: gpurun -- 'bash tools/ab_bench.sh <tag> [configs]'
TAG=${1:-ab}; shift
CONFIGS=${@:-metric}
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; exit $rc; fi; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; ok $rc
for c in $CONFIGS; do for rep in 1 2; do
  timeout -k 10 200 python bench.py --config $c --steps 60 --no-cpu-baseline > $OUT/${TAG}_${c}_prod$rep.json 2>/dev/null; ok $?
  NMPC_AMD_LIB=$GRAFT_REPO_ROOT/nmpc_nav_control_amd/lib/${VARNAME:-variant}/libnmpc_amd.so timeout -k 10 200 python bench.py --config $c --steps 60 --no-cpu-baseline > $OUT/${TAG}_${c}_var$rep.json 2>/dev/null; ok $?
done; done
python - <<PY
import json, glob
for f in sorted(glob.glob("$OUT/${TAG}_*_*.json")):
    d = json.load(open(f)); r = d.get("roofline") or {}
    print(f.split("/")[-1], d["value"], d["ms_per_step"], r.get("kernel_ms_mean"), d["qp_iter_mean"], d["qp_iter_max"], d["failed_solves"])
PY
