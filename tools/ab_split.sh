#!/bin/bash
# Split launches (one wave per robot for small batches) A/B: GPU parity tests on the product library, the C capsule
# driver (diff N=80, one robot) with and without splitting, and the bench configs against lib/base (the previous
# kernel, make variant VARNAME=base). usage: gpurun -- 'bash tools/ab_split.sh <tag> [configs]'
TAG=${1:-sp}; shift
CONFIGS=${@:-metric diff1024}
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; exit $rc; fi; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; ok $rc
for rep in 1 2; do
  timeout -k 10 60 build/capsule_latency 300 > $OUT/${TAG}_cap_split$rep.json 2>/dev/null; ok $?
  NMPC_AMD_SPLIT_MAX=0 timeout -k 10 60 build/capsule_latency 300 > $OUT/${TAG}_cap_nosplit$rep.json 2>/dev/null; ok $?
  echo "split   $(cat $OUT/${TAG}_cap_split$rep.json)"
  echo "nosplit $(cat $OUT/${TAG}_cap_nosplit$rep.json)"
done
for c in $CONFIGS; do for rep in 1 2; do
  timeout -k 10 200 python bench.py --config $c --steps 60 --no-cpu-baseline > $OUT/${TAG}_${c}_prod$rep.json 2>/dev/null; ok $?
  NMPC_AMD_LIB=$GRAFT_REPO_ROOT/nmpc_nav_control_amd/lib/base/libnmpc_amd.so timeout -k 10 200 python bench.py --config $c --steps 60 --no-cpu-baseline > $OUT/${TAG}_${c}_base$rep.json 2>/dev/null; ok $?
done; done
python - <<PY
import json, glob
for f in sorted(glob.glob("$OUT/${TAG}_*_*[0-9].json")):
    if "_cap_" in f: continue
    d = json.load(open(f)); r = d.get("roofline") or {}
    print(f.split("/")[-1], d["value"], d["ms_per_step"], r.get("kernel_ms_mean"), d["qp_iter_mean"], d["qp_iter_max"], d["failed_solves"])
PY
