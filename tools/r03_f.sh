#!/bin/bash
# row-parallel kernel: GPU tests, capsule latency and small-batch benches against the team kernel
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03f; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; grep -E "FAIL|Error" $OUT/tests.log | head -5
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  timeout -k 10 60 build/capsule_latency 300 > $OUT/cap_rowpar$rep.json 2>/dev/null || exit 1
  NMPC_AMD_ROWPAR_MAX=0 timeout -k 10 60 build/capsule_latency 300 > $OUT/cap_team$rep.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --config diff1024 --steps 60 --no-cpu-baseline > $OUT/d1024_rowpar$rep.json 2>/dev/null || exit 1
  NMPC_AMD_ROWPAR_MAX=0 timeout -k 10 200 python bench.py --config diff1024 --steps 60 --no-cpu-baseline > $OUT/d1024_team$rep.json 2>/dev/null || exit 1
done
cat $OUT/cap_*.json
python - <<PY
import json, glob, os
for f in sorted(glob.glob("$OUT/d1024*.json")):
    d = json.load(open(f)); r = d.get("roofline") or {}
    print(os.path.basename(f), d['value'], d['ms_per_step'], r.get('kernel_ms_mean'), d['qp_iter'], d['failed_solves'])
PY
