#!/bin/bash
# row-parallel kernel: GPU tests, capsule latency against the team kernel, phase stamps
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03f; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; grep -E "FAIL|Error" $OUT/tests.log | head -5
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  timeout -k 10 60 build/capsule_latency 300 > $OUT/cap_rowpar$rep.json 2>/dev/null || exit 1
  NMPC_AMD_ROWPAR_MAX=0 timeout -k 10 60 build/capsule_latency 300 > $OUT/cap_team$rep.json 2>/dev/null || exit 1
done
cat $OUT/cap_*.json
timeout -k 10 120 python tools/phase_stamps_rowpar.py diff 4 80 30 > $OUT/rp_stamps.txt 2>&1; cat $OUT/rp_stamps.txt
