#!/bin/bash
# round-3 first GPU pass: the -m gpu suite, then the stationary bench at two windows and same-box A/Bs of the
# round-3 kernel changes (lib/dzrec: DZ back in the lane record; lib/mstore: that + masked P1 stores).
# usage (GPU box): bash tools/r03_a.sh
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03a
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
LIB=$GRAFT_REPO_ROOT/nmpc_nav_control_amd/lib
B() { timeout -k 10 240 python bench.py "$@"; }
B --steps 20 --warmup 5 > $OUT/metric_s20.json 2> $OUT/metric_s20.err || exit 1
for rep in 1 2; do
  B --steps 100 --warmup 10 --no-cpu-baseline > $OUT/metric_s100_prod$rep.json 2>/dev/null || exit 1
  NMPC_AMD_LIB=$LIB/dzrec/libnmpc_amd.so B --steps 100 --warmup 10 --no-cpu-baseline > $OUT/metric_s100_dzrec$rep.json 2>/dev/null || exit 1
  NMPC_AMD_LIB=$LIB/mstore/libnmpc_amd.so B --steps 100 --warmup 10 --no-cpu-baseline > $OUT/metric_s100_mstore$rep.json 2>/dev/null || exit 1
done
B --steps 20 --warmup 5 --no-cpu-baseline > $OUT/metric_s20_b.json 2>/dev/null || exit 1
B --steps 100 --warmup 10 --no-cpu-baseline --no-renew > $OUT/metric_s100_norenew.json 2>/dev/null || exit 1
B --steps 100 --warmup 10 --no-cpu-baseline --groups 2 > $OUT/metric_s100_g2.json 2>/dev/null || exit 1
python - <<PY
import json, glob
for f in sorted(glob.glob("$OUT/*.json")):
    d = json.load(open(f)); r = d.get("roofline") or {}
    print(f.split("/")[-1], d["value"], d["ms_per_step"], r.get("kernel_ms_mean"), d.get("qp_iter"), d["failed_solves"], d.get("u0_max_abs_err"))
PY
