#!/bin/bash
# One GPU round trip for a latency-kernel change: the GPU suite, same-box A/B bench lines of the metric (team
# kernel) and diff1024 (segmented row-parallel kernel) configs against variant libraries, the C-driven one-robot
# capsule latency (cold / warm QP start) of the product library and of the first variant, and the row-parallel
# kernel's phase stamps (diag build, lib/diag). Stops at the first failing step.
# usage: gpurun -- 'bash tools/ab_latency.sh <tag> <variant> [<variant> ...]'   (variant = a lib/<name>/ directory)
TAG=${1:-abl}; shift
VARS=("$@")
OUT=$GRAFT_REPO_ROOT/gpurun_out
LIB=$GRAFT_REPO_ROOT/nmpc_nav_control_amd/lib
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1; ok $? tests
tail -2 $OUT/${TAG}_tests.log
SPECS=()
for v in "${VARS[@]}"; do SPECS+=("$v=NMPC_AMD_LIB=@ROOT/nmpc_nav_control_amd/lib/$v/libnmpc_amd.so"); done
timeout -k 10 400 python tools/ab_env.py $TAG "metric diff1024" "${SPECS[@]}" --reps=2; ok $? ab
for m in cold warm; do
  timeout -k 10 60 build/capsule_latency 300 $m > $OUT/${TAG}_cap_${m}_prod.json; ok $? cap_prod
  if [ ${#VARS[@]} -gt 0 ]; then
    LD_LIBRARY_PATH=$LIB/${VARS[0]} timeout -k 10 60 build/capsule_latency 300 $m > $OUT/${TAG}_cap_${m}_${VARS[0]}.json
    ok $? cap_var
  fi
done
tail -n 2 $OUT/${TAG}_cap_*.json
if [ -f $LIB/diag/libnmpc_amd.so ]; then
  timeout -k 10 120 python tools/phase_stamps_rowpar.py diff 1024 40 > $OUT/${TAG}_rpstamps_B1024.txt 2>&1; ok $? stamps1024
  timeout -k 10 120 python tools/phase_stamps_rowpar.py diff 1 80 > $OUT/${TAG}_rpstamps_B1.txt 2>&1; ok $? stamps1
  tail -n 8 $OUT/${TAG}_rpstamps_*.txt
fi
