#!/bin/bash
# One GPU round trip: the GPU parity suite, smoke, the default bench line (with the CPU baseline), the C-driven
# one-robot capsule latency (warm and cold IPM start) and the memory-counter calibration. Stops at the first
# failing step. usage: gpurun --timeout 900 -- 'bash tools/gpu_check.sh <tag> [bench args...]'
TAG=${1:-gc}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1; ok $? tests
tail -2 $OUT/${TAG}_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1; ok $? smoke
timeout -k 10 300 python bench.py "$@" > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err; ok $? bench
timeout -k 10 60 build/capsule_latency 300 warm > $OUT/${TAG}_cap_warm.json 2> $OUT/${TAG}_cap_warm.err; ok $? cap_warm
timeout -k 10 60 build/capsule_latency 300 cold > $OUT/${TAG}_cap_cold.json 2> $OUT/${TAG}_cap_cold.err; ok $? cap_cold
bash tools/mall_calibration.sh $TAG; ok $? mall
