#!/bin/bash
# Round profile on one GPU box: VALU and memory-counter microbenchmarks, the one-robot capsule latency (warm and cold
# IPM start), a bench line per BASELINE config, the rocprofv3 kernel trace of the headline bench, and the PMC passes
# per config (tools/pmc.sh). Stops at the first failing step. Collect with tools/collect_round.sh.
# usage: gpurun --timeout 1200 -- 'bash tools/profile_round.sh <tag> [configs]'
#        PART=main (everything but the PMC passes) or PART=pmc (only them) splits it over two calls
TAG=${1:-prof}; shift
CONFIGS=${@:-metric diff1024 omni4 tric mixed}
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
PART=${PART:-all}
if [ "$PART" != pmc ]; then
timeout -k 10 60 build/ubench_valu > $OUT/${TAG}_ubench.json 2> $OUT/${TAG}_ubench.err; ok $? ubench
bash tools/mall_calibration.sh $TAG > $OUT/${TAG}_mall.log 2>&1; ok $? mall
for mode in warm cold; do
  timeout -k 10 120 build/capsule_latency 300 $mode > $OUT/${TAG}_capsule_c_$mode.json 2> $OUT/${TAG}_capsule_c_$mode.err; ok $? capsule_$mode
done
for c in $CONFIGS; do
  timeout -k 10 300 python bench.py --config $c > $OUT/${TAG}_bench_$c.json 2> $OUT/${TAG}_bench_$c.err; ok $? bench_$c
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $OUT/${TAG}_prof.log 2>&1; ok $? prof
fi
cd $GRAFT_REPO_ROOT
[ "$PART" == main ] && { echo done; exit 0; }
for c in $CONFIGS; do
  bash tools/pmc.sh ${TAG}_$c --config $c > $OUT/${TAG}_pmc_$c.log 2>&1; ok $? pmc_$c
done
echo done
