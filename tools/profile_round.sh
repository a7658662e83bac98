#!/bin/bash
# Round profile on one GPU box: VALU ubench, bench line per BASELINE config, rocprofv3 kernel-trace stats of the
# headline bench, PMC passes per config. Stops at the first failing step.
# usage: gpurun --timeout 1100 -- 'bash tools/profile_round.sh <tag> [configs]'
TAG=${1:-prof}; shift
CONFIGS=${@:-metric diff1024 omni4 tric mixed}
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; exit $rc; fi; }
timeout -k 10 60 build/ubench_valu > $OUT/${TAG}_ubench.json 2> $OUT/${TAG}_ubench.err; rc=$?; echo "ubench rc=$rc"; ok $rc
timeout -k 10 120 build/capsule_latency 300 > $OUT/${TAG}_capsule_c.json 2> $OUT/${TAG}_capsule_c.err; rc=$?; echo "capsule rc=$rc"; ok $rc
for c in $CONFIGS; do
  timeout -k 10 300 python bench.py --config $c > $OUT/${TAG}_bench_$c.json 2> $OUT/${TAG}_bench_$c.err; rc=$?; echo "bench $c rc=$rc"; ok $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $OUT/${TAG}_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; ok $rc
cd $GRAFT_REPO_ROOT
for c in $CONFIGS; do
  bash tools/pmc.sh ${TAG}_$c --config $c; ok $?
done
