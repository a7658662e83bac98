#!/bin/bash
# Round-3 evidence, part B: the driver's bench window (--steps 20 --warmup 5) against the default window on the same
# box (twice each), then PMC passes (tools/pmc.sh, stationary 240-tick closed-loop warm-up) for
# the configs given. usage: gpurun --timeout 1150 -- 'bash tools/profile_r03b.sh <tag> [configs]'
TAG=${1:-p3b}; shift
CONFIGS=${@:-metric diff1024 omni4}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
if [ -z "$NO_WINDOWS" ]; then
  for r in 1 2; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/win_s20_$r.json 2> $OUT/win_s20_$r.err; ok $? s20
    timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/win_s100_$r.json 2> $OUT/win_s100_$r.err; ok $? s100
  done
fi
for c in $CONFIGS; do
  bash tools/pmc.sh $TAG/$c --config $c; ok $? pmc_$c
done
echo "profile_r03b done"
