#!/bin/bash
# A round's closing collection in one GPU call, ordered so that the bench lines cite this call's own PMC records:
# the GPU parity suite and smoke, the PMC passes per config (tools/pmc.sh), their summaries written into the box's
# profiles/<round>/pmc/ (which bench.py reads), then microbenchmarks, capsule latency, a bench line per config and
# the rocprofv3 kernel trace of the headline bench. Stops at the first failing step. Collect with
# python tools/collect_round.py <tag> <round> <commit>.
# usage: gpurun --timeout 1200 -- 'NMPC_SOURCE_COMMIT=<sha> bash tools/final_profile.sh <tag> <round> [configs]'
#   (the snapshot on the box has no .git; the sha goes into the PMC summaries the bench lines cite)
TAG=${1:-fin}; RND=${2:-r04}; shift 2
CONFIGS=${@:-metric diff1024 omni4 tric mixed}
OUT=$GRAFT_REPO_ROOT/gpurun_out
export NMPC_SOURCE_COMMIT=${NMPC_SOURCE_COMMIT:-unknown}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
declare -A KEY=([metric]=diff_N40_B4096 [diff1024]=diff_N40_B1024 [omni4]=omni4_N40_B4096 [tric]=tric_N60_B8192_g2
                [mixed]=diff_N40_B2731+omni4_N40_B2731+tric_N40_B2730)
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1; ok $? tests
tail -1 $OUT/${TAG}_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1; ok $? smoke
timeout -k 10 60 build/ubench_valu > $OUT/${TAG}_ubench.json 2> $OUT/${TAG}_ubench.err; ok $? ubench
mkdir -p profiles/$RND && cp $OUT/${TAG}_ubench.json profiles/$RND/ubench_valu.json  # the measured basis bench.py reads
for c in $CONFIGS; do
  bash tools/pmc.sh ${TAG}_$c --config $c > $OUT/${TAG}_pmc_$c.log 2>&1; ok $? pmc_$c
  python3 tools/pmc_summary.py $OUT/${TAG}_$c ${KEY[$c]} --round $RND --last 10 --write > /dev/null; ok $? pmc_summary_$c
done
timeout -k 10 60 build/ubench_master > $OUT/${TAG}_master.json; ok $? ubench_master
bash tools/mall_calibration.sh $TAG > $OUT/${TAG}_mall.log 2>&1; ok $? mall
mkdir -p profiles/$RND/pmc && cp $OUT/${TAG}_mall.json profiles/$RND/pmc/mall_calibration.json  # (bench.py reads it)
for mode in warm cold; do
  timeout -k 10 120 build/capsule_latency 300 $mode > $OUT/${TAG}_capsule_c_$mode.json 2> $OUT/${TAG}_capsule_c_$mode.err; ok $? capsule_$mode
done
for c in $CONFIGS; do
  timeout -k 10 300 python bench.py --config $c > $OUT/${TAG}_bench_$c.json 2> $OUT/${TAG}_bench_$c.err; ok $? bench_$c
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $OUT/${TAG}_prof.log 2>&1; ok $? prof
echo done
