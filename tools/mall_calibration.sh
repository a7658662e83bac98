#!/bin/bash
# Calibrate the L2 memory-side request counters (bench.py roofline.hbm): tools/ubench_mall.hip streams a table
# that stays resident in the 256 MiB Infinity Cache (64 MiB x 16 reps) and one that cannot (2 GiB x 2 reps), each
# under one rocprofv3 --pmc pass of the four TCC_EA0 request counters; tools/pmc_summary.py --mall turns the two
# into requests per byte read and the verdict (does TCC_EA0_RDREQ_DRAM exclude Infinity-Cache hits?).
# usage: gpurun -- 'bash tools/mall_calibration.sh <tag>'   -> gpurun_out/<tag>_mall.json
TAG=${1:-mall}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; exit $rc; fi; }
for spec in "64 16" "2048 2"; do
  set -- $spec
  timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum \
      -d $OUT/${TAG}_mall_$1 -o run --output-format csv -- $GRAFT_REPO_ROOT/build/ubench_mall $1 $2 3 \
      > $OUT/${TAG}_mall_$1.log 2>&1; rc=$?; echo "mall $1 MiB rc=$rc"; ok $rc
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py --mall $OUT/${TAG}_mall > $OUT/${TAG}_mall.json; ok $?
cat $OUT/${TAG}_mall.json
