#!/bin/bash
# Record stride A/B: the product library (records stored up to the gradient: tric 64 B per lane)
# against lib/rssfull (make variant VARNAME=rssfull VARIANT_FLAGS=-DNMPC_RSS_FULL: the round-3 80-B tric records),
# bench lines interleaved, then the memory PMC passes of both on the tric config.
# usage: gpurun --timeout 1100 -- 'bash tools/rss_ab.sh <tag> [configs]'
TAG=${1:-rss}; shift
CONFIGS=${@:-tric}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
python tools/ab_env.py $TAG "$CONFIGS" rssfull=NMPC_AMD_LIB=@ROOT/nmpc_nav_control_amd/lib/rssfull/libnmpc_amd.so --reps=3; ok $? ab
cd /tmp && export TMPDIR=/tmp
CMD="python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --config tric"
for v in prod rssfull; do
  if [ $v == rssfull ]; then export NMPC_AMD_LIB=$GRAFT_REPO_ROOT/nmpc_nav_control_amd/lib/rssfull/libnmpc_amd.so; fi
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/${TAG}_${v}_pmc2 -o run --output-format csv -- $CMD > $OUT/${TAG}_${v}_pmc2.log 2>&1; ok $? pmc2_$v
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $OUT/${TAG}_${v}_pmc3 -o run --output-format csv -- $CMD > $OUT/${TAG}_${v}_pmc3.log 2>&1; ok $? pmc3_$v
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/${TAG}_${v}_pmc1 -o run --output-format csv -- $CMD > $OUT/${TAG}_${v}_pmc1.log 2>&1; ok $? pmc1_$v
done
echo done
