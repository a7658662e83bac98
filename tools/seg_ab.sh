#!/bin/bash
# Segmented Riccati (k_sqp_rti_rowpar SEG) on the GPU box: its parity tests, the C-driven one-robot capsule latency
# (N = 80, warm and cold IPM start) for several segment counts, and same-box bench A/B of the configs where the team
# kernel leaves SIMDs idle (diff1024) or where one wave per robot might pay (metric), row-parallel kernel allowed up to
# the batch size. Stops at the first failing step.
# usage: gpurun --timeout 1100 -- 'bash tools/seg_ab.sh <tag> [segs] [configs]'
TAG=${1:-seg}
SEGS=${2:-"0 4 5 8"}
CONFIGS=${3-"diff1024 metric"}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1; ok $? tests
tail -1 $OUT/${TAG}_tests.log
for S in $SEGS; do
  for mode in warm cold; do
    NMPC_AMD_SEG=$S timeout -k 10 60 build/capsule_latency 300 $mode > $OUT/${TAG}_cap_s${S}_$mode.json 2> $OUT/${TAG}_cap_s${S}_$mode.err; ok $? cap_$S
    echo "S=$S $mode $(cat $OUT/${TAG}_cap_s${S}_$mode.json)"
  done
done
# rp4: every robot on the segmented kernel (one wave each, 4 segments); rp0: the serial row-parallel phases;
# (VARIANTS overrides the list, REPS the repetitions)
[ -z "$CONFIGS" ] && exit 0
python tools/ab_env.py $TAG "$CONFIGS" ${VARIANTS:-rp4=NMPC_AMD_ROWPAR_MAX=8192,NMPC_AMD_SEG=4 rp0=NMPC_AMD_ROWPAR_MAX=8192,NMPC_AMD_SEG=0} \
    --reps=${REPS:-2}; ok $? ab
