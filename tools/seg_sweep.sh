#!/bin/bash
# Segment-count sweep on the GPU box: the diff1024 bench line with the segment rows of both waves
# (NMPC_AMD_SEG_ROWS=8) against the default, and the one-robot capsule latency (C driver, cold and warm QP start)
# for forced segment counts NMPC_AMD_SEG=S. Stops at the first failing step.
# usage: gpurun -- 'bash tools/seg_sweep.sh <tag> [S ...]'
TAG=${1:-sweep}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 300 python tools/ab_env.py $TAG "diff1024" seg8=NMPC_AMD_SEG_ROWS=8 --reps=2; ok $? ab
for S in "$@"; do
  for m in cold warm; do
    NMPC_AMD_SEG=$S timeout -k 10 60 build/capsule_latency 300 $m > $OUT/${TAG}_cap_${m}_S$S.json; ok $? cap_$S
    echo "S=$S $m $(cat $OUT/${TAG}_cap_${m}_S$S.json)"
  done
done
