#!/bin/bash
# Tail hand-off: its GPU tests, then a same-box A/B of the cap (NMPC_AMD_HAND_CAP) on the bench configs.
# usage: gpurun -- 'bash tools/r03_hand.sh <tag> "<configs>" [variants...]'
TAG=${1:-hand}; CONFIGS=${2:-metric}; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_handoff.py -x -v --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1; rc=$?; echo "tests rc=$rc"
if [ $rc -ne 0 ]; then tail -30 $OUT/${TAG}_tests.log; exit $rc; fi
timeout -k 10 900 python tools/ab_env.py $TAG "$CONFIGS" "$@" --reps=2
