#!/bin/bash
# GPU test subsets against the product library and A/B variant libraries (lib/<name>/), one pytest process each.
# Test failures (pytest exit 1) go on to the next library; anything else (a crash, a time limit) stops the script.
# usage: gpurun -- 'bash tools/gpu_tests_ab.sh <tag> "<pytest args>" [<variant> ...]'
TAG=${1:-gab}; ARGS=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out
LIB=$GRAFT_REPO_ROOT/nmpc_nav_control_amd/lib
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for v in prod "$@"; do
  if [ "$v" = prod ]; then unset NMPC_AMD_LIB; else export NMPC_AMD_LIB=$LIB/$v/libnmpc_amd.so; fi
  timeout -k 10 500 python -u -m pytest $ARGS -q -rf --timeout 120 --timeout-method thread > $OUT/${TAG}_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/${TAG}_$v.log | tail -12
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc at $v"; exit $rc; fi
done
