#!/bin/bash
# GPU suite at HEAD, then a same-box A/B of the initial slack floor (cold thr0 / warm-started robots' thr0_warm).
cd $GRAFT_REPO_ROOT; OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/thr0_tests.log 2>&1; rc=$?
tail -3 $OUT/thr0_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1200 python -u tools/ab_env.py thr0 "metric tric omni4" w10=NMPC_AMD_THR0_WARM=0.1 w05=NMPC_AMD_THR0_WARM=0.05 \
  c50=NMPC_AMD_THR0=0.5,NMPC_AMD_THR0_WARM=0.25 c50w10=NMPC_AMD_THR0=0.5,NMPC_AMD_THR0_WARM=0.1 --reps=2
