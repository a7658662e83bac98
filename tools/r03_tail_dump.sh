#!/bin/bash
# GPU suite at HEAD and a tick dump of the metric fleet for the CPU tail study (tools/tail_study.py: which robots set
# the per-tick IPM maximum; cold / warm start-point rules in the fp64 emulator).
cd $GRAFT_REPO_ROOT; OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/thr0_tests.log 2>&1; rc=$?
tail -3 $OUT/thr0_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/tick_dump.py metric 260 3 $OUT/tick_dump_metric.npz
