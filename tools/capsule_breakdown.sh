#!/bin/bash
# Single-robot capsule latency breakdown on a GPU box: shim host timings, per-phase stamps (diag build, 4 robots
# N=80) and a rocprofv3 kernel trace of the C capsule driver. usage: gpurun -- bash tools/capsule_breakdown.sh
cd $GRAFT_REPO_ROOT; OUT=$GRAFT_REPO_ROOT/gpurun_out
NMPC_AMD_SHIM_TIMING=1 timeout -k 10 60 build/capsule_latency 100 > $OUT/${TAG:-cb}_cap.json 2> $OUT/${TAG:-cb}_cap.err && \
timeout -k 10 120 python tools/phase_stamps.py diff 4 80 > $OUT/${TAG:-cb}_stamps.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/${TAG:-cb}_prof -o run --output-format csv -- $GRAFT_REPO_ROOT/build/capsule_latency 300 > $OUT/${TAG:-cb}_prof.log 2>&1
