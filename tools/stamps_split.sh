#!/bin/bash
# P0 / IPM phase cycles (diag build) of a small run-mode batch, split launch vs unsplit (NMPC_AMD_SPLIT_MAX=0).
# usage: gpurun -- 'bash tools/stamps_split.sh <tag> [B] [N]'
TAG=${1:-ss}; B=${2:-4}; N=${3:-80}
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/phase_stamps.py diff $B $N > $OUT/${TAG}_split.txt 2>&1 && \
NMPC_AMD_SPLIT_MAX=0 timeout -k 10 120 python tools/phase_stamps.py diff $B $N > $OUT/${TAG}_nosplit.txt 2>&1
