#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03h
timeout -k 10 1100 python tools/ab_env.py r03h/rp "metric diff1024 omni4 tric mixed" rp=NMPC_AMD_ROWPAR_MAX=100000 --reps=1
