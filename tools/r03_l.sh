#!/bin/bash
# A/B of the current build against lib/base (the previous commit): GPU tests, then bench configs
# warm loads): GPU tests, then same-box A/B against the previous build (lib/base)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03l
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r03l/tests.log 2>&1 || exit $?
timeout -k 10 1000 python tools/ab_env.py r03l/p0b "metric diff1024 omni4 tric" base=NMPC_AMD_LIB=@ROOT/nmpc_nav_control_amd/lib/base/libnmpc_amd.so --reps=2
