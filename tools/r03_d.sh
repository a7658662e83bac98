#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03d
timeout -k 10 900 python tools/ab_env.py r03d/wim "metric" w50=NMPC_AMD_WARM_ITER_MAX=50 w10=NMPC_AMD_WARM_ITER_MAX=10 w16=NMPC_AMD_WARM_ITER_MAX=16 cold=NMPC_AMD_WARM=0 --reps=2 || exit 1
timeout -k 10 900 python tools/ab_env.py r03d/wim "omni4 tric diff1024 mixed" w50=NMPC_AMD_WARM_ITER_MAX=50 cold=NMPC_AMD_WARM=0 --reps=1
