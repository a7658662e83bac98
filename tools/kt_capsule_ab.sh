#!/bin/bash
# rocprofv3 kernel trace of build/capsule_latency for the product and lib/noov (P0 overlap A/B): the solve kernel alone
cd /tmp && export TMPDIR=/tmp
for v in prod noov; do
  if [ $v = prod ]; then LDP=""; else LDP="$GRAFT_REPO_ROOT/nmpc_nav_control_amd/lib/noov"; fi
  LD_LIBRARY_PATH=$LDP timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/kt_$v -o run --output-format csv -- $GRAFT_REPO_ROOT/build/capsule_latency 300 cold > $GRAFT_REPO_ROOT/gpurun_out/kt_$v.log 2>&1 || exit 1
done
