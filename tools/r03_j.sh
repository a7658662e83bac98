#!/bin/bash
# fused fleet statistics: GPU tests of the fleet loop, then a same-box A/B of the metric bench (fused vs torch ops)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03j
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fleet.py > gpurun_out/r03j/tests.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r03j/fused_$r.json 2> gpurun_out/r03j/fused_$r.err || exit $?
  NMPC_FLEET_FUSED_STATS=0 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r03j/torch_$r.json 2> gpurun_out/r03j/torch_$r.err || exit $?
done
