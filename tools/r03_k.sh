#!/bin/bash
# fleet-sim kernel with 16 lanes per robot: fleet tests, metric bench twice, kernel stats
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03k
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fleet.py tests/test_gpu_sim_regress.py > gpurun_out/r03k/tests.log 2>&1 || exit $?
for r in 1 2; do timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r03k/bench_$r.json 2> gpurun_out/r03k/bench_$r.err || exit $?; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03k/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 30 > $GRAFT_REPO_ROOT/gpurun_out/r03k/prof.log 2>&1
