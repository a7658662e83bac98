#!/bin/bash
# GPU-box round trip: parity tests, smoke, bench, rocprofv3 kernel trace. Stops at the first crash/timeout.
# usage (from this container):  gpurun --timeout 1100 -- 'bash tools/gpu_run.sh <tag> [bench args...]'
TAG=${1:-r}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP rc=$rc"; exit $rc; fi; }
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q > $OUT/${TAG}_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; ok $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; ok $rc
timeout -k 10 400 python bench.py "$@" > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err; rc=$?; echo "bench rc=$rc"; ok $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $OUT/${TAG}_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; ok $rc
