#!/bin/bash
# Round profile refresh on the GPU box: gpu_run.sh (tests, smoke, metric bench, kernel trace) + PMC passes, then
# bench lines and kernel traces of the other configs and of the path discretizer. Stops at the first crash.
# usage: gpurun --timeout 1200 -- 'bash tools/gpu_profile_all.sh <tag>'
TAG=${1:-r}
OUT=$GRAFT_REPO_ROOT/gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP rc=$rc"; exit $rc; fi; }
bash $GRAFT_REPO_ROOT/tools/gpu_run.sh $TAG || exit $?
bash $GRAFT_REPO_ROOT/tools/pmc.sh $TAG || exit $?
cd $GRAFT_REPO_ROOT
for c in diff1024 omni4 tric mixed; do
  timeout -k 10 300 python bench.py --config $c --steps 50 > $OUT/${TAG}_bench_$c.json 2> $OUT/${TAG}_bench_$c.err; rc=$?; echo "bench $c rc=$rc"; ok $rc
done
timeout -k 10 120 python tools/bench_path.py --B 4096 > $OUT/${TAG}_path_4096.json 2>&1; rc=$?; echo "path rc=$rc"; ok $rc
timeout -k 10 120 python tools/bench_path.py --B 65536 > $OUT/${TAG}_path_65536.json 2>&1; rc=$?; echo "path64k rc=$rc"; ok $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_pathprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_path.py --B 4096 > $OUT/${TAG}_pathprof.log 2>&1; rc=$?; echo "pathprof rc=$rc"; ok $rc
