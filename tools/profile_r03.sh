#!/bin/bash
# Round-3 evidence on one GPU box, part A: VALU ubench, capsule latency (C driver, row-parallel default and the team
# split launch), the capsule bench with the same-box one-core oracle, one bench line per BASELINE config, a rocprofv3
# kernel-trace of the headline bench, a marker (roctx) + kernel trace of the capsule driver, and phase stamps (diag
# build) of the team kernel at B=4096 / 1024 and of the row-parallel kernel at B=4 N=80. Stops at the first failure.
# Part B (PMC passes per config) is tools/pmc.sh per config. usage: gpurun --timeout 1100 -- 'bash tools/profile_r03.sh <tag>'
TAG=${1:-p3}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 60 build/ubench_valu > $OUT/ubench.json 2> $OUT/ubench.err; ok $? ubench
timeout -k 10 120 build/capsule_latency 300 > $OUT/capsule_c.json 2> $OUT/capsule_c.err; ok $? capsule
NMPC_AMD_ROWPAR_MAX=0 timeout -k 10 120 build/capsule_latency 300 > $OUT/capsule_c_team.json 2> $OUT/capsule_c_team.err; ok $? capsule_team
timeout -k 10 240 python tools/bench_capsule.py > $OUT/capsule_py.json 2> $OUT/capsule_py.err; ok $? capsule_py
for c in metric diff1024 omni4 tric mixed; do
  timeout -k 10 300 python bench.py --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err; ok $? bench_$c; echo "bench $c done"
done
timeout -k 10 120 python tools/phase_stamps.py diff 4096 40 > $OUT/stamps_team_B4096.txt 2>&1; ok $? stamps4096
timeout -k 10 120 python tools/phase_stamps.py diff 1024 40 > $OUT/stamps_team_B1024.txt 2>&1; ok $? stamps1024
timeout -k 10 120 python tools/phase_stamps_rowpar.py diff 4 80 > $OUT/stamps_rowpar_B4_N80.txt 2>&1; ok $? stamps_rowpar
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $OUT/prof.log 2>&1; ok $? prof
timeout -k 10 120 rocprofv3 --marker-trace --kernel-trace --stats -d $OUT/capprof -o run --output-format csv -- $GRAFT_REPO_ROOT/build/capsule_latency 300 > $OUT/capprof.log 2>&1; ok $? capprof
echo "profile_r03 done"
