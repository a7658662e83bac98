# round-6 auxiliary profiles: Python capsule mirror + batch_solve + one-core oracle, RCCL world-1 lines, phase stamps
mkdir -p gpurun_out
OUT=$GRAFT_REPO_ROOT/gpurun_out
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 300 python tools/bench_capsule.py > $OUT/a6_capsule.json 2> $OUT/a6_capsule.err; ok $? capsule
bash tools/rccl_check.sh a6_rccl; ok $? rccl
timeout -k 10 120 python tools/phase_stamps.py diff 4096 40 > $OUT/a6_team_stamps.txt 2>&1; ok $? team_stamps
timeout -k 10 120 python tools/phase_stamps_rowpar.py diff 1024 40 > $OUT/a6_rpstamps_B1024.txt 2>&1; ok $? rp1024
timeout -k 10 120 python tools/phase_stamps_rowpar.py diff 1 80 > $OUT/a6_rpstamps_B1.txt 2>&1; ok $? rp1
echo done
