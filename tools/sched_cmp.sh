set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_schedule.py -x -q --timeout 120 --timeout-method thread > $O/sched_tests.log 2>&1; rc=$?; echo tests rc=$rc; [ $rc -eq 0 ] || exit $rc
for c in tric mixed; do for s in off sorted interleaved; do
NMPC_AMD_SCHED=$s timeout -k 10 200 python bench.py --config $c --steps 50 --no-cpu-baseline > $O/sched_${c}_$s.json 2>$O/sched_${c}_$s.err; rc=$?; echo $c $s rc=$rc; [ $rc -eq 0 ] || exit $rc
done; done
