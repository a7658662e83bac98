#!/bin/bash
# GPU parity tests on the LDS-ring variant library, then product vs variant bench lines (same box).
# (test_gpu_path is skipped: variant builds compile the path discretizer without its -ffp-contract=off bit-parity flag)
# usage: gpurun -- 'bash tools/ab_ring.sh <tag> [configs]'
TAG=${1:-ring}; shift
CONFIGS=${@:-metric}
OUT=$GRAFT_REPO_ROOT/gpurun_out
V=$GRAFT_REPO_ROOT/nmpc_nav_control_amd/lib/variant/libnmpc_amd.so
cd $GRAFT_REPO_ROOT
NMPC_AMD_LIB=$V timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --deselect tests/test_gpu_path.py --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1; rc=$?; echo "variant tests rc=$rc"; tail -3 $OUT/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for c in $CONFIGS; do
  timeout -k 10 200 python bench.py --config $c --steps 60 --no-cpu-baseline > $OUT/${TAG}_${c}_prod.json 2>/dev/null || exit 1
  NMPC_AMD_LIB=$V timeout -k 10 200 python bench.py --config $c --steps 60 --no-cpu-baseline > $OUT/${TAG}_${c}_ring.json 2>/dev/null || exit 1
  for k in prod ring; do python -c "import json; d=json.load(open('$OUT/${TAG}_${c}_$k.json')); r=d.get('roofline') or {}; print('$c $k', d['value'], d['ms_per_step'], r.get('kernel_ms_mean'), d['qp_iter_mean'], d['qp_iter_max'], d['failed_solves'])"; done
done
