#!/bin/bash
# GPU parity tests + one bench line per config (no CPU baseline). usage: gpurun -- 'bash tools/quick_check.sh <tag> [configs]'
TAG=${1:-qc}; shift
CONFIGS=${@:-metric}
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; exit $rc; fi; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; ok $rc
for c in $CONFIGS; do
  timeout -k 10 200 python bench.py --config $c --steps 60 --no-cpu-baseline > $OUT/${TAG}_${c}.json 2>/dev/null; ok $?
  python -c "import json; d=json.load(open('$OUT/${TAG}_${c}.json')); r=d.get('roofline') or {}; print('$c', d['value'], d['ms_per_step'], r.get('kernel_ms_mean'), d['qp_iter_mean'], d['qp_iter_max'], d['failed_solves'])"
done
