#!/bin/bash
# same-box A/B under the stationary loop: stream groups and warm-start kappa per config
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03e; mkdir -p $OUT
run() { local tag=$1; shift; timeout -k 10 200 python bench.py --steps 60 --no-cpu-baseline "$@" > $OUT/$tag.json 2>/dev/null || { echo "STOP $tag"; exit 1; }; }
for rep in 1 2; do
  run metric_g1_$rep --config metric
  run metric_g2_$rep --config metric --groups 2
  run tric_g1_$rep --config tric --groups 1
  run tric_g2_$rep --config tric
  run omni4_g1_$rep --config omni4
  run omni4_g2_$rep --config omni4 --groups 2
  NMPC_AMD_WARM_KAPPA=0.05 run metric_k005_$rep --config metric
  NMPC_AMD_WARM_KAPPA=0.05 run omni4_k005_$rep --config omni4
  NMPC_AMD_WARM_KAPPA=0.05 run tric_k005_$rep --config tric
done
python - <<PY
import json, glob, os
for f in sorted(glob.glob("$OUT/*.json")):
    d = json.load(open(f)); r = d.get("roofline") or {}
    print(f"{os.path.basename(f)[:-5]:18s} {d['value']:>11.1f} {d['ms_per_step']:.4f} {r.get('kernel_ms_mean')} {d['qp_iter']['mean']:.2f} {d['qp_iter']['max']} {d['failed_solves']}")
PY
