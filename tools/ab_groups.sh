#!/bin/bash
# Same-box A/B of stream groups (FleetNode groups / decoupled ticks) on the bench configs.
# usage: gpurun -- 'bash tools/ab_groups.sh <tag>'
TAG=${1:-abg}
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT && mkdir -p $OUT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; exit $rc; fi; }
run() {  # name, env, args
  local name=$1; shift
  env $1 timeout -k 10 200 python bench.py --no-cpu-baseline ${@:2} > $OUT/${TAG}_$name.json 2> $OUT/${TAG}_$name.err; ok $?
  python3 -c "import json; d=json.load(open('$OUT/${TAG}_$name.json')); print('$name', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'], d['qp_iter_mean'], d['qp_iter_max'])"
}
for rep in 1 2; do
  run metric_g1_$rep X=1 --config metric
  run metric_g2_$rep X=1 --config metric --groups 2
  run metric_g4_$rep X=1 --config metric --groups 4
  run metric_g8_$rep X=1 --config metric --groups 8
  run metric_g4s_$rep NMPC_AMD_SCHED=sorted --config metric --groups 4
  run metric_g8s_$rep NMPC_AMD_SCHED=sorted --config metric --groups 8
done
run mixed_joined X=1 --config mixed --joined
run mixed_dec X=1 --config mixed
run mixed_dec_g2 X=1 --config mixed --groups 2
run tric_g1 X=1 --config tric
run tric_g2 X=1 --config tric --groups 2
run tric_g4s NMPC_AMD_SCHED=sorted --config tric --groups 4
run omni4_g1 X=1 --config omni4
run omni4_g4 X=1 --config omni4 --groups 4
run diff1024_g1 X=1 --config diff1024
run diff1024_g4 X=1 --config diff1024 --groups 4
