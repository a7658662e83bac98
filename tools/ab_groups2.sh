#!/bin/bash
# Same-box A/B of stream groups, second round: hardware queues, placement, groups 3.
TAG=${1:-abg2}
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT && mkdir -p $OUT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; exit $rc; fi; }
run() {  # name, env, args
  local name=$1; shift
  env $(echo $1 | tr , " ") timeout -k 10 200 python bench.py --no-cpu-baseline ${@:2} > $OUT/${TAG}_$name.json 2> $OUT/${TAG}_$name.err; ok $?
  python3 -c "import json; d=json.load(open('$OUT/${TAG}_$name.json')); print('$name', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'], d['qp_iter_mean'], d['qp_iter_max'])"
}
run metric_g1 X=1 --config metric
run metric_g2 X=1 --config metric --groups 2
run metric_g3 X=1 --config metric --groups 3
run metric_g4_q8 GPU_MAX_HW_QUEUES=8 --config metric --groups 4
run metric_g8_q16 GPU_MAX_HW_QUEUES=16 --config metric --groups 8
run metric_g16_q24 GPU_MAX_HW_QUEUES=24 --config metric --groups 16
run metric_g8s_q16 GPU_MAX_HW_QUEUES=16,NMPC_AMD_SCHED=sorted --config metric --groups 8
run tric_g2s NMPC_AMD_SCHED=sorted --config tric --groups 2
run tric_g4_q8 GPU_MAX_HW_QUEUES=8 --config tric --groups 4
run tric_g8_q16 GPU_MAX_HW_QUEUES=16 --config tric --groups 8
run mixed_dec_s NMPC_AMD_SCHED=sorted --config mixed
run mixed_dec_off NMPC_AMD_SCHED=off --config mixed
run mixed_g2_q8 GPU_MAX_HW_QUEUES=8 --config mixed --groups 2
run mixed_g4_q16 GPU_MAX_HW_QUEUES=16 --config mixed --groups 4
run omni4_g4_q8 GPU_MAX_HW_QUEUES=8 --config omni4 --groups 4
run diff1024_g4_q8 GPU_MAX_HW_QUEUES=8 --config diff1024 --groups 4
