#!/bin/bash
# The RCCL calls of the multi-GPU bench on a one-GPU box: torch.distributed.run with one rank and bench.py --dist
# (process group over RCCL at world size 1: the timed region's barriers and MAX all-reduce, and with --gather the
# per-tick command all-gather on the decoupled gather stream). usage: gpurun -- 'bash tools/rccl_check.sh <tag>'
TAG=${1:-rccl}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in metric mixed; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 1 --config $c --steps 20 --warmup 5 --no-cpu-baseline --dist --gather \
      > $OUT/${TAG}_$c.json 2> $OUT/${TAG}_$c.err; ok $? $c
  python -c "import json; d=json.load(open('$OUT/${TAG}_$c.json')); print('$c', d['value'], d['config']['rccl_gather'], d['failed_solves'])"
done
