#!/bin/bash
# Same-box A/B of the one-robot capsule latency (build/capsule_latency, diff N = 80, the reference node's call
# sequence): the product library and variant libraries (lib/<name>/, resolved through LD_LIBRARY_PATH: the driver
# and the solver library find libnmpc_amd.so by name), cold and warm QP start, the libraries taken in turn per rep.
# usage: gpurun -- 'bash tools/cap_ab.sh <tag> <reps> <variant> [<variant> ...]'
TAG=${1:-cab}; REPS=${2:-2}; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out
LIB=$GRAFT_REPO_ROOT/nmpc_nav_control_amd/lib
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
for v in "$@"; do echo "$v: $(LD_LIBRARY_PATH=$LIB/$v ldd build/capsule_latency | grep libnmpc_amd)"; done
for rep in $(seq 1 $REPS); do
  for v in prod "$@"; do
    for m in cold warm; do
      if [ $v = prod ]; then
        timeout -k 10 60 build/capsule_latency 300 $m > $OUT/${TAG}_${v}_${m}_${rep}.json; ok $? $v
      else
        LD_LIBRARY_PATH=$LIB/$v timeout -k 10 60 build/capsule_latency 300 $m > $OUT/${TAG}_${v}_${m}_${rep}.json; ok $? $v
      fi
      echo "$v $m $rep $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['run_wall_ms_p50'], d['run_wall_ms_mean'], d['qp_iter_mean'])" $OUT/${TAG}_${v}_${m}_${rep}.json)"
    done
  done
done
