#!/bin/bash
# Same-box A/B of the one-robot capsule latency (build/capsule_latency, diff N = 80, the reference node's call
# sequence): the product library and variant libraries (lib/<name>/, resolved through LD_LIBRARY_PATH: the driver
# and the solver library find libnmpc_amd.so by name), cold and warm QP start, the libraries taken in turn per rep.
# usage: gpurun -- 'bash tools/cap_ab.sh <tag> <reps> <variant> [<variant> ...]'
#   a variant is a lib/<name>/ directory, or <name>@VAR=value: the product library with that environment setting
TAG=${1:-cab}; REPS=${2:-2}; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out
LIB=$GRAFT_REPO_ROOT/nmpc_nav_control_amd/lib
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
for v in "$@"; do
  case $v in *@*) echo "$v: product library, ${v#*@}";;
             *) echo "$v: $(LD_LIBRARY_PATH=$LIB/$v ldd build/capsule_latency | grep libnmpc_amd)";; esac
done
for rep in $(seq 1 $REPS); do
  for v in prod "$@"; do
    name=${v%@*}
    for m in cold warm; do
      f=$OUT/${TAG}_${name}_${m}_${rep}.json
      if [ $v = prod ]; then
        timeout -k 10 60 build/capsule_latency 300 $m > $f; ok $? $v
      elif [[ $v == *@* ]]; then
        env ${v#*@} timeout -k 10 60 build/capsule_latency 300 $m > $f; ok $? $v
      else
        LD_LIBRARY_PATH=$LIB/$v timeout -k 10 60 build/capsule_latency 300 $m > $f; ok $? $v
      fi
      echo "$name $m $rep $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['run_wall_ms_p50'], d['run_wall_ms_mean'], d['qp_iter_mean'])" $f)"
    done
  done
done
