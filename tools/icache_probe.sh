#!/bin/bash
# Instruction-fetch counters of the solve kernels (study: does the row-parallel kernel's 60 KB of code wait on
# instruction fetch?). Lists the device's counters, then one --pmc pass per counter group that the list holds, over
# the one-robot capsule (C driver), diff1024 and the metric bench. Kernel dispatches only, no trace domains.
# usage: gpurun -- 'bash tools/icache_probe.sh <tag> [lib variant dir]'
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-ic}
VAR=${2:-}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 120 rocprofv3 --list-avail > $OUT/${TAG}_counters.txt 2>&1; ok $? list
have() { grep -qw "$1" $OUT/${TAG}_counters.txt; }
G1=""
for c in SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU; do
  if have $c; then G1="$G1 $c"; fi
done
G2=""
for c in SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ; do
  if have $c; then G2="$G2 $c"; fi
done
echo "group1:$G1"
echo "group2:$G2"
ENVV=""
if [ -n "$VAR" ]; then ENVV="$GRAFT_REPO_ROOT/nmpc_nav_control_amd/lib/$VAR"; fi
run() {  # run <name> <group> <command...>
  local name=$1 grp=$2; shift 2
  if [ -z "$grp" ]; then return 0; fi
  NMPC_AMD_LIB=${ENVV:+$ENVV/libnmpc_amd.so} LD_LIBRARY_PATH=${ENVV:+$ENVV:}$LD_LIBRARY_PATH \
    timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/${TAG}_${name} -o run --output-format csv -- "$@" \
    > $OUT/${TAG}_${name}.log 2>&1
}
for g in 1 2; do
  eval grp=\$G$g
  run cap_g$g "$grp" $GRAFT_REPO_ROOT/build/capsule_latency 100 cold; ok $? cap_g$g
  run d1024_g$g "$grp" python3 $GRAFT_REPO_ROOT/bench.py --config diff1024 --steps 5 --warmup 2 --closed-loop-warmup 60 --no-cpu-baseline; ok $? d1024_g$g
  run metric_g$g "$grp" python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --closed-loop-warmup 60 --no-cpu-baseline; ok $? metric_g$g
done
echo done
