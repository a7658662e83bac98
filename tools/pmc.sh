#!/bin/bash
# PMC passes on the bench (one counter group per pass, kernel dispatches only; no trace domains).
# usage: gpurun -- 'bash tools/pmc.sh <tag> [bench args...]'
#        then python tools/pmc_summary.py gpurun_out/<tag> <config key> --write
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-p}; shift
cd /tmp && export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; exit $rc; fi; }
CMD="python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --closed-loop-warmup ${PMC_WARMUP:-240} --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/${TAG}_pmc1 -o run --output-format csv -- $CMD > $OUT/${TAG}_pmc1.log 2>&1; rc=$?; echo "pmc1 rc=$rc"; ok $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/${TAG}_pmc2 -o run --output-format csv -- $CMD > $OUT/${TAG}_pmc2.log 2>&1; rc=$?; echo "pmc2 rc=$rc"; ok $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $OUT/${TAG}_pmc3 -o run --output-format csv -- $CMD > $OUT/${TAG}_pmc3.log 2>&1; rc=$?; echo "pmc3 rc=$rc"; ok $rc
# pass 5: the L2's memory-side requests and the share of them destined for DRAM (roofline.hbm; calibrated against
# an Infinity-Cache-resident and a non-resident table by tools/ubench_mall.hip)
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum -d $OUT/${TAG}_pmc5 -o run --output-format csv -- $CMD > $OUT/${TAG}_pmc5.log 2>&1; rc=$?; echo "pmc5 rc=$rc"; ok $rc
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32 SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVES SQ_WAVE_CYCLES -d $OUT/${TAG}_pmc4 -o run --output-format csv -- $CMD > $OUT/${TAG}_pmc4.log 2>&1; rc=$?; echo "pmc4 rc=$rc"; ok $rc
