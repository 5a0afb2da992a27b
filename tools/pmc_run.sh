#!/bin/bash
# Collect PMC counters for each kernel variant in separate rocprofv3 passes.
# Usage: tools/pmc_run.sh OUTDIR CFG
set -e
OUT=${1:-gpurun_out/pmc}; CFG=${2:-3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_TRANS_F32 SQ_BUSY_CYCLES"
B="GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
for k in pixel wavequeue; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $A -d $OUT/${k}_A -o run --output-format csv -- python3 tools/prof_kernels.py $k $CFG 2 > $OUT/${k}_A.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $B -d $OUT/${k}_B -o run --output-format csv -- python3 tools/prof_kernels.py $k $CFG 2 > $OUT/${k}_B.log 2>&1
done
