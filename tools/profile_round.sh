#!/bin/bash
# Round profile set for bench.py's default workload (run on the GPU box):
#   1. rocprofv3 --kernel-trace --stats of bench.py        -> kernel durations
#   2. --pmc FETCH_SIZE            (own pass)               -> HBM read bytes
#   3. --pmc WRITE_SIZE            (own pass)               -> HBM write bytes
#   4. --pmc SQ_* VALU counters    (own pass)               -> VALU instruction mix
#   5. --pmc SQ_ACTIVE_INST_VALU(2) (own pass)              -> VALU issue quad-cycles, dual issue
# Usage: [PROF_KIND=pixel|table|table-spec] [PROF_CFG=3] [PROF_STEPS=20] [PROF_BATCH=1] \
#          tools/profile_round.sh OUTDIR [bench args...]
# PROF_BATCH > 1: the PMC passes also render the frames as batches of that many
# (the k_*_frames kernels bench.py times for batched configurations).
# The PMC passes render bench.py's own sweep frames for PROF_STEPS steps
# (tools/prof_kernels.py), so pass the same --steps to the bench.
set -e
OUT=$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --inflight 1 "$@" > "$OUT/bench_traced.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 tools/prof_kernels.py "${PROF_KIND:-pixel}" "${PROF_CFG:-3}" "${PROF_STEPS:-20}" "${PROF_BATCH:-1}" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 tools/prof_kernels.py "${PROF_KIND:-pixel}" "${PROF_CFG:-3}" "${PROF_STEPS:-20}" "${PROF_BATCH:-1}" > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_TRANS_F32 SQ_BUSY_CYCLES -d "$OUT/sq" -o run --output-format csv -- python3 tools/prof_kernels.py "${PROF_KIND:-pixel}" "${PROF_CFG:-3}" "${PROF_STEPS:-20}" "${PROF_BATCH:-1}" > "$OUT/sq.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT -d "$OUT/sq2" -o run --output-format csv -- python3 tools/prof_kernels.py "${PROF_KIND:-pixel}" "${PROF_CFG:-3}" "${PROF_STEPS:-20}" "${PROF_BATCH:-1}" > "$OUT/sq2.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE -d "$OUT/sq3" -o run --output-format csv -- python3 tools/prof_kernels.py "${PROF_KIND:-pixel}" "${PROF_CFG:-3}" "${PROF_STEPS:-20}" "${PROF_BATCH:-1}" > "$OUT/sq3.log" 2>&1
echo done
