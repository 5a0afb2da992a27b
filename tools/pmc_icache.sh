#!/bin/bash
OUT=$1; K=${2:-pixel}
mkdir -p $OUT; cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_ANY SQ_WAVE_CYCLES -d $OUT/ic_$K -o run --output-format csv -- python3 tools/prof_kernels.py $K 3 2 > $OUT/ic_$K.log 2>&1
