#!/bin/bash
# Interleaved bench.py A/B (frames in flight): librm.so and every tools/variants/librm_*.so,
# ROUNDS rounds, one bench process per (round, library).  Usage: tools/ab_bench_rounds.sh ROUNDS [bench args...]
n=$1; shift
for r in $(seq 1 "$n"); do
  for so in opengl-raymarching-in-compute-shader_amd/librm.so tools/variants/librm_*.so; do
    case "$so" in *librm_stats*) continue;; esac
    RM_LIBRM=$so timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > /tmp/ab.json 2>/dev/null || exit 1
    python3 -c "import json,sys;d=json.load(open('/tmp/ab.json'));print(sys.argv[1], d['ms_per_step'], d['roofline']['mean_kernel_ms'])" "$r $so"
  done
done
