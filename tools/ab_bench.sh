#!/bin/bash
# A/B: bench.py (frames in flight, default cfg3) and probe_perf.py for librm.so and every
# tools/variants/librm_*.so.  Usage: tools/ab_bench.sh [bench args...]
for so in opengl-raymarching-in-compute-shader_amd/librm.so tools/variants/librm_*.so; do
  case "$so" in *librm_stats*) continue;; esac
  RM_LIBRM=$so timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > /tmp/ab.json 2>/dev/null || exit 1
  ms=$(python -c "import json;d=json.load(open('/tmp/ab.json'));print(d['ms_per_step'], d['roofline']['mean_kernel_ms'], d['parity'])")
  echo "$so bench_ms kernel_ms parity: $ms"
done
