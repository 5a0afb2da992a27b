#!/bin/bash
# time the pixel kernel of each librm variant (cfg3, cfg2)
for so in opengl-raymarching-in-compute-shader_amd/librm.so tools/variants/librm_*.so; do
  echo "== $so"; RM_LIBRM=$so timeout -k 10 120 python tools/probe_perf.py || exit 1
done
