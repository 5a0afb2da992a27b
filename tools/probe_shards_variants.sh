#!/bin/bash
for so in opengl-raymarching-in-compute-shader_amd/librm.so tools/variants/librm_*.so; do
  echo "== $so"; RM_LIBRM=$so timeout -k 10 200 python tools/probe_shards.py || exit 1
done
