#!/bin/bash
# Interleaved A/B of the scene-table kernels (generic, then hiprtc-specialised)
# against tools/variants/librm_*.so, cfg3.  Run on the GPU box.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ab_kernel.py --table --cfg 3 --rounds 3 > gpurun_out/abt.log 2>&1
timeout -k 10 200 python -u tools/ab_kernel.py --table --spec --cfg 3 --rounds 3 >> gpurun_out/abt.log 2>&1
