#!/bin/bash
# Interleaved A/B of both scene-table kernels (generic, specialised) against tools/variants/librm_*.so, cfg3.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_kernel.py --table --cfg 3 --rounds ${ROUNDS:-3} > gpurun_out/abts.log 2>&1
timeout -k 10 300 python -u tools/ab_kernel.py --table --spec --cfg 3 --rounds ${ROUNDS:-3} >> gpurun_out/abts.log 2>&1
cat gpurun_out/abts.log
