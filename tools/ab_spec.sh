#!/bin/bash
# Interleaved A/B of the specialised scene-table kernel against tools/variants/librm_*.so, cfg3.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_kernel.py --table --spec --cfg 3 --rounds ${ROUNDS:-4} > gpurun_out/abs.log 2>&1
cat gpurun_out/abs.log
