#!/bin/bash
# GPU scene-table tests, then the A/B of both table kernels (tools/ab_tables.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scene.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/scene_tests.log 2>&1 || { tail -30 gpurun_out/scene_tests.log; exit 1; }
tail -2 gpurun_out/scene_tests.log
bash tools/ab_tables.sh
