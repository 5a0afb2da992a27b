set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scene.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/scene_tests.log 2>&1 || { tail -30 gpurun_out/scene_tests.log; exit 1; }
tail -2 gpurun_out/scene_tests.log
timeout -k 10 200 python -u tools/ab_kernel.py --table --cfg 3 --rounds 3 > gpurun_out/abg.log 2>&1
timeout -k 10 200 python -u tools/ab_kernel.py --table --cfg 2 --rounds 3 --frames 60 >> gpurun_out/abg.log 2>&1
timeout -k 10 200 python -u tools/ab_kernel.py --table --cfg 1 --rounds 3 --frames 60 >> gpurun_out/abg.log 2>&1
cat gpurun_out/abg.log
