set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_bench_dist.py -x -v --timeout 120 --timeout-method thread > gpurun_out/g2_comm.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g2_tests.log 2>&1 && \
RM_BENCH_FORCE_DIST=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/g2_bench_dist1.log 2>&1
