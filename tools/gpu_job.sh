set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g1_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/g1_bench20.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 120 --warmup 5 --no-cpu-baseline > gpurun_out/g1_bench120.log 2>&1
