set -e
mkdir -p gpurun_out
: > gpurun_out/host.log
for c in 3 2 1; do
  timeout -k 10 150 python -u bench.py --no-cpu-baseline --config $c > gpurun_out/h.json 2>/dev/null
  python3 -c "import json,sys; d=json.load(open('gpurun_out/h.json')); print('cfg', sys.argv[1], d['value'], d['ms_per_step'], 'host', d['host_issue_ms_per_step'], d['config']['frames_in_flight'])" $c >> gpurun_out/host.log
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bench_dist.py >> gpurun_out/host.log 2>&1
