#!/bin/bash
# bench.py cfg3 at several frames-in-flight counts and graph settings (GPU box).
set -e
mkdir -p gpurun_out
: > gpurun_out/inflight.log
for args in "--inflight 3" "--inflight 4" "--inflight 2" "--inflight 6" "--inflight 3 --graph 1" "--inflight 4 --graph 1" "--inflight 3 --steps 120"; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline $args > gpurun_out/if.json 2>/dev/null
  python3 -c "import json,sys; d=json.load(open('gpurun_out/if.json')); print(sys.argv[1], d['value'], d['ms_per_step'], d['fps'])" "$args" >> gpurun_out/inflight.log
done
