#!/bin/bash
# Round's bench lines for every BASELINE config and the scene-table kernels (one
# MI355X): cfg1 / cfg2 over the whole 120-frame sweep, cfg3-5 and the tables with
# the driver's 20 steps.  Writes OUT/cfgN.json, OUT/table.json, OUT/tablespec.json.
set -e
OUT=${1:-gpurun_out/bench_all}
mkdir -p "$OUT"
for c in 1 2; do timeout -k 10 300 python bench.py --config $c --steps 120 --warmup 5 > "$OUT/cfg$c.json"; done
for c in 3 4 5; do timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > "$OUT/cfg$c.json"; done
timeout -k 10 300 python bench.py --config 3 --steps 20 --warmup 5 --scene table --no-cpu-baseline > "$OUT/table.json"
timeout -k 10 300 python bench.py --config 3 --steps 20 --warmup 5 --scene table-spec --no-cpu-baseline > "$OUT/tablespec.json"
echo done
