#!/bin/bash
# Interleaved A/B of bench.py's issue method on one GPU (cfg by $CFG, default 3),
# the driver's steps / warmup; prints ms_per_step, frames per launch, contexts.
#   VARIANTS="A:;B:--batch 1 --inflight 2" bash tools/ab_issue.sh
set -e
CFG=${CFG:-3}
ROUNDS=${ROUNDS:-5}
STEPS=${STEPS:-20}
IFS=';' read -ra VS <<< "${VARIANTS:-A:;C:--batch 1 --inflight 3;D:--batch 1 --inflight 4;E:--batch 2 --inflight 3}"
for r in $(seq 1 $ROUNDS); do
  for spec in "${VS[@]}"; do
    v=${spec%%:*}; extra=${spec#*:}
    timeout -k 10 120 python bench.py --config $CFG --steps $STEPS --warmup 5 --no-cpu-baseline $extra > gpurun_out/ab_$v.json 2>/dev/null
    python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', d['ms_per_step'], d['config']['frames_per_launch'], d['config']['contexts_in_flight'])"
  done
done
