#!/bin/bash
# Scene-table profile set (row (f) 4): the bench line, rocprof kernel stats and PMC of
# --scene table and --scene table-spec.  Usage: tools/gpu_tables.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02}
mkdir -p gpurun_out
for kind in table table-spec; do
  timeout -k 10 300 python -u bench.py --scene $kind --steps 20 --warmup 5 > gpurun_out/${TAG}_${kind}_bench.json \
    2> gpurun_out/${TAG}_${kind}_bench.err || { echo "bench $kind failed"; tail -20 gpurun_out/${TAG}_${kind}_bench.err; exit 1; }
  PROF_KIND=$kind PROF_STEPS=20 timeout -k 10 900 bash tools/profile_round.sh gpurun_out/prof_${TAG}_${kind} \
    --scene $kind --steps 20 --warmup 5 || { echo "profile $kind failed"; exit 1; }
done
echo done
