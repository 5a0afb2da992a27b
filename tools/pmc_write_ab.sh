#!/bin/bash
# HBM write/read bytes per cfg-3 launch for librm.so and each tools/variants/librm_*.so
# (one rocprofv3 --pmc pass per counter and library).  Usage: tools/pmc_write_ab.sh OUTDIR
set -e
OUT=${1:-gpurun_out/pmcw}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for so in opengl-raymarching-in-compute-shader_amd/librm.so tools/variants/librm_*.so; do
  case "$so" in *librm_stats*) continue;; esac
  n=$(basename "$so" .so)
  for c in WRITE_SIZE FETCH_SIZE; do
    RM_LIBRM=$so timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c -d "$OUT/$n.$c" -o run --output-format csv -- python3 tools/prof_kernels.py pixel 3 3 > "$OUT/$n.$c.log" 2>&1
  done
  python3 - "$OUT/$n" "$n" <<'PY'
import csv, collections, sys
tot = collections.defaultdict(float); disp = collections.defaultdict(set)
for c in ("WRITE_SIZE", "FETCH_SIZE"):
    for r in csv.DictReader(open(f"{sys.argv[1]}.{c}/run_counter_collection.csv")):
        if "k_sample<false>" in r["Kernel_Name"]:
            tot[c] += float(r["Counter_Value"]); disp[c].add(r["Dispatch_Id"])
print(sys.argv[2], {c: round(tot[c] / len(disp[c]) / 1024, 1) for c in tot}, "MB (KiB-unit counters / 1024)")
PY
done
