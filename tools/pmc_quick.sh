#!/bin/bash
# Quick occupancy / issue counters of the cfg-3 render kernel (one rocprofv3 pass).
#   tools/pmc_quick.sh OUTDIR
set -e
OUT=${1:-gpurun_out/pmcq}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d "$OUT/a" -o run --output-format csv -- python3 tools/prof_kernels.py pixel 3 3 > "$OUT/a.log" 2>&1
python3 - "$OUT/a" <<'PY'
import csv, collections, sys, os
rows = list(csv.DictReader(open(os.path.join(sys.argv[1], "run_counter_collection.csv"))))
per = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for r in rows:
    per[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"]); disp[r["Kernel_Name"]].add(r["Dispatch_Id"])
kt = {}
for r in csv.DictReader(open(os.path.join(sys.argv[1], "run_kernel_trace.csv"))):
    kt.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, cs in per.items():
    if "k_sample" not in k and "k_pixel" not in k: continue
    n = len(disp[k]); c = {a: v / n for a, v in cs.items()}
    ns = sum(kt[k]) / len(kt[k])
    clk = c["GRBM_GUI_ACTIVE"] / 8 / (ns * 1e-9) / 1e9
    cyc = ns * 1e-9 * clk * 1e9
    print(k, f"time {ns/1e6:.3f} ms clock {clk:.2f} GHz")
    print(f"  resident waves/SIMD {c['SQ_WAVE_CYCLES'] * 4 / (1024 * cyc):.2f}")
    print(f"  VALU busy {c['SQ_INSTS_VALU'] * 2 / (1024 * cyc):.3f}  VALU/wave {c['SQ_INSTS_VALU']/c['SQ_WAVES']:.0f}  SALU/wave {c['SQ_INSTS_SALU']/c['SQ_WAVES']:.0f}")
    print("  ", {a: round(v) for a, v in c.items()})
PY
