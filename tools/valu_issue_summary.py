"""VALU issue-slot utilisation per kernel from a rocprofv3 --pmc pass.

  python tools/valu_issue_summary.py DIR SUB [SUB ...]

Each DIR/SUB holds run_counter_collection.csv + run_kernel_trace.csv of one
rocprofv3 pass with SQ_ACTIVE_INST_VALU, SQ_ACTIVE_INST_VALU2, SQ_INSTS_VALU,
SQ_INSTS_VALU_TRANS_F32 and GRBM_GUI_ACTIVE (tools/valu_peak, or
tools/prof_kernels.py).  Per kernel (production instances) it prints the mean
per launch and
  busyquad/cap  = (ACTIVE_INST_VALU - ACTIVE_INST_VALU2) / (1024 SIMDs x cycles / 4):
                  the share of the SIMDs' VALU issue slots (one per quad-cycle,
                  holding one instruction or two dual-issued ones) in use;
  dual-share    = 2 VALU2 / ACTIVE_INST_VALU: instructions issued in pairs;
  v*2cyc/cap    = the executed lane-instruction fraction bench.py's roofline
                  `frac` reports (every instruction at 2 cycles).
GRBM_GUI_ACTIVE is summed over the 8 XCDs.  Diagnostic tool, not part of the product.
"""
import collections
import csv
import sys


def main(base, subs):
    for p in subs:
        rows = list(csv.DictReader(open(f"{base}/{p}/run_counter_collection.csv")))
        tr = {r["Dispatch_Id"]: r for r in csv.DictReader(open(f"{base}/{p}/run_kernel_trace.csv"))}
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        ns = collections.defaultdict(set)
        for r in rows:
            k = r["Kernel_Name"]
            if "<true" in k:
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            ns[k].add(r["Dispatch_Id"])
        for k, c in agg.items():
            n = len(ns[k])
            c = {a: v / n for a, v in c.items()}
            dur = sum(int(tr[d]["End_Timestamp"]) - int(tr[d]["Start_Timestamp"]) for d in ns[k]) / n * 1e-9
            cyc = c["GRBM_GUI_ACTIVE"] / 8  # per XCD
            cap = cyc / 4 * 1024
            v, a, v2 = c["SQ_INSTS_VALU"], c["SQ_ACTIVE_INST_VALU"], c["SQ_ACTIVE_INST_VALU2"]
            print("%-10s %-42s n%3d %.4f ms clk %.2f GHz VALU %.4g act %.4g VALU2 %.4g  busyquad/cap %.3f  "
                  "dual-share %.3f  v*2cyc/cap %.3f" % (p, k[:42], n, dur * 1e3, cyc / dur / 1e9, v, a, v2,
                                                       (a - v2) / cap, 2 * v2 / a if a else 0,
                                                       v * 2 / (cyc * 1024)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
