"""Summarise a tools/profile_round.sh output dir into profiles/<tag>_*.{csv,json,md}.

Writes:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of bench.py
  profiles/<tag>_pmc.json           per-dispatch PMC means (FETCH_SIZE, WRITE_SIZE, SQ_*) of the
                                    dominant kernel + derived HBM bytes per launch
  profiles/<tag>_bench.json         the bench line printed under the profiler
"""
import csv
import collections
import json
import os
import shutil
import sys


def pmc(d):
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        per[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Kernel_Name"]].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in cs.items()} for k, cs in per.items()}


def main(src, tag, workload="cfg3", dst="profiles"):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(dst, f"{tag}_kernel_stats.csv"))
    out = {}
    for sub in ("fetch", "write", "sq", "sq2", "sq3"):
        p = os.path.join(src, sub)
        if not os.path.isdir(p):
            continue
        for k, cs in pmc(p).items():
            if "rmd::k_" in k:
                out.setdefault(k, {}).update(cs)
    batch = int(os.environ.get("PROF_BATCH", "1"))
    for k, cs in out.items():
        # a batched launch (k_*_frames, PROF_BATCH frames): counters per frame
        if "_frames" in k and batch > 1:
            for c in list(cs):
                cs[c] /= batch
            cs["frames_per_launch"] = batch
            cs["note"] = f"per frame: per-launch means of launches of {batch} frames, divided by {batch}"
        elif "_frames" in k:
            cs["frames_per_launch"] = 1  # (bench.py reads batch kernels' entries only with this field)
        # rocprofv3 FETCH_SIZE / WRITE_SIZE are in KiB; gfx950 FETCH_SIZE reads 1/2 of a wide
        # coalesced stream (MI355X_MICROARCH.md §HBM) — reported raw and doubled.
        if "FETCH_SIZE" in cs or "WRITE_SIZE" in cs:
            f = cs.get("FETCH_SIZE", 0.0) * 1024
            w = cs.get("WRITE_SIZE", 0.0) * 1024
            cs["hbm_read_bytes_raw"] = f
            cs["hbm_read_bytes_corrected"] = 2 * f
            cs["hbm_write_bytes"] = w
            cs["hbm_bytes_per_launch"] = 2 * f + w
        # VALU issue (gfx950, tools/valu_peak.hip): a SIMD issues one VALU slot per
        # quad-cycle, or two dual-issuable instructions of different waves in one;
        # SQ_ACTIVE_INST_VALU counts each wave's issue quad-cycles (2 for a
        # transcendental), SQ_ACTIVE_INST_VALU2 the quad-cycles that issued two.
        if "SQ_ACTIVE_INST_VALU2" in cs and "SQ_ACTIVE_INST_VALU" in cs:
            cs["valu_busy_quads"] = cs["SQ_ACTIVE_INST_VALU"] - cs["SQ_ACTIVE_INST_VALU2"]
            if "GRBM_GUI_ACTIVE" in cs:  # summed over the 8 XCDs
                cap = cs["GRBM_GUI_ACTIVE"] / 8 / 4 * 1024
                cs["valu_issue_frac_same_run"] = cs["valu_busy_quads"] / cap
    # bench.py matches a summary to its workload through _meta
    kind, cfg, steps = (os.environ.get("PROF_KIND", "pixel"), os.environ.get("PROF_CFG", "3"),
                        os.environ.get("PROF_STEPS", "20"))
    head = os.popen("git rev-parse --short=12 HEAD 2>/dev/null").read().strip()
    out["_meta"] = {"workload": workload, "source": os.path.basename(os.path.normpath(src)),
                    "frames": f"bench_frames({steps}) of cfg{cfg}: step k -> sweep frame k*120//{steps}",
                    "commit": head,
                    "passes": f"separate rocprofv3 --pmc runs of tools/prof_kernels.py {kind} {cfg} {steps} {batch}"}
    json.dump(out, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1, sort_keys=True)
    log = open(os.path.join(src, "bench_traced.log")).read().splitlines()
    line = [l for l in log if l.startswith("{")]
    if line:
        open(os.path.join(dst, f"{tag}_bench_traced.json"), "w").write(line[-1] + "\n")
    print("wrote", dst, tag, [k for k in out if k != "_meta"])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(sys.argv[3:4]))
