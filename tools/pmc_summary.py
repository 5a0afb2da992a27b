"""Summarise rocprofv3 counter_collection CSVs: per kernel name, sum of each counter per dispatch."""
import csv, sys, collections, glob, os
def load(d):
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"]
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in cs.items()} for k, cs in per.items()}
for d in sys.argv[1:]:
    for k, cs in load(d).items():
        if "k_" not in k: continue
        print(d, k[:40])
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {v:16.4g}")
