"""Summarise rocprofv3 --pmc CSVs: per-counter mean over dispatches, per kernel."""
import csv, glob, os, sys, collections
vals = collections.defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        per = collections.defaultdict(float)
        for r in rows:
            per[(r["Kernel_Name"][:40], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, disp, c), v in per.items():
            vals[(k, c)].append(v)
for (k, c), v in sorted(vals.items()):
    print(f"{k:42s} {c:28s} n={len(v):4d} mean={sum(v)/len(v):.6g}")
