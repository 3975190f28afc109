"""Summarise rocprofv3 --pmc CSVs (per kernel name: mean of each counter over dispatches)."""
import csv, glob, sys, collections
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "csum" not in k and "read_probe" not in k:
            continue
        acc[k][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, m in acc.items():
    per = collections.defaultdict(list)
    for (disp, c), vals in m.items():
        per[c].append(sum(vals))
    short = k.split("(")[0][:70]
    print(short, {c: f"{sum(v)/len(v):.4g}" for c, v in sorted(per.items())})
