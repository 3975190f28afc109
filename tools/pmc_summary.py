"""Mean of each PMC counter per kernel (by template instance) over the passes of
tools/pmc_variants.sh (tooling).  Usage: python tools/pmc_summary.py gpurun_out/<tag> [packets]"""
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
pk = float(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
vals = {}
for f in glob.glob(os.path.join(d, "**", "p*_counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_csum" not in k:
            continue
        m = re.search(r"k_csum_d<([^>]*)>", k)
        key = m.group(1) if m else k[:60]
        vals.setdefault(key, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for key, cs in sorted(vals.items()):
    print(key)
    for c, v in sorted(cs.items()):
        m = sum(v) / len(v)
        print(f"   {c:24s} {m:14.1f}   per pkt {m / pk:9.3f}")
