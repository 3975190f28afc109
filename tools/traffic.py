"""HBM traffic per launch of the checksum kernel from rocprofv3 --pmc CSVs (tooling).

Correction per MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE (= TCC_EA0_RDREQ x 64 B, in KiB)
reports exactly half of the bytes of a wide coalesced streaming read (128-B requests tallied at
64 B), so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE (KiB) is exact for 16-B-per-lane
stores and is taken as is.  Usage: python tools/traffic.py profiles/r01_pmc_c2 [kernel-substring (default k_csum)]
"""
import csv, glob, json, sys, collections
d = sys.argv[1]
ks = sys.argv[2] if len(sys.argv) > 2 else "k_csum"
vals = collections.defaultdict(list)
name = None
for f in sorted(glob.glob(f"{d}/pass*.csv")):
    for r in csv.DictReader(open(f)):
        if ks in r["Kernel_Name"]:
            name = r["Kernel_Name"].split("(")[0]
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
out = {
    "kernel": name,
    "dispatches": len(vals["FETCH_SIZE"]),
    "FETCH_SIZE_KiB": fetch,
    "WRITE_SIZE_KiB": write,
    "read_bytes_corrected": 2 * fetch * 1024,
    "write_bytes": write * 1024,
    "hbm_bytes_per_launch": 2 * fetch * 1024 + write * 1024,
    "correction": "read = 2 x FETCH_SIZE (gfx950 half-count of 128-B requests), MI355X_MICROARCH.md §HBM",
}
for c in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY",
          "GRBM_GUI_ACTIVE", "TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum"):
    if vals.get(c):
        out[c] = sum(vals[c]) / len(vals[c])
json.dump(out, open(f"{d}/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
