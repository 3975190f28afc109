"""Summarise tools/pmc_deep.sh passes (tooling): mean of each counter over the measured kernel's
dispatches, per packet where that reads better, one JSON per config.
usage: python tools/pmc_deep_summary.py <tag> [out_dir]"""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PACKETS = {"c1": 1 << 20, "c2": 1 << 20, "c3": 1 << 20, "c4": 1 << 18, "nat": 10_000_000, "natprobe": 10_000_000,
           # C3's size classes in batch 0 (seed 0x20241020; tools/prof_one.py --class-len prints them)
           "c3_64": 349686, "c3_576": 349183, "c3_1500": 349707}


def main(tag, out_dir=None):
    res = {}
    for d in sorted(glob.glob(os.path.join(REPO, "gpurun_out", f"{tag}_deep_*"))):
        if not os.path.isdir(d):
            continue
        cfg = os.path.basename(d)[len(tag) + 6:]
        kern = "vpcsum::k_nat" if cfg.startswith("nat") else "k_csum"
        vals = {}
        for f in sorted(glob.glob(os.path.join(d, "p*_counter_collection.csv"))):
            for r in csv.DictReader(open(f)):
                if kern in r["Kernel_Name"]:
                    vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        mean = {k: sum(v) / len(v) for k, v in vals.items()}
        n = PACKETS.get(cfg, 1)
        out = {"kernel_substring": kern, "packets": n, **{k: round(v, 1) for k, v in mean.items()}}
        for k, v in mean.items():
            out[k + "_per_packet"] = round(v / n, 4)
        if "TCP_UTCL1_TRANSLATION_MISS" in mean and mean.get("TCP_UTCL1_REQUEST"):
            out["utcl1_miss_rate"] = round(mean["TCP_UTCL1_TRANSLATION_MISS"] / mean["TCP_UTCL1_REQUEST"], 4)
        if mean.get("TCP_TCC_READ_REQ"):
            out["tcc_read_latency_cycles"] = round(mean.get("TCP_TCC_READ_REQ_LATENCY", 0) / mean["TCP_TCC_READ_REQ"], 1)
        if mean.get("SQ_INSTS_VMEM_RD"):   # algorithmic bytes per vector-load instruction (1,024 at most: 64 x 16 B)
            alg = {"c3_64": 84.0, "c3_576": 596.0, "c3_1500": 1520.0, "c3": 733.4, "c2": 1520.0, "c1": 84.0}.get(cfg)
            if alg:
                out["alg_bytes_per_vmem_rd"] = round(alg * n / mean["SQ_INSTS_VMEM_RD"], 1)
        if mean.get("SQ_WAVE_CYCLES"):
            for k in ("SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_VMEM_TA_ADDR_FIFO_FULL", "SQ_VMEM_TA_CMD_FIFO_FULL",
                      "SQ_ACTIVE_INST_VMEM"):
                if k in mean:
                    out[k + "_frac_of_wave_cycles"] = round(mean[k] / mean["SQ_WAVE_CYCLES"], 4)
        res[cfg] = out
        if out_dir:
            os.makedirs(out_dir, exist_ok=True)
            json.dump(out, open(os.path.join(out_dir, f"{cfg}.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
