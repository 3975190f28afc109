"""Copy the judged evidence of one GPU round (tools/gpu_full.sh) from gpurun_out/ into profiles/
under a round tag (tooling).  Usage: python tools/save_profiles.py r01c

  <tag>_c2_kernel_stats.csv     rocprofv3 --kernel-trace --stats of `bench.py` (gpu_round.sh prof)
  <tag>_bench_<wl>.json         bench.py JSON lines (c2 headline, c1/c3/c4 from gpu_extra.sh)
  <tag>_pmc_<wl>/pass<i>_k_csum.csv + summary.json   --pmc passes (k_csum* rows) + tools/traffic.py
  <tag>_nat_c5.json, <tag>_hostpath_c2.json          tools/natbench.py, tools/hostpath.py
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(REPO, "gpurun_out")
P = os.path.join(REPO, "profiles")


def json_line(log):
    if not os.path.exists(log):
        return None
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    return None


def main(tag):
    os.makedirs(P, exist_ok=True)
    ks = os.path.join(G, "prof", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(P, f"{tag}_c2_kernel_stats.csv"))
    for wl, log in (("c2", "bench.log"), ("c1", "bench_c1.log"), ("c3", "bench_c3.log"), ("c4", "bench_c4.log")):
        d = json_line(os.path.join(G, log))
        if d:
            json.dump(d, open(os.path.join(P, f"{tag}_bench_{wl}.json"), "w"))
    for name, out in (("natbench.log", "nat_c5"), ("hostpath.log", "hostpath_c2"),
                      ("pattern_all.log", "pattern_ceiling"), ("bench_2rank.log", "bench_2rank_1gpu")):
        d = json_line(os.path.join(G, name))
        if d:
            json.dump(d, open(os.path.join(P, f"{tag}_{out}.json"), "w"), indent=1)
    fl = os.path.join(G, "flush_latency.json")
    if os.path.exists(fl) and json_line(fl):
        json.dump(json_line(fl), open(os.path.join(P, f"{tag}_flush_latency.json"), "w"), indent=1)
    for src in sorted(glob.glob(os.path.join(G, "pmc_*"))):
        wl = os.path.basename(src)[4:]
        kern = "k_nat4w" if wl == "nat" else "k_csum"
        dst = os.path.join(P, f"{tag}_pmc_{wl}")
        os.makedirs(dst, exist_ok=True)
        for f in sorted(glob.glob(os.path.join(src, "p*_counter_collection.csv"))):
            i = os.path.basename(f).split("_")[0][1:]
            rows = list(csv.DictReader(open(f)))
            keep = [r for r in rows if kern in r["Kernel_Name"]]
            if not keep:
                continue
            with open(os.path.join(dst, f"pass{i}_{kern}.csv"), "w", newline="") as fo:
                w = csv.DictWriter(fo, fieldnames=list(keep[0].keys()))
                w.writeheader()
                w.writerows(keep)
        subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "traffic.py"), dst, kern],
                              stdout=subprocess.DEVNULL)
    print("saved", sorted(f for f in os.listdir(P) if f.startswith(tag)))


if __name__ == "__main__":
    main(sys.argv[1])
