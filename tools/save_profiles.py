"""Copy the judged evidence of one measurement call (tools/gpu_r02.sh <tag>) from gpurun_out/ into
profiles/ (tooling).  Usage: python tools/save_profiles.py <tag>

  <tag>_bench_<cfg>.json          bench.py JSON lines (c2 headline; c1 c3 c4 c4_strong c5)
  <tag>_c2_kernel_stats.csv       rocprofv3 --kernel-trace --stats of `bench.py` (headline command)
  <tag>_pmc_<cfg>/pass<i>.csv     --pmc passes, rows of the measured kernel only
  <tag>_pmc_<cfg>/summary.json    per-launch means + HBM bytes (tools/traffic.py rules)
  <tag>_hostpath_c2.json          tools/hostpath.py

Every summary.json records the tree it measured: `src_hash` (vproxy_amd/build.py:source_hash of the
library sources, computed on the GPU box into gpurun_out/<tag>_src.json by the measurement script),
`head` / `head_time` (this repo's HEAD when the summary was saved; `head_matches_src` says whether
HEAD's sources hash to `src_hash`), so bench.py can take the traffic of the tree it benches.
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
PACKETS = {"c1": 1 << 20, "c2": 1 << 20, "c3": 1 << 20, "c4": 1 << 18}
sys.path.insert(0, REPO)
from vproxy_amd.build import source_hash  # noqa: E402


def git(*args) -> str:
    return subprocess.check_output(["git", "-C", REPO] + list(args), text=True).strip()


def provenance(tag: str) -> dict:
    """The measured tree (the box's source hash, else this tree's) and this repo's HEAD."""
    f = os.path.join(G, f"{tag}_src.json")
    src = json.load(open(f))["src_hash"] if os.path.exists(f) else source_hash()
    head = git("rev-parse", "HEAD")
    head_src = source_hash(lambda p: _show(head, p))
    return {"tag": tag, "src_hash": src, "head": head, "head_time": int(git("show", "-s", "--format=%ct", head)),
            "head_matches_src": head_src == src and source_hash() == src}


def _show(commit: str, path: str):
    try:
        return subprocess.check_output(["git", "-C", REPO, "show", f"{commit}:{path}"], stderr=subprocess.DEVNULL)
    except subprocess.CalledProcessError:
        return None


def json_line(log):
    if not os.path.exists(log):
        return None
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    return None


def summarise(src, dst, kern, packets, prov=None):
    """Mean of each counter over the kernel's dispatches, plus HBM bytes per launch.  Reads:
    FETCH_SIZE = TCC_EA0_RDREQ x 64 B, and every read request of these kernels is 128 B
    (TCC_EA0_RDREQ_128B = TCC_EA0_RDREQ for K2 on C1-C3 and for the NAT kernel's scattered header
    windows, profiles/r02u_read_request_sizes.json): read bytes = 2 x FETCH_SIZE for both."""
    vals = {}
    os.makedirs(dst, exist_ok=True)
    for f in sorted(glob.glob(os.path.join(src, "p*_counter_collection.csv"))):
        i = os.path.basename(f).split("_")[0][1:]
        keep = [r for r in csv.DictReader(open(f)) if kern in r["Kernel_Name"]]
        if not keep:
            continue
        with open(os.path.join(dst, f"pass{i}.csv"), "w", newline="") as fo:
            w = csv.DictWriter(fo, fieldnames=list(keep[0].keys()))
            w.writeheader()
            w.writerows(keep)
        for r in keep:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    out = {"kernel_substring": kern, "packets": packets, "dispatches": len(vals.get("FETCH_SIZE", [])),
           **(prov or {}), **mean}
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        rd, wr = mean["FETCH_SIZE"] * 1024, mean["WRITE_SIZE"] * 1024
        out["write_bytes"] = wr
        out["read_bytes_corrected"] = 2 * rd
        out["hbm_bytes_per_launch"] = 2 * rd + wr
        out["correction"] = ("read = 2 x FETCH_SIZE: FETCH_SIZE tallies 64 B per request and every read "
                             "request is 128 B (TCC_EA0_RDREQ_128B, profiles/r02u_read_request_sizes.json)")
        for k in ("hbm_bytes_per_launch", "write_bytes"):
            out[k + "_per_packet"] = round(out[k] / packets, 2)
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum"):
        if k in mean:
            out[k + "_per_packet"] = round(mean[k] / packets, 3)
    json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1)


def resummarise(tag):
    """Recompute the summaries of committed PMC passes (profiles/<tag>_pmc_*/pass*.csv)."""
    for dst in sorted(glob.glob(os.path.join(P, f"{tag}_pmc_*"))):
        cfg = os.path.basename(dst)[len(tag) + 5:]
        old = json.load(open(os.path.join(dst, "summary.json")))
        tmp = dst + ".src"
        os.makedirs(tmp, exist_ok=True)
        for f in glob.glob(os.path.join(dst, "pass*.csv")):
            shutil.copy(f, os.path.join(tmp, "p" + os.path.basename(f)[4:-4] + "_counter_collection.csv"))
        summarise(tmp, dst, old["kernel_substring"], old["packets"],
                  {k: old[k] for k in ("tag", "src_hash", "head", "head_time", "head_matches_src", "provenance")
                   if k in old})
        shutil.rmtree(tmp)


def main(tag):
    os.makedirs(P, exist_ok=True)
    prov = provenance(tag)
    for cfg in ("c2", "c1", "c3", "c4", "c4_strong", "c5", "c5pre", "c4s_8rank", "c5_8rank", "c2_2rank", "c5_2rank"):
        d = json_line(os.path.join(G, f"{tag}_bench_{cfg}.log"))
        if d:
            json.dump(d, open(os.path.join(P, f"{tag}_bench_{cfg}.json"), "w"), indent=1)
    ks = os.path.join(G, f"{tag}_trace", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(P, f"{tag}_c2_kernel_stats.csv"))
    for src in sorted(glob.glob(os.path.join(G, f"{tag}_pmc_*"))):
        if not os.path.isdir(src):
            continue
        cfg = os.path.basename(src)[len(tag) + 5:]
        nat, pre = cfg.startswith("nat"), cfg.startswith("pre")
        summarise(src, os.path.join(P, f"{tag}_pmc_{cfg}"), "vpcsum::k_pre" if pre else "vpcsum::k_nat" if nat else "k_csum",
                  10_000_000 if nat or pre else PACKETS[cfg], prov)
    for tr in ("nat", "c5pre"):   # kernel traces of the C5 commands
        ks = os.path.join(G, f"{tag}_trace_{tr}", "run_kernel_stats.csv")
        if os.path.exists(ks):
            shutil.copy(ks, os.path.join(P, f"{tag}_{tr}_kernel_stats.csv"))
    d = json_line(os.path.join(G, f"{tag}_hostpath.log"))
    if d:
        json.dump(d, open(os.path.join(P, f"{tag}_hostpath_c2.json"), "w"), indent=1)
    fl = os.path.join(G, f"{tag}_flush.log")   # tools/flush_latency: one JSON object per line
    if os.path.exists(fl):
        rows = [json.loads(x) for x in open(fl) if x.startswith("{")]
        if rows:
            json.dump({"src_hash": prov["src_hash"], "head": prov["head"], "rows": rows},
                      open(os.path.join(P, f"{tag}_flush_latency.json"), "w"), indent=1)
    for name, out in (("preflush", "preflush"), ("c3split", "c3split"), ("c3var", "c3_variants")):
        d = json_line(os.path.join(G, f"{tag}_{name}.log"))
        if d:
            json.dump({"src_hash": prov["src_hash"], "head": prov["head"], **d},
                      open(os.path.join(P, f"{tag}_{out}.json"), "w"), indent=1)
    vm = sorted(glob.glob(os.path.join(G, f"{tag}_vm_*.log")))   # tools/verify_modes.sh logs
    if vm:
        dst = os.path.join(P, f"{tag}_verify_modes")
        os.makedirs(dst, exist_ok=True)
        for f in vm:
            shutil.copy(f, dst)
        json.dump({"src_hash": prov["src_hash"], "head": prov["head"]}, open(os.path.join(dst, "src.json"), "w"))
    print("saved", sorted(f for f in os.listdir(P) if f.startswith(tag)))


if __name__ == "__main__":
    if sys.argv[1] == "--resummarise":
        resummarise(sys.argv[2])
    else:
        main(sys.argv[1])
