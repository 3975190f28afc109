"""Give the PMC summaries saved before round 4 the provenance fields tools/save_profiles.py now
writes (tooling, run once).  A summary committed before then did not record its tree, so it gets the
tree of the commit that added it: `head` = that commit, `src_hash` = vproxy_amd/build.py:source_hash
of the library sources in it, `provenance` says so.  usage: python tools/backfill_provenance.py"""
import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from vproxy_amd.build import source_hash  # noqa: E402


def git(*args) -> str:
    return subprocess.check_output(["git", "-C", REPO] + list(args), text=True).strip()


def show(commit, path):
    try:
        return subprocess.check_output(["git", "-C", REPO, "show", f"{commit}:{path}"], stderr=subprocess.DEVNULL)
    except subprocess.CalledProcessError:
        return None


def main():
    n = 0
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_*", "summary.json"))):
        d = json.load(open(f))
        if "src_hash" in d:
            continue
        rel = os.path.relpath(f, REPO)
        log = git("log", "--diff-filter=A", "--format=%H %ct", "--", rel).splitlines()
        if not log:
            continue
        commit, ct = log[-1].split()
        prov = {"tag": os.path.basename(os.path.dirname(f)).split("_pmc_")[0],
                "src_hash": source_hash(lambda p: show(commit, p)), "head": commit, "head_time": int(ct),
                "head_matches_src": True,
                "provenance": "backfilled in round 4: the tree of the commit that added this summary"}
        json.dump({**{k: d[k] for k in ("kernel_substring", "packets", "dispatches") if k in d}, **prov,
                   **{k: v for k, v in d.items() if k not in ("kernel_substring", "packets", "dispatches")}},
                  open(f, "w"), indent=1)
        n += 1
    print(f"backfilled {n} summaries")


if __name__ == "__main__":
    main()
