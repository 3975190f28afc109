"""bench.py's roofline.traffic comes from the PMC summary of the tree it benches:
a summary whose src_hash equals the running library's sources wins; without one, the newest by
commit time (never by tag name), reported as stale.  CPU only."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from vproxy_amd.build import source_files, source_hash  # noqa: E402

ROUND3_FINAL_SRC = "5e3c0c844d770e36"   # the library sources of round 3's final tree (4cd5325..70aed42)


def _summary(root, tag, cfg, src, head_time, bytes_per_pkt):
    d = os.path.join(root, f"{tag}_pmc_{cfg}")
    os.makedirs(d)
    json.dump({"packets": 1000, "hbm_bytes_per_launch": bytes_per_pkt * 1000.0, "src_hash": src,
               "head": f"commit-{tag}", "head_time": head_time}, open(os.path.join(d, "summary.json"), "w"))


def test_matching_source_beats_newer_summaries(tmp_path):
    _summary(tmp_path, "r04a", "c2", "aaaa", 100, 1500)
    _summary(tmp_path, "r04z", "c2", "bbbb", 300, 1600)
    t, prov = bench.pmc_traffic("c2", 2000, str(tmp_path), "aaaa")
    assert t == 3_000_000 and prov["source"].startswith("r04a_") and prov["stale"] is False


def test_fallback_is_newest_commit_not_tag_name(tmp_path):
    # 'r03z' sorts after 'r03yp' by name but was measured earlier (round 3's trap)
    _summary(tmp_path, "r03z", "nat15", "old1", 1000, 235)
    _summary(tmp_path, "r03yp", "nat15", "old2", 2000, 209)
    t, prov = bench.pmc_traffic("nat15", 1000, str(tmp_path), "current")
    assert t == 209_000 and prov["source"].startswith("r03yp_") and prov["stale"] is True
    assert prov["head"] == "commit-r03yp"


def test_round3_final_tree_picks_its_own_summaries():
    t, prov = bench.pmc_traffic("c2", 1 << 20, src=ROUND3_FINAL_SRC)
    assert prov["source"] == os.path.join("profiles", "r03ys_pmc_c2", "summary.json") and not prov["stale"]
    assert abs(t / (1 << 20) - 1556.3) < 0.5
    t, prov = bench.pmc_traffic("nat15", 10_000_000, src=ROUND3_FINAL_SRC)
    assert prov["source"] == os.path.join("profiles", "r03yp_pmc_nat15", "summary.json") and not prov["stale"]
    assert abs(t / 10_000_000 - 209.2) < 0.1   # not r03z's 235 B/pkt


def test_every_committed_summary_records_its_tree():
    import glob
    fs = glob.glob(os.path.join(REPO, "profiles", "*_pmc_*", "summary.json"))
    assert fs
    for f in fs:
        d = json.load(open(f))
        assert len(d.get("src_hash", "")) == 16 and d.get("head") and d.get("head_time"), f


def test_source_hash_covers_the_library_sources():
    files = source_files()
    assert "include/vpcsum.h" in files and "vproxy_amd/csrc/kernels.hip" in files
    assert "vproxy_amd/csrc/nat.hip" in files and "vproxy_amd/csrc/api.cpp" in files
    h = source_hash()
    assert len(h) == 16 and h == source_hash()
    # a change to any source changes the hash
    assert source_hash(lambda p: b"x" if p.endswith("nat.hip") else open(os.path.join(REPO, p), "rb").read()) != h
