"""Register, scratch and LDS budgets of the shipped gfx950 kernels, read from the code objects the
build left in vproxy_amd/csrc/*.o (no GPU needed).  They guard what DESIGN.md states and the
launchers assume: every default K2 build (compute and verify, unstaged and staging, and their
window builds for arenas past 4 GiB) fits 6 waves per SIMD (the dense-frame grid is one resident
round of it, §5 items 26, 28, 29), and no default kernel spills to scratch (the NAT rewrite once
kept its accumulator struct there, §7)."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def kernels(obj: str) -> dict:
    """{mangled name: {vgpr_count, private_segment_fixed_size, group_segment_fixed_size}}"""
    path = os.path.join(REPO, "vproxy_amd", "csrc", obj)
    if not os.path.exists(path) or not os.path.exists(os.path.join(LLVM, "clang-offload-bundler")):
        pytest.skip("build artefacts or ROCm LLVM tools missing")
    with tempfile.TemporaryDirectory() as td:
        fat, co = os.path.join(td, "k.fat"), os.path.join(td, "k.co")
        subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", path])
        subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--type=o", f"--input={fat}",
                               f"--targets={TARGET}", f"--output={co}", "--unbundle"])
        notes = subprocess.check_output([os.path.join(LLVM, "llvm-readelf"), "--notes", co], text=True)
    # one YAML map per kernel, its first key marked "- ": collect the keys of each map
    res, cur = {}, None
    entries = []
    for line in notes.splitlines():
        m = re.match(r"(\s+)(- )?\.(\w+):\s+(\S+)", line)
        if not m:
            continue
        indent, dash, key, val = m.groups()
        if dash and len(indent) <= 3:   # a kernel entry (the args' own list items are deeper)
            cur = {}
            entries.append(cur)
        if cur is not None and len(indent) <= 4 and key in ("name", "vgpr_count", "private_segment_fixed_size",
                                                                "group_segment_fixed_size"):
            cur[key] = val if key == "name" else int(val)
    for e in entries:
        if "name" in e:
            res[e.pop("name")] = e
    return res


def pick(ks: dict, pattern: str) -> dict:
    sel = {k: v for k, v in ks.items() if re.search(pattern, k)}
    assert sel, f"no kernel matches {pattern}"
    return sel


def test_k2_default_builds_budgets():
    ks = kernels("kernels.hip.o")
    # k_csum_d<8, 6, 2, 2, VERIFY, NT, 1, 0, -9, true, false, DS, WIN, WGS>: the default builds,
    # their window builds for arenas past 4 GiB (WIN) and the workgroup-sorted build (WGS)
    unstaged_compute = pick(ks, r"k_csum_dILi8ELi6ELi2ELi2ELb0ELb[01]ELi1ELi0ELin9ELb1ELb0ELb0ELb[01]ELb0E")
    staged_compute = pick(ks, r"k_csum_dILi8ELi6ELi2ELi2ELb0ELb[01]ELi1ELi0ELin9ELb1ELb0ELb1ELb[01]ELb0E")
    sorted_units = pick(ks, r"k_csum_dILi8ELi6ELi2ELi2ELb[01]ELb[01]ELi1ELi0ELin9ELb1ELb0ELb1ELb0ELb1E")
    verify = pick(ks, r"k_csum_dILi8ELi6ELi2ELi2ELb1ELb[01]ELi1ELi0ELin9ELb1ELb0ELb[01]ELb[01]ELb[01]E")
    assert len(unstaged_compute) == len(staged_compute) == len(sorted_units) == 4 and len(verify) == 10
    staged_compute.update(sorted_units)
    # every default build fits 6 waves per SIMD (the verify and staging builds since round 4: the
    # stored field written to the slot by the lane that loads it, a scalar wave index, opaque
    # result-store indices)
    for k, v in {**unstaged_compute, **staged_compute, **verify}.items():
        assert v["vgpr_count"] <= 80, (k, v)
    for k, v in {**unstaged_compute, **staged_compute, **verify}.items():
        assert v["private_segment_fixed_size"] == 0, (k, v)
    # the slot plans, and the staged result words: 16 KiB and 26 KiB per workgroup (+ 64 B of class
    # counts in the workgroup-sorted build)
    assert all(v["group_segment_fixed_size"] <= 16384 for v in unstaged_compute.values())
    assert all(v["group_segment_fixed_size"] <= 26624 + 64 for v in staged_compute.values())


def test_no_scratch_in_default_kernels():
    ks = {**kernels("kernels.hip.o"), **kernels("nat.hip.o")}
    # the NAT kernels at their default occupancy (k_natq ... WPE 1), the byte kernel, the lane
    # layout, parse, service, probes, every K2 build (the window builds included); the
    # forced-occupancy tuning shapes (WPE 6 / 8) may spill
    default = {k: v for k, v in ks.items()
               if re.search(r"k_natq\w*ELi1EEEv|k_natw|k_natILi|k_parse_ether|k_csum_service|k_pattern_probe|k_read_probe|"
                            r"k_csum_d", k)}
    assert len(default) > 20
    spills = {k: v["private_segment_fixed_size"] for k, v in default.items() if v["private_segment_fixed_size"]}
    assert not spills, spills
