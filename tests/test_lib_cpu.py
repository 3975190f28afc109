"""CPU-side checks of the product library: it builds, loads, and exports exactly the C-ABI
that include/vpcsum.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "vpcsum.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(\w+)\s*\(", src, re.M)))


@pytest.fixture(scope="module")
def libpath():
    from vproxy_amd import build
    return build.build()


def test_header_declares_expected_surface():
    fns = header_functions()
    assert len(fns) >= 25
    assert "vpcsum_compute_async" in fns and "Java_io_vproxy_vpcsum_VPCsum_submit" in fns


def test_binding_lists_every_header_symbol():
    from vproxy_amd import vpcsum
    assert sorted(vpcsum.EXPORTS) == header_functions()


def test_so_exports_every_declared_symbol(libpath):
    out = subprocess.check_output(["nm", "-D", "--defined-only", libpath], text=True)
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing


def test_so_loads_and_reports_abi(libpath):
    L = ctypes.CDLL(libpath)
    for f in header_functions():
        assert hasattr(L, f)
    L.vpcsum_abi_version.restype = ctypes.c_int
    assert L.vpcsum_abi_version() == 4


def test_code_object_is_gfx950(libpath):
    # the embedded HIP fat binary names its only target
    data = open(libpath, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"gfx942" not in data and b"gfx90a" not in data


def test_fails_loudly_without_library(monkeypatch, tmp_path):
    from vproxy_amd import vpcsum
    monkeypatch.setattr(vpcsum, "_lib", None)
    monkeypatch.setattr(vpcsum, "LIB", str(tmp_path / "missing.so"))
    with pytest.raises(vpcsum.VpcsumUnavailable):
        vpcsum.lib()


def test_descriptor_layout_matches_header():
    from vproxy_amd import vpcsum
    from oracle import oracle as O
    assert vpcsum.DESC_DTYPE == O.DESC_DTYPE and vpcsum.DESC_DTYPE.itemsize == 16
    assert vpcsum.NAT4_DTYPE.itemsize == 16
    assert [vpcsum.DESC_DTYPE.fields[k][1] for k in vpcsum.DESC_DTYPE.names] == [0, 8, 10, 12, 13, 14, 15]


def test_cpp_consumer_builds(libpath, tmp_path):
    """The C-ABI is consumable from plain C++ (no torch, no Python): compile + link only."""
    exe = tmp_path / "capi_smoke"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(REPO, "include"),
                           os.path.join(REPO, "tests", "cpp", "capi_smoke.cpp"), "-L", os.path.dirname(libpath),
                           "-lvpcsum", "-o", str(exe)])
    assert exe.exists()


def test_pni_env_layout_and_errno(libpath, tmp_path):
    """PNIEnv offsets equal the PNI runtime's (pni.h:15-73: message at 8, errno_ at 4104, return_
    at 4112, 4128 bytes), checked by _Static_assert in a C file; running it throws through two PNI
    entry points (argument errors, no GPU needed) and finds type, message and errno_ set."""
    exe = tmp_path / "pni_layout"
    subprocess.check_call(["gcc", "-std=c11", "-O1", "-Wall", "-I", os.path.join(REPO, "include"),
                           os.path.join(REPO, "tests", "cpp", "pni_layout.c"), "-L", os.path.dirname(libpath),
                           "-lvpcsum", "-Wl,-rpath," + os.path.dirname(libpath), "-o", str(exe)])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "pni layout ok" in r.stdout, (r.returncode, r.stdout, r.stderr)


def test_survey_entry_points_refuse_before_init(libpath):
    """SURVEY.md §8(b)'s names (vpcsum_init / vpcsum_batch_submit / vpcsum_batch_wait /
    vpcsum_nat_submit) work over one process-wide group; before vpcsum_init every one of them
    fails with a message instead of touching a device (no GPU call here)."""
    L = ctypes.CDLL(libpath)
    L.vpcsum_last_error.restype = ctypes.c_char_p
    h = ctypes.c_uint64()
    assert L.vpcsum_batch_submit(None, ctypes.c_uint64(0), None, ctypes.c_uint32(0), None, None,
                                 ctypes.c_uint32(0), ctypes.byref(h)) != 0
    assert b"vpcsum_init first" in L.vpcsum_last_error()
    assert L.vpcsum_batch_wait(ctypes.c_uint64(1)) != 0
    assert L.vpcsum_nat_submit(None, ctypes.c_uint64(0), None, None, ctypes.c_uint32(0), None,
                               ctypes.c_uint32(0), ctypes.byref(h)) != 0
    assert L.vpcsum_register_arena(None, ctypes.c_uint64(0)) != 0
    assert L.vpcsum_shutdown() == 0   # nothing to shut down: a no-op


def test_allocation_failure_returns_error(libpath, tmp_path):
    """A host allocation failure inside an extern "C" entry returns -1 with a message instead of
    unwinding a C++ exception into the caller (api.cpp VPC_CATCH): tests/cpp/alloc_fail.cpp makes
    the global operator new throw during vpcsum_group_create_list (no GPU call before it)."""
    exe = tmp_path / "alloc_fail"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(REPO, "include"),
                           os.path.join(REPO, "tests", "cpp", "alloc_fail.cpp"), "-L", os.path.dirname(libpath),
                           "-lvpcsum", "-Wl,-rpath," + os.path.dirname(libpath), "-o", str(exe)])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "out of host memory" in r.stdout, (r.returncode, r.stdout, r.stderr)


def test_default_group_calls_race_shutdown_without_gpu(libpath):
    """The process-wide group's entry points from several threads racing vpcsum_shutdown (no GPU
    here, so every call is refused): no crash, every refusal says "vpcsum_init first"."""
    import threading
    L = ctypes.CDLL(libpath)
    L.vpcsum_last_error.restype = ctypes.c_char_p
    bad = []

    def worker():
        h = ctypes.c_uint64()
        for _ in range(2000):
            if L.vpcsum_batch_submit(None, ctypes.c_uint64(0), None, ctypes.c_uint32(0), None, None,
                                     ctypes.c_uint32(0), ctypes.byref(h)) == 0 or \
                    b"vpcsum_init first" not in L.vpcsum_last_error():
                bad.append(1)
            L.vpcsum_batch_wait(ctypes.c_uint64(1))

    ts = [threading.Thread(target=worker) for _ in range(4)]
    for t in ts:
        t.start()
    for _ in range(2000):
        assert L.vpcsum_shutdown() == 0
    for t in ts:
        t.join()
    assert not bad


def test_registration_audit_covers_every_page():
    """The release audit (vpcsum._audit_points) asks HIP about both ends of a released range and
    one address in every page between them, at most 256 spread evenly over a larger range."""
    from vproxy_amd.vpcsum import _audit_points
    p, n = 0x1010, 164238
    pts = _audit_points(p, n)
    assert p in pts and p + n - 1 in pts
    assert {q >> 12 for q in pts} == set(range(p >> 12, ((p + n - 1) >> 12) + 1))
    assert all(p <= q < p + n for q in pts)
    big = _audit_points(0x10, 1 << 30)
    assert len(big) <= 258 and min(big) == 0x10 and max(big) == 0x10 + (1 << 30) - 1
    assert _audit_points(0x2000, 1) == [0x2000, 0x2000]
