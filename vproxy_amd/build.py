"""Build libvpcsum.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo
snapshot to the GPU box)."""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libvpcsum.so")
SOURCES = ["kernels.hip", "nat.hip", "api.cpp"]
HEADERS = ["internal.h", "device_common.h", "pre_common.h", os.path.join("..", "..", "include", "vpcsum.h")]
ARCH = os.environ.get("VPCSUM_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    raise RuntimeError("hipcc not found")


def source_files() -> list[str]:
    """Repo-relative paths of every file the library is built from."""
    return sorted(os.path.relpath(os.path.normpath(os.path.join(CSRC, s)), REPO) for s in SOURCES + HEADERS)


def source_hash(read=None) -> str:
    """Hash of the library's sources (the evidence key of profiles/*/summary.json: a PMC summary
    describes the kernels of exactly one source tree).  read(path) -> bytes | None lets tooling
    hash the tree of a past commit; the default reads the working tree."""
    import hashlib
    if read is None:
        def read(p):
            f = os.path.join(REPO, p)
            return open(f, "rb").read() if os.path.exists(f) else None
    h = hashlib.sha256()
    for p in source_files():
        b = read(p)
        if b is None:
            continue
        h.update(p.encode() + b"\0" + str(len(b)).encode() + b"\0" + b)
    return h.hexdigest()[:16]


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [__file__]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    objs = []
    inc = ["-I", os.path.join(REPO, "include"), "-I", CSRC]
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"] + inc
    procs = []
    for s in SOURCES:   # the translation units compile in parallel
        src = os.path.join(CSRC, s)
        obj = os.path.join(CSRC, s + ".o")
        cmd = [hipcc()] + common + ["-c", src, "-o", obj]
        if s.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"]
        if verbose:
            print(" ".join(cmd))
        procs.append((subprocess.Popen(cmd), cmd))
        objs.append(obj)
    for p, cmd in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    tmp = LIB + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
