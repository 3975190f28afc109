"""What HIP does with overlapping host registrations (round 6, the intermittent-fault inquiry).

Attribute queries only -- no kernel reads any of these ranges, so nothing here can fault.  Each case
registers host memory with libvpcsum contexts (hipHostRegister(Mapped)) in some order, and after each
step records hipPointerGetAttributes (type, device pointer) for the ranges involved:

  same_range      two contexts register the same array; unregister A, then B
  same_range_rev  the same, unregistered B first
  shared_page     two arrays in one page, each registered by its own context
  sub_range       an array and a sub-slice of it (another context)

  same_start      a range and a longer one from the same address (another context)
  after_double    a double registration undone as well as HIP allows, then a fresh array at the
                  same pages registered and unregistered once: does the old registration resurface?

Each case runs in a fresh process (no HIP state carried between cases); one JSON line per case.
Usage: python tools/reg_probe.py [case]
"""
import ctypes
import json
import mmap
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    torch.cuda.init()
    from vproxy_amd import vpcsum as V
    L = V.lib()
    H = None

    def attr(p):
        nonlocal H
        V.hip_holds_registered(p)   # loads the runtime handle
        H = V._hip
        a = V._PtrAttr()
        rc = H.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p))
        H.hipGetLastError()
        return {"rc": rc, "type": a.type, "dev": hex(a.devicePointer or 0), "host": hex(a.hostPointer or 0)}

    def ctx():
        h = ctypes.c_void_p()
        assert L.vpcsum_ctx_create(0, 1 << 20, 1024, ctypes.byref(h)) == 0
        return h.value

    def reg(c, p, n):
        rc = L.vpcsum_ctx_register_arena(ctypes.c_void_p(c), ctypes.c_void_p(p), ctypes.c_uint64(n))
        return {"rc": rc, "err": L.vpcsum_last_error().decode() if rc else ""}

    def unreg(c, p):
        rc = L.vpcsum_ctx_unregister_arena(ctypes.c_void_p(c), ctypes.c_void_p(p))
        return {"rc": rc, "err": L.vpcsum_last_error().decode() if rc else ""}

    def destroy(c):
        rc = L.vpcsum_ctx_destroy(ctypes.c_void_p(c))
        return {"rc": rc, "err": L.vpcsum_last_error().decode() if rc else ""}

    page = mmap.PAGESIZE
    case = sys.argv[1]
    steps = []
    # page-aligned buffers of our own (mmap), so "same page" and "same address" are controlled
    buf = mmap.mmap(-1, 16 * page)
    arr = np.frombuffer(buf, np.uint8)
    p = arr.ctypes.data
    a, b = ctx(), ctx()
    if case in ("same_range", "same_range_rev"):
        n = 16 * page
        steps.append(("reg A", reg(a, p, n), attr(p)))
        steps.append(("reg B", reg(b, p, n), attr(p)))
        first, second = (a, b) if case == "same_range" else (b, a)
        steps.append(("unreg first", unreg(first, p), attr(p), attr(p + 5 * page)))
        steps.append(("unreg second", unreg(second, p), attr(p), attr(p + 5 * page)))
    elif case == "shared_page":
        steps.append(("reg A [0,1000)", reg(a, p, 1000), attr(p), attr(p + 2000)))
        steps.append(("reg B [2000,3000)", reg(b, p + 2000, 1000), attr(p), attr(p + 2000)))
        steps.append(("unreg A", unreg(a, p), attr(p), attr(p + 2000)))
        steps.append(("unreg B", unreg(b, p + 2000), attr(p), attr(p + 2000)))
    elif case == "sub_range":
        steps.append(("reg A whole", reg(a, p, 16 * page), attr(p), attr(p + 5 * page)))
        steps.append(("reg B [4p,8p)", reg(b, p + 4 * page, 4 * page), attr(p), attr(p + 5 * page)))
        steps.append(("unreg B", unreg(b, p + 4 * page), attr(p), attr(p + 5 * page)))
        steps.append(("unreg A", unreg(a, p), attr(p), attr(p + 5 * page)))
    elif case == "same_start":
        steps.append(("reg A [0,4p)", reg(a, p, 4 * page), attr(p), attr(p + 6 * page)))
        steps.append(("reg B [0,8p)", reg(b, p, 8 * page), attr(p), attr(p + 6 * page)))
        steps.append(("unreg A", unreg(a, p), attr(p), attr(p + 6 * page)))
        steps.append(("unreg B", unreg(b, p), attr(p), attr(p + 6 * page)))
    elif case == "after_double":
        n = 16 * page
        steps.append(("reg A", reg(a, p, n)))
        steps.append(("reg B", reg(b, p, n)))
        steps.append(("unreg A", unreg(a, p), attr(p)))
        steps.append(("unreg B", unreg(b, p), attr(p)))
        c = ctx()
        steps.append(("reg C [2p,6p)", reg(c, p + 2 * page, 4 * page), attr(p + 3 * page), attr(p + 8 * page)))
        steps.append(("unreg C", unreg(c, p + 2 * page), attr(p + 3 * page), attr(p + 8 * page), attr(p)))
        destroy(c)
    steps.append(("destroy", destroy(a), destroy(b), attr(p), attr(p + 5 * page)))
    print(json.dumps({"case": case, "p": hex(p), "steps": steps}))


def all_cases():
    import subprocess
    for case in ("same_range", "same_range_rev", "shared_page", "sub_range", "same_start", "after_double"):
        r = subprocess.run([sys.executable, os.path.abspath(__file__), case], capture_output=True, text=True, timeout=120)
        sys.stdout.write(r.stdout if r.returncode == 0 else json.dumps({"case": case, "rc": r.returncode,
                                                                         "stderr": r.stderr[-2000:]}) + "\n")
        sys.stdout.flush()
if __name__ == "__main__":
    if len(sys.argv) > 1:
        main()
    else:
        all_cases()
