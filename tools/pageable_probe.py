"""Does the HIP runtime keep pageable host memory page-locked after an ordinary torch copy?
(tooling, round 6: the intermittent illegal-address fault at torch's pageable copies,
DESIGN_HISTORY.md "Round 6: the intermittent fault").

Ordinary copies only, each from or into a live array: host-to-device of fresh numpy arrays of
several sizes (`torch.from_numpy(a).cuda()`, as the tests' inputs) and device-to-host
(`t.cpu()`, as their results).  After each copy, and again after a device synchronise, HIP is
asked (hipPointerGetAttributes) about every page of the host array; a page it calls page-locked
means the runtime pinned that pageable memory for the copy and kept the pin.  No copy ever
touches freed memory, so nothing here can fault.  Output: one JSON line."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402


def held(p, n):
    pts = [p, p + n - 1] + [((p >> 12) + k) << 12 for k in range(1, ((p + n - 1) >> 12) - (p >> 12))]
    return sum(1 for q in pts if V.hip_holds_registered(q)), len(pts)


def main():
    import torch
    torch.cuda.init()
    V.lib()
    res = []
    for size in (2852, 65536, 164238, 1 << 20, 1458318, 8 << 20, 64 << 20):
        for rep in range(3):
            a = np.random.default_rng(size + rep).integers(0, 256, size, dtype=np.uint8)
            t = torch.from_numpy(a).cuda()
            h2d_now = held(a.ctypes.data, a.nbytes)
            torch.cuda.synchronize()
            h2d_sync = held(a.ctypes.data, a.nbytes)
            b = t.cpu().numpy()
            d2h_now = held(b.ctypes.data, b.nbytes)
            torch.cuda.synchronize()
            d2h_sync = held(b.ctypes.data, b.nbytes)
            assert np.array_equal(a, b)
            res.append({"bytes": size, "rep": rep, "h2d_src_pages_held": h2d_now, "after_sync": h2d_sync,
                        "d2h_dst_pages_held": d2h_now, "d2h_after_sync": d2h_sync})
            del a, b, t
    print(json.dumps({"copies": res}))


if __name__ == "__main__":
    main()
