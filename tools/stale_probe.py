"""Does HIP still hold any page of a released zero-copy arena? (tooling, round 6: the third
illegal-address fault, DESIGN_HISTORY.md "Round 6: the intermittent fault").

Repeats the host-memory sequence of `test_window_units_host_context[True]`, the test before both
faults at `test_gathered_units[2048-14]` -- a context registers a ~164-KB heap array, runs a
zero-copy verify and a zero-copy write-back into it, closes -- and then, instead of the torch
copies that faulted, only ASKS HIP (hipPointerGetAttributes) about every page of the released
range and of fresh numpy arrays of the sizes the next test allocates (its 1.46-MB input copy, its
2,852-B results, a 713-B status array).  No copy touches those arrays and no kernel reads them,
so nothing here can fault.  Output: one JSON line (iterations, how often an array reused the
released addresses, and every page HIP called page-locked that no registration holds)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from vproxy_amd import vpcsum as V  # noqa: E402


def pages(ptr, n):
    return [ptr, ptr + n - 1] + [((ptr >> 12) + k) << 12 for k in range(1, ((ptr + n - 1) >> 12) - (ptr >> 12))]


def main():
    import torch
    torch.cuda.init()
    orc = O.Oracle()
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    hits, reused = [], 0
    for it in range(iters):
        good, desc = orc.synth(64 * 40 + 5, 64, 14, O.SYNTH_C1, O.SEED, 31 + it)
        want = good.copy()
        orc.process(want, desc, O.MODE_COMPUTE, write=True)
        ctx = V.Context(0, max_arena=good.nbytes, max_pkts=len(desc))
        ctx.register(good)
        ctx.run(good, desc, O.MODE_VERIFY)
        out = np.zeros(len(desc), np.uint32)
        ctx.wait(ctx.submit(good, desc, out, None, O.MODE_WRITE))
        assert np.array_equal(good, want)
        ctx.close()
        old = (good.ctypes.data, good.nbytes)
        del good, want, out
        fresh = {"input_copy": np.empty(1458318, np.uint8), "results": np.empty(713, np.uint32),
                 "status": np.empty(713, np.uint8), "arena_164k": np.empty(164238, np.uint8)}
        for name, (p, n) in [("released", old)] + [(k, (a.ctypes.data, a.nbytes)) for k, a in fresh.items()]:
            if name != "released" and not (p + n <= old[0] or old[0] + old[1] <= p):
                reused += 1
            bad = [hex(q) for q in pages(p, n) if V.hip_holds_registered(q)]
            if bad:
                hits.append({"iter": it, "array": name, "ptr": hex(p), "bytes": n, "pages_held": bad[:8]})
        del fresh
    print(json.dumps({"iterations": iters, "fresh_arrays_overlapping_released_range": reused, "held_pages": hits}))


if __name__ == "__main__":
    main()
