"""C3 by size class (tooling): K2 and the pattern probe on the whole mixed batch and on each
class's packets alone (same arena, descriptor subsets), algorithmic GB/s.  Shows which class
holds the gap between K2 and its pattern ceiling; the default build (workgroup-sorted units where
the sample finds a mixed batch) next to the same staging build without the sort (variant 79), and
verify mode.  Output: one JSON line."""
import json, os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402
from bench import WORKLOADS, algorithmic_bytes  # noqa: E402

cus = torch.cuda.get_device_properties(0).multi_processor_count
sink = torch.zeros(1024, dtype=torch.int32, device="cuda")


def timed(fn, iters=20, rounds=5):
    for _ in range(3):
        fn()
    r = []
    for _ in range(rounds):
        e0, e1 = V.Event(), V.Event()
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        r.append(e0.elapsed_ms(e1) / iters)
    return float(np.median(r))


sid, n, stride, _ = WORKLOADS["c3"]
arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
V.synth(arena, n, stride, 0, sid, 0x20241020, 0, d)
torch.cuda.synchronize()
desc = V.tensor_to_desc(d)
res = {}
for name, sel in (("all", np.ones(n, bool)), ("64", desc["l3_len"] == 64), ("576", desc["l3_len"] == 576),
                  ("1500", desc["l3_len"] == 1500)):
    sub = np.ascontiguousarray(desc[sel])
    m = len(sub)
    ds = V.desc_to_tensor(sub)
    nb = algorithmic_bytes(sub)
    out = torch.zeros(m, dtype=torch.int32, device="cuda")
    k2 = timed(lambda: V.compute(arena, ds, m, out, None, 0, 0))
    k2i = timed(lambda: V.compute(arena, ds, m, out, None, 0, 79))   # the staging build without the workgroup sort
    k2v = timed(lambda: V.compute(arena, ds, m, out, None, 1, 0))    # verify mode (out only)
    pr = min(timed(lambda: V.pattern_probe(arena, ds, m, sink, cus * b)) for b in (2, 4, 12))
    # the same reads in K2's unit order (each wave its own 64 consecutive packets)
    pu = min(timed(lambda: V.pattern_probe(arena, ds, m, sink, (cus * b) | (1 << 31))) for b in (2, 4, 5))
    res[name] = {"packets": m, "bytes": nb, "k2_ms": round(k2, 4), "k2_GBps": round(nb / k2 / 1e6, 1),
                 "k2_unsorted_GBps": round(nb / k2i / 1e6, 1), "k2_verify_GBps": round(nb / k2v / 1e6, 1),
                 "probe_GBps": round(nb / pr / 1e6, 1), "probe_unit_order_GBps": round(nb / pu / 1e6, 1),
                 "k2_frac_of_probe": round(pr / k2, 3)}
print(json.dumps(res))
