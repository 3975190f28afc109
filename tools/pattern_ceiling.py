"""Per-workload read ceiling of the frame layout: k_pattern_probe reads exactly K2's chunks
(--stride=N: another frame stride; descriptors included, no results written, no checksum work).  Prints both as algorithmic
GB/s over the same bytes, and K2's fraction of the pattern ceiling.  Output: one JSON line."""
import json, os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402
from bench import WORKLOADS, algorithmic_bytes  # noqa: E402

cus = torch.cuda.get_device_properties(0).multi_processor_count
sink = torch.zeros(1024, dtype=torch.int32, device="cuda")
res = {}


def timed(fn, iters=30, rounds=5):
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


args = [a for a in sys.argv[1:] if not a.startswith("--")]
for w in (args[0].split(",") if args else ["c2", "c3", "c4", "c1"]):
    sid, n, stride, _ = WORKLOADS[w]
    stride = next((int(a[9:]) for a in sys.argv if a.startswith("--stride=")), stride)   # e.g. c1 in 2-KB frames
    arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    V.synth(arena, n, stride, 0, sid, 0x20241020, 0, d)
    torch.cuda.synchronize()
    nb = algorithmic_bytes(V.tensor_to_desc(d))
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    probe = {bpc: timed(lambda: V.pattern_probe(arena, d, n, sink, cus * bpc)) for bpc in (2, 4, 8, 12)}
    if "--orders" in sys.argv:   # the same reads in K2's unit order, and K2's interleaved variant
        for tag, bits in (("unit_order", 1 << 31), ("pipelined", 1 << 30), ("unit_order_pipelined", 3 << 30)):
            uo = {bpc: timed(lambda: V.pattern_probe(arena, d, n, sink, (cus * bpc) | bits)) for bpc in (1, 2, 3, 4)}
            res[f"{w}_{tag}_GBps"] = {b: round(nb / t / 1e6, 1) for b, t in uo.items()}
        res[w + "_k2_variants_GBps"] = {f"{v}/{b}": round(nb / timed(lambda: V.compute(arena, d, n, out, None, 0, v, blocks_per_cu=b)) / 1e6, 1)
                                        for v in (0,) for b in (0, 2)}
    best = min(probe, key=probe.get)
    k2 = timed(lambda: V.compute(arena, d, n, out, None, 0, 0))
    res[w] = {"pattern_probe_GBps": {b: round(nb / t / 1e6, 1) for b, t in probe.items()},
              "pattern_ceiling_GBps": round(nb / probe[best] / 1e6, 1),
              "k2_GBps": round(nb / k2 / 1e6, 1), "k2_frac_of_pattern": round(probe[best] / k2, 4)}
    del arena, d, out
    torch.cuda.empty_cache()
print(json.dumps(res))
