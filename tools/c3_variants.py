"""C3 per size class, every kernel variant given (tooling): which kernel shape streams each class
best.  The batch's descriptors are split by class (64 / 576 / 1500 B); each subset and the whole
batch are timed with each variant id of vpcsum_compute_async (0 = default K2; 2..11, 78 = the
team-per-packet kernel, whose teams take packets in grid order) and the pattern probe in grid and
unit order.  Launches rotate over two batches (uncached).  Output: one JSON line, GB/s.
usage: python tools/c3_variants.py [--variants 0,79,78,8,9,11] [--mode 0]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402
from bench import WORKLOADS, algorithmic_bytes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="0,79,78,8,9,11")
ap.add_argument("--mode", type=int, default=0)
ap.add_argument("--bpc", default="0")
a = ap.parse_args()
cus = torch.cuda.get_device_properties(0).multi_processor_count
sink = torch.zeros(8192, dtype=torch.int32, device="cuda")
sid, n, stride, _ = WORKLOADS["c3"]
arenas = [torch.zeros(n * stride, dtype=torch.uint8, device="cuda") for _ in range(2)]
ds = [torch.zeros(n * 16, dtype=torch.uint8, device="cuda") for _ in range(2)]
for b in range(2):
    V.synth(arenas[b], n, stride, 0, sid, 0x20241020, b * n, ds[b])
torch.cuda.synchronize()
descs = [V.tensor_to_desc(d) for d in ds]


def timed(fn, iters=20, rounds=4):
    for i in range(4):
        fn(i)
    r = []
    for _ in range(rounds):
        e0, e1 = V.Event(), V.Event()
        e0.record()
        for i in range(iters):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        r.append(e0.elapsed_ms(e1) / iters)
    return float(np.median(r))


res = {}
for name in ("all", "64", "576", "1500"):
    subs = []
    for b in range(2):
        sel = np.ones(n, bool) if name == "all" else descs[b]["l3_len"] == int(name)
        subs.append(np.ascontiguousarray(descs[b][sel]))
    m = min(len(s) for s in subs)
    dt = [V.desc_to_tensor(s[:m]) for s in subs]
    nb = algorithmic_bytes(subs[0][:m])
    out = torch.zeros(m, dtype=torch.int32, device="cuda")
    st = torch.zeros(m, dtype=torch.uint8, device="cuda") if a.mode else None
    r = {"packets": m, "B_per_pkt": round(nb / m, 1)}
    for v in map(int, a.variants.split(",")):
        for bpc in map(int, a.bpc.split(",")):
            ms = timed(lambda i: V.compute(arenas[i & 1], dt[i & 1], m, out, st, a.mode, v, blocks_per_cu=bpc))
            r[f"v{v}" + (f"_b{bpc}" if bpc else "")] = round(nb / ms / 1e6, 1)
    r["probe_grid"] = round(max(nb / timed(lambda i: V.pattern_probe(arenas[i & 1], dt[i & 1], m, sink, cus * bb)) / 1e6
                                for bb in (2, 4, 12)), 1)
    r["probe_unit"] = round(max(nb / timed(lambda i: V.pattern_probe(arenas[i & 1], dt[i & 1], m, sink,
                                                                       (cus * bb) | (1 << 31))) / 1e6 for bb in (2, 4, 5)), 1)
    res[name] = r
print(json.dumps(res))
