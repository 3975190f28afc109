"""C3's pattern ceiling with and without cache reuse (tooling).

bench.py prices C3 against k_pattern_probe re-reading ONE resident batch.  A 1M-packet C3 batch
touches ~805 MB of 128-B lines, so part of a repeated batch may still sit in the 256-MB Infinity
Cache; K2 and the probe may profit differently.  Here NB batches lie in NB arenas and the launches
either rotate over them (no launch finds the previous one's lines) or repeat batch 0.  Kernels: K2
(default), the probe in grid order (2 / 4 / 12 workgroups per CU) and in K2's unit order (5 / 12).
Prints one JSON line, algorithmic GB/s (median of rounds) per kernel and mode."""
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
ap.add_argument("--workload", default="c3")
ap.add_argument("--batches", type=int, default=2)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--teams", default="0")
args = ap.parse_args()

sid, n, stride, text = WORKLOADS[args.workload]
nb = args.batches
cus = torch.cuda.get_device_properties(0).multi_processor_count
arenas = [torch.zeros(n * stride, dtype=torch.uint8, device="cuda") for _ in range(nb)]
descs = [torch.zeros(n * 16, dtype=torch.uint8, device="cuda") for _ in range(nb)]
for b in range(nb):
    V.synth(arenas[b], n, stride, 0, sid, 0x20241020, b * n, descs[b])
torch.cuda.synchronize()
nbytes = [algorithmic_bytes(V.tensor_to_desc(d)) for d in descs]
out = torch.zeros(n, dtype=torch.int32, device="cuda")
sink = torch.zeros(8192, dtype=torch.int32, device="cuda")

kernels = {}
for t in map(int, args.teams.split(",")):
    kernels[f"k2_v{t}"] = (lambda t: lambda b: V.compute(arenas[b], descs[b], n, out, None, 0, t))(t)
for bpc in (2, 4, 12):
    kernels[f"probe_grid_{bpc}"] = (lambda g: lambda b: V.pattern_probe(arenas[b], descs[b], n, sink, g))(cus * bpc)
for bpc in (5, 12):
    kernels[f"probe_unit_{bpc}"] = (lambda g: lambda b: V.pattern_probe(arenas[b], descs[b], n, sink, g))(
        (cus * bpc) | (1 << 31))

res = {(k, m): [] for k in kernels for m in ("rotate", "repeat")}
e0, e1 = V.Event(), V.Event()
for r in range(args.rounds):
    for k, fn in kernels.items():
        for m in ("rotate", "repeat"):
            pick = (lambda i: i % nb) if m == "rotate" else (lambda i: 0)
            for i in range(nb):
                fn(pick(i))
            e0.record()
            for i in range(args.iters):
                fn(pick(i))
            e1.record()
            torch.cuda.synchronize()
            tot = sum(nbytes[pick(i)] for i in range(args.iters))
            res[(k, m)].append(tot / (e0.elapsed_ms(e1) * 1e-3) / 1e9)
summary = {"workload": text, "batches": nb, "algorithmic_B_per_pkt": round(nbytes[0] / n, 1),
           "GBps": {f"{k}/{m}": round(float(np.median(a)), 1) for (k, m), a in res.items()}}
print(json.dumps(summary))
