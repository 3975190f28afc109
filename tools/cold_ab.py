"""A/B of kernel variants on data the caches cannot hold between launches (tooling).

The bench re-reads one resident batch, so lines a kernel leaves in the 256-MB Infinity Cache can
serve the next launch.  Here NB batches of the workload lie in NB arenas, and the launches rotate
over them: the lines touched per round exceed the cache, so each launch reads its batch from HBM.
Prints algorithmic GB/s per variant, rotating and (for comparison) repeating one batch.
usage: python tools/cold_ab.py --workload c1 --stride 2048 --teams 70,73 [--batches 4]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402
from bench import WORKLOADS, algorithmic_bytes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c1")
ap.add_argument("--stride", type=int, default=0)
ap.add_argument("--teams", default="70,73")
ap.add_argument("--batches", type=int, default=4)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--iters", type=int, default=40)
ap.add_argument("--mode", type=int, default=0, help="0 compute, 1 verify (status bytes written too)")
ap.add_argument("--no-out", action="store_true", help="no out words (verify: the status bytes are the result)")
ap.add_argument("--packets", type=int, default=0, help="packets per batch instead of the workload's")
ap.add_argument("--bpc", default="0", help="workgroups per CU to try (0 = the launcher's choice)")
args = ap.parse_args()

sid, n, stride, text = WORKLOADS[args.workload]
stride = args.stride or stride
n = args.packets or n
nb = args.batches
# one arena per batch (each below 4 GiB, as K2's buffer addressing needs), disjoint sub-streams
arenas = [torch.zeros(n * stride, dtype=torch.uint8, device="cuda") for _ in range(nb)]
descs = [torch.zeros(n * 16, dtype=torch.uint8, device="cuda") for _ in range(nb)]
for b in range(nb):
    V.synth(arenas[b], n, stride, 0, sid, 0x20241020, b * n, descs[b])
torch.cuda.synchronize()
nbytes = algorithmic_bytes(V.tensor_to_desc(descs[0]))
out = torch.zeros(n, dtype=torch.int32, device="cuda")
st = torch.zeros(n, dtype=torch.uint8, device="cuda") if args.mode & 1 else None
ref = torch.zeros(n, dtype=torch.int32, device="cuda")
variants = [(int(t), int(b)) for t in args.teams.split(",") for b in args.bpc.split(",")]
V.compute(arenas[1], descs[1], n, ref, None, 0, 4)
for t, b in variants:   # every variant's results, once
    V.compute(arenas[1], descs[1], n, out, None, 0, t, blocks_per_cu=b)
    assert torch.equal(out, ref), f"variant {t} differs"
o = None if args.no_out else out
res = {(t, b, m): [] for t, b in variants for m in ("rotate", "repeat")}
e0, e1 = V.Event(), V.Event()
for r in range(args.rounds):
    for t, b in variants:
        for m in ("rotate", "repeat"):
            pick = (lambda i: i % nb) if m == "rotate" else (lambda i: 0)
            for i in range(nb):
                V.compute(arenas[pick(i)], descs[pick(i)], n, o, st, args.mode, t, blocks_per_cu=b)
            e0.record()
            for i in range(args.iters):
                V.compute(arenas[pick(i)], descs[pick(i)], n, o, st, args.mode, t, blocks_per_cu=b)
            e1.record()
            torch.cuda.synchronize()
            res[(t, b, m)].append(nbytes / (e0.elapsed_ms(e1) / args.iters) / 1e6)
print(f"{text}, stride {stride}, {nb} batches of {n} packets: algorithmic {nbytes / n:.1f} B/pkt, mode {args.mode}"
      f"{', no out' if args.no_out else ''}")
for (t, b, m), a in res.items():
    print(f"variant={t} bpc={b or 'def'} {m:6s}: median {np.median(a):7.1f} GB/s  max {max(a):7.1f}")
