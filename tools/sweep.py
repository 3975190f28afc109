"""Variant sweep of the checksum kernel on one GPU (tooling): lanes/packet x load policy x
workgroups/CU, interleaved rounds in one process (guide §5.4 rule 24), HIP-event timed."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402
from bench import WORKLOADS, algorithmic_bytes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c2")
ap.add_argument("--teams", default="2,3,4,5,6")
ap.add_argument("--bpc", default="0")
ap.add_argument("--nt", default="1,0")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--mode", type=int, default=0)
ap.add_argument("--noout", type=int, default=0)
ap.add_argument("--full", default="0", help="1 = no sampled low-concurrency grid (K2 tuning bit 14)")
ap.add_argument("--stride", type=int, default=0, help="frame stride instead of the workload's (e.g. c1 in 2-KB frames)")
args = ap.parse_args()

sid, n, stride, text = WORKLOADS[args.workload]
if args.stride:
    stride, text = args.stride, f"{text}, stride {args.stride}"
arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
V.synth(arena, n, stride, 0, sid, 0x20241020, 0, d)
torch.cuda.synchronize()
nbytes = algorithmic_bytes(V.tensor_to_desc(d))
ref = torch.zeros(n, dtype=torch.int32, device="cuda")
V.compute(arena, d, n, ref, None, 0, 4)
variants = [(t, b, nt, f) for t in map(int, args.teams.split(",")) for b in map(int, args.bpc.split(","))
            for nt in map(int, args.nt.split(",")) for f in map(int, args.full.split(","))]
res = {v: [] for v in variants}
out = torch.zeros(n, dtype=torch.int32, device="cuda")
st = torch.zeros(n, dtype=torch.uint8, device="cuda")
e0, e1 = V.Event(), V.Event()
for r in range(args.rounds):
    for v in variants:
        t, b, nt, f = v
        o_ = None if args.noout in (1, 3) else out
        s_ = None if args.noout in (1, 2) else st
        run = lambda: V.compute(arena, d, n, o_, s_, args.mode, t, plain_loads=not nt, blocks_per_cu=b,
                                 full_grid=bool(f))
        for _ in range(3):
            run()
        e0.record()
        for _ in range(args.iters):
            run()
        e1.record()
        ms = e0.elapsed_ms(e1) / args.iters
        res[v].append(nbytes / ms / 1e6)
        if r == 0 and args.noout in (0, 2) and (t < 30 or t >= 33):
            assert torch.equal(out, ref), f"variant {v} differs"
print(f"{text}: algorithmic {nbytes / n:.1f} B/pkt")
for v in variants:
    a = np.array(res[v])
    print(f"variant={v[0]} bpc={v[1] or 'def'} nt={v[2]} full={v[3]}:  median {np.median(a):7.1f} GB/s  max {a.max():7.1f}")
