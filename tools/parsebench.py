"""Rate of the batched Ethernet parse on the GPU (tooling): 1M frames of a bench workload (IPv4 /
IPv6 EtherType written into each frame's Ethernet header), vpcsum_parse_ether_async with and
without flow tuples, then parse + verify of the parsed descriptors (the ingress pair of
INTEGRATION.md §4).  Batches rotate over >= 1 GiB of arena, as in bench.py.  Output: one JSON line.
usage: python tools/parsebench.py [--workload c2] [--iters 50]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402
from bench import ROTATE_BYTES, WORKLOADS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c2")
ap.add_argument("--iters", type=int, default=50)
args = ap.parse_args()

sid, n, stride, text = WORKLOADS[args.workload]
nb = max(1, -(-ROTATE_BYTES // (n * stride)))
arenas, offs, lens = [], [], []
for b in range(nb):
    a = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    V.synth(a, n, stride, 14, sid, 0x20241020, b * n, d)   # L3 at frame offset 14
    torch.cuda.synchronize()
    desc = V.tensor_to_desc(d)
    fr = a.view(n, stride)
    ver = torch.from_numpy(desc["l3_ver"].astype(np.uint8)).cuda()
    fr[:, 12] = torch.where(ver == 4, 0x08, 0x86).to(torch.uint8)
    fr[:, 13] = torch.where(ver == 4, 0x00, 0xDD).to(torch.uint8)
    arenas.append(a)
    offs.append(torch.arange(n, dtype=torch.int64, device="cuda") * stride)
    lens.append(torch.from_numpy((desc["l3_len"].astype(np.int64) + 14).astype(np.uint32)).cuda())
dd = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
st = torch.zeros(n, dtype=torch.uint8, device="cuda")
tu = torch.zeros(n * V.TUPLE_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
out = torch.zeros(n, dtype=torch.int32, device="cuda")


def timed(fn):
    for i in range(nb):
        fn(i)
    e0, e1 = V.Event(), V.Event()
    e0.record()
    for i in range(args.iters):
        fn(i % nb)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_ms(e1) / args.iters


res = {"workload": text, "frames": n, "batches_rotated": nb}
ms = timed(lambda i: V.parse_ether(arenas[i], offs[i], lens[i], n, dd, st))
res["parse_ms"], res["parse_Mpps"] = round(ms, 4), round(n / ms / 1e3, 1)
ms = timed(lambda i: V.parse_ether(arenas[i], offs[i], lens[i], n, dd, st, tuples=tu))
res["parse_tuples_ms"], res["parse_tuples_Mpps"] = round(ms, 4), round(n / ms / 1e3, 1)


def parse_verify(i):
    V.parse_ether(arenas[i], offs[i], lens[i], n, dd, st, tuples=tu)
    V.compute(arenas[i], dd, n, out, st, V.MODE_VERIFY)


ms = timed(parse_verify)
res["parse_tuples_verify_ms"], res["parse_tuples_verify_Mpps"] = round(ms, 4), round(n / ms / 1e3, 1)
assert int((st.cpu().numpy() & 0x80).sum()) == 0, "every synthetic frame parses"
print(json.dumps(res))
