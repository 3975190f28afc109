"""Pre-image flush (vpcsum_pre_async, VPCSUM_F_PRE) shapes on BASELINE config C5's frames, against
its probe build and the NAT rewrite, interleaved rounds (tooling).

The frames: C5 (10M x 1500 B IPv4 TCP / UDP, valid sums), the 16-B pre-images of their addresses
and ports, Java's setters applied (new bytes, stale sums), F_PRE on every descriptor.  Each shape
is the mode's tuning word of vpcsum_pre_async (nat.hip launch_pre); the flush is re-applied every
launch (the sums drift, the work does not change).  At the end a fresh flush is verified.
usage: python tools/presweep.py [--n N] [--modes 0,0x1000,...] [--nat]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--modes", default="0")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--nat", action="store_true", help="also the NAT rewrite (vpcsum_nat4_async) on the same frames")
a = ap.parse_args()
n, stride = a.n, 2048
arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
g = torch.Generator(device="cpu").manual_seed(5)
rw = torch.randint(0, 256, (n, 16), dtype=torch.uint8, generator=g)
rw[:, 12] = V.NAT_SRC | V.NAT_DST | V.NAT_SPORT | V.NAT_DPORT
rw[:, 13:] = 0
rw = rw.cuda()


def prep():
    V.synth(arena, n, stride, 0, V.SYNTH_C5, 0x20241020, 0, d)
    V.compute(arena, d, n, None, None, V.MODE_WRITE)
    fr = arena.view(n, stride)
    p4 = torch.zeros((n, 16), dtype=torch.uint8, device="cuda")
    p4[:, 0:8] = fr[:, 12:20]
    p4[:, 8:12] = fr[:, 20:24]
    p4[:, 12] = V.NAT_SRC | V.NAT_DST | V.NAT_SPORT | V.NAT_DPORT
    fr[:, 12:20] = rw[:, 0:8]
    fr[:, 20:24] = rw[:, 8:12]
    d.view(n, 16)[:, 14] |= V.F_PRE
    torch.cuda.synchronize()
    return p4


pre = prep()
dn = d.clone()
dn.view(n, 16)[:, 14] &= 0xFF ^ V.F_PRE
shapes = [("probe", 0x800000)] + [(f"pre_{m}", int(m, 0)) for m in a.modes.split(",")]
if a.nat:
    shapes.append(("nat", None))
res = {"packets": n}
for _ in range(a.rounds):
    for name, mode in shapes:
        def run():
            if mode is None:
                V.nat4(arena, dn, rw, n, None, V.NAT_RFC1624)
            else:
                V.pre(arena, d, pre, n, None, None, V.MODE_WRITE | mode, V.PRE_FMT_PRE4)
        for _ in range(3):
            run()
        e0, e1 = V.Event(), V.Event()
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_ms(e1) / a.iters
        res.setdefault(name, []).append(round(n / ms / 1e3, 1))   # Mpps
pre = prep()
V.pre(arena, d, pre, n, None, None, V.MODE_WRITE, V.PRE_FMT_PRE4)
st = torch.zeros(n, dtype=torch.uint8, device="cuda")
V.compute(arena, dn, n, None, st, V.MODE_VERIFY)
torch.cuda.synchronize()
res["all_verify"] = bool(((st & 3) == 3).all())
print(json.dumps(res))
