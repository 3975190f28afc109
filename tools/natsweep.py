"""NAT (BASELINE config C5) kernel shapes against the NAT pattern probe, interleaved rounds (tooling).

Times vpcsum_nat4_async in the bench's form (RFC 1624, no status, every packet's addresses and
ports rewritten) for each nat_mode tuning word given, and the pattern probe
(vpcsum_nat4_pattern_probe_async) with the tuning word in VPCSUM_NAT_PROBE_TUNE (read once per
process: run the tool once per probe shape).
With --rec, the same shapes over vpcsum_nat4_rec_t records (descriptor + entry in one 32-B record,
vpcsum_nat4r_async) and their probe, interleaved with the two-stream form.
usage: VPCSUM_NAT_PROBE_TUNE=0x20000 python tools/natsweep.py [--n N] [--modes 0,0x20000,...] [--rec]"""
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
ap.add_argument("--rec", action="store_true", help="also the 32-B record format (vpcsum_nat4r_async)")
a = ap.parse_args()
n, stride = a.n, 2048
arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
V.synth(arena, n, stride, 0, V.SYNTH_C5, 0x20241020, 0, d)
V.compute(arena, d, n, None, None, V.MODE_WRITE)
g = torch.Generator(device="cpu").manual_seed(5)
rw = torch.randint(0, 256, (n, 16), dtype=torch.uint8, generator=g)
rw[:, 12] = V.NAT_SRC | V.NAT_DST | V.NAT_SPORT | V.NAT_DPORT
rw[:, 13:] = 0
rw = rw.cuda()
rec = torch.cat([d.view(n, 16), rw.view(n, 16)], dim=1).contiguous() if a.rec else None
shapes = [("probe", None)] + [(f"nat_{m}", int(m, 0)) for m in a.modes.split(",")]
if a.rec:
    shapes += [("probe_rec", None)] + [(f"rec_{m}", int(m, 0)) for m in a.modes.split(",")]
res = {"packets": n, "probe_tune": os.environ.get("VPCSUM_NAT_PROBE_TUNE", "0")}
for _ in range(a.rounds):
    for name, mode in shapes:
        def run():
            if name == "probe_rec":
                V.nat4r_pattern_probe(arena, rec, n)
            elif mode is None:
                V.nat4_pattern_probe(arena, d, rw, n)
            elif name.startswith("rec_"):
                V.nat4r(arena, rec, n, None, V.NAT_RFC1624 | mode)
            else:
                V.nat4(arena, d, rw, n, None, V.NAT_RFC1624 | mode)
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
# every shape leaves the same bytes (the rewrite is idempotent once applied): verify all packets
st = torch.zeros(n, dtype=torch.uint8, device="cuda")
V.compute(arena, d, n, None, st, V.MODE_VERIFY)
torch.cuda.synchronize()
res["all_verify"] = bool(((st & 3) == 3).all())
print(json.dumps(res))
