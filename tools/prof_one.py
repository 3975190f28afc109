"""Run one checksum-kernel variant a few times (for rocprofv3 --pmc / --kernel-trace)."""
import argparse, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V
from bench import WORKLOADS
ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c2")
ap.add_argument("--variants", default="0")
ap.add_argument("--bpc", type=int, default=0)
ap.add_argument("--mode", type=int, default=0, help="checksum mode: 0 compute (out only), 1 verify (out + status)")
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--nat", type=int, default=-1, help="nat_mode: profile vpcsum_nat4_async on C5 instead")
ap.add_argument("--nat-mask", type=int, default=0x0F, help="rewrite mask of every entry (0: read-only pass)")
ap.add_argument("--nat-n", type=int, default=10_000_000, help="C5 packets (BASELINE: 10M)")
ap.add_argument("--nat-probe", action="store_true", help="the NAT pattern probe (same memory operations, no rewrite)")
ap.add_argument("--class-len", type=int, default=0, help="only the workload's packets of this L3 length (C3 classes)")
ap.add_argument("--pre", type=lambda x: int(x, 0), default=-1,
                help="vpcsum_pre_async mode bits: profile the pre-image flush on C5 (bench --preimage's step)")
a = ap.parse_args()
if a.pre >= 0:
    n, stride = a.nat_n, 2048
    arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    V.synth(arena, n, stride, 0, V.SYNTH_C5, 0x20241020, 0, d)
    V.compute(arena, d, n, None, None, V.MODE_WRITE)
    g = torch.Generator(device="cpu").manual_seed(5)
    rw = torch.randint(0, 256, (n, 16), dtype=torch.uint8, generator=g).cuda()
    fr = arena.view(n, stride)
    p4 = torch.zeros((n, 16), dtype=torch.uint8, device="cuda")
    p4[:, 0:8] = fr[:, 12:20]
    p4[:, 8:12] = fr[:, 20:24]
    p4[:, 12] = V.NAT_SRC | V.NAT_DST | V.NAT_SPORT | V.NAT_DPORT
    fr[:, 12:20] = rw[:, 0:8]
    fr[:, 20:24] = rw[:, 8:12]
    d.view(n, 16)[:, 14] |= V.F_PRE
    for _ in range(a.iters):
        V.pre(arena, d, p4, n, None, None, V.MODE_WRITE | a.pre, V.PRE_FMT_PRE4)
    torch.cuda.synchronize()
    print("done")
    sys.exit(0)
if a.nat >= 0:
    n, stride = a.nat_n, 2048
    arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    V.synth(arena, n, stride, 0, V.SYNTH_C5, 0x20241020, 0, d)
    V.compute(arena, d, n, None, None, V.MODE_WRITE)
    g = torch.Generator(device="cpu").manual_seed(5)
    rw = torch.randint(0, 256, (n, 16), dtype=torch.uint8, generator=g)
    rw[:, 12] = a.nat_mask
    rw[:, 13:] = 0
    rw = rw.cuda()
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    for _ in range(a.iters):
        if a.nat_probe:
            V.nat4_pattern_probe(arena, d, rw, n)
        else:
            V.nat4(arena, d, rw, n, st, a.nat)
    torch.cuda.synchronize()
    print("done")
    sys.exit(0)
sid, n, stride, _ = WORKLOADS[a.workload]
arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
V.synth(arena, n, stride, 0, sid, 0x20241020, 0, d)
if a.class_len:   # a size class of the batch alone (same arena, descriptor subset)
    desc = V.tensor_to_desc(d)
    sub = desc[desc["l3_len"] == a.class_len]
    n = len(sub)
    d = V.desc_to_tensor(sub)
    print("packets", n)
out = torch.zeros(n, dtype=torch.int32, device="cuda")
st = torch.zeros(n, dtype=torch.uint8, device="cuda") if a.mode == 1 else None
for v in map(int, a.variants.split(",")):
    for _ in range(a.iters):
        V.compute(arena, d, n, out, st, a.mode, v, blocks_per_cu=a.bpc)
torch.cuda.synchronize()
print("done")
