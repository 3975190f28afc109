"""Phase A + C cost of K2 alone: 1M descriptors that all fail validation (no bytes streamed)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V
n, stride = 1 << 20, 2048
arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
V.synth(arena, n, stride, 0, V.SYNTH_C2, 0x20241020, 0, d)
torch.cuda.synchronize()
dv = d.view(n, 16)
out = torch.zeros(n, dtype=torch.int32, device="cuda")
for name, mut in (("valid C2", None), ("all bad (ver 0)", 12), ("ip-only (header 20 B)", 14)):
    dd = dv.clone()
    if mut == 12:
        dd[:, 12] = 0
    elif mut == 14:
        dd[:, 14] = V.F_IP
    for bpc in (0, 2, 12):
        for _ in range(3):
            V.compute(arena, dd, n, out, None, 0, 0, blocks_per_cu=bpc)
        e0, e1 = V.Event(), V.Event()
        e0.record()
        for _ in range(20):
            V.compute(arena, dd, n, out, None, 0, 0, blocks_per_cu=bpc)
        e1.record()
        print(f"{name:24s} bpc={bpc or 'def':>3}: {e0.elapsed_ms(e1) / 20 * 1e3:7.1f} us")
