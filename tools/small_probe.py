"""Read-ceiling of small jobs: k_read_probe time vs buffer size and grid (launch ramp + drain),
to price C1 (84 HBM B/pkt x 1M = 88 MB) against what a pure read of that size achieves."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402
cus = torch.cuda.get_device_properties(0).multi_processor_count
buf = torch.ones(2048 << 20, dtype=torch.uint8, device="cuda")
sink = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
for mb in (8, 32, 88, 256, 2048):
    nb = mb << 20
    for bpc in (1, 2, 4, 8):
        g = cus * bpc
        for _ in range(3):
            V.read_probe(buf, nb, sink, g)
        r = []
        for _ in range(5):
            e0, e1 = V.Event(), V.Event()
            e0.record()
            for _ in range(20):
                V.read_probe(buf, nb, sink, g)
            e1.record()
            r.append(e0.elapsed_ms(e1) / 20 * 1e3)
        us = float(np.median(r))
        print(f"{mb:5d} MB  blocks/CU={bpc}: {us:8.1f} us  {nb / us / 1e3:7.1f} GB/s")
