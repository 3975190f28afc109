"""Streaming-read ceiling vs grid size (k_read_probe over a 2 GiB buffer), for the roofline context."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402
nb = 2048 * 1048576
buf = torch.ones(nb, dtype=torch.uint8, device="cuda")
sink = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
cus = torch.cuda.get_device_properties(0).multi_processor_count
for bpc in (1, 2, 3, 4, 6, 8, 16):
    g = cus * bpc
    for _ in range(3):
        V.read_probe(buf, nb, sink, g)
    r = []
    for _ in range(5):
        e0, e1 = V.Event(), V.Event()
        e0.record()
        for _ in range(10):
            V.read_probe(buf, nb, sink, g)
        e1.record()
        r.append(nb * 10 / (e0.elapsed_ms(e1) * 1e-3) / 1e9)
    print(f"probe blocks/CU={bpc:2d} grid={g:5d}: median {np.median(r):7.1f} GB/s max {max(r):7.1f}")
