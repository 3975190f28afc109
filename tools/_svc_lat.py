import sys, time, numpy as np
sys.path.insert(0, '.')
import torch
from vproxy_amd import vpcsum as V
from oracle import oracle as O
orc = O.Oracle()
a, d = orc.synth(8192, 2048, 0, O.SYNTH_C2, O.SEED, 0)
arena = np.zeros(64 << 20, np.uint8); arena[:a.size] = a
ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=8192)
ctx.register(arena)
ctx.set_service(200000)
for b in (32, 1024):
    dsc = d[:b].copy(); o = np.zeros(b, np.uint32)
    for i in range(12):
        t = time.perf_counter()
        ctx.wait(ctx.submit(arena, dsc, o, None, V.MODE_WRITE))
        print(b, "host us", round((time.perf_counter() - t) * 1e6, 1), flush=True)
ctx.set_service(0)
