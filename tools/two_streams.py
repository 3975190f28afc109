"""K2 launches back to back on one stream against two (and three) streams taking alternate batches (tooling):
does a second batch in flight hide the launch's ramp and tail?  Uncached input (batches rotated
over >= 1 GiB), algorithmic GB/s from wall clock over K launches.  Output: one JSON line.
usage: python tools/two_streams.py [c2,c1,c3] [--steps K]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402
from bench import WORKLOADS, algorithmic_bytes  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
steps = next((int(a[8:]) for a in sys.argv if a.startswith("--steps=")), 200)
res = {}
for w in (args[0].split(",") if args else ["c2", "c1", "c3"]):
    sid, n, stride, _ = WORKLOADS[w]
    nb = max(2, -(-(1 << 30) // (n * stride)))
    nb = max(nb, 3)
    arenas = [torch.zeros(n * stride, dtype=torch.uint8, device="cuda") for _ in range(nb)]
    ds = [torch.zeros(n * 16, dtype=torch.uint8, device="cuda") for _ in range(nb)]
    for b in range(nb):
        V.synth(arenas[b], n, stride, 0, sid, 0x20241020, b * n, ds[b])
    torch.cuda.synchronize()
    nbytes = algorithmic_bytes(V.tensor_to_desc(ds[0]))
    outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(3)]
    streams = [torch.cuda.current_stream(), torch.cuda.Stream(), torch.cuda.Stream()]

    def run(k_streams, k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            s = streams[i % k_streams]
            V.compute(arenas[i % nb], ds[i % nb], n, outs[i % k_streams], None, V.MODE_COMPUTE, stream=s)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    for k_streams in (1, 2, 3):
        run(k_streams, 50)
    r = {1: [], 2: [], 3: []}
    for _ in range(4):
        for k_streams in (1, 2, 3):
            r[k_streams].append(nbytes * steps / run(k_streams, steps) / 1e9)
    ref = torch.zeros(n, dtype=torch.int32, device="cuda")
    V.compute(arenas[(steps - 1) % nb], ds[(steps - 1) % nb], n, ref, None, V.MODE_COMPUTE)
    torch.cuda.synchronize()
    res[w] = {"batches": nb, "one_stream_GBps": [round(x, 1) for x in r[1]],
              "two_streams_GBps": [round(x, 1) for x in r[2]],
              "three_streams_GBps": [round(x, 1) for x in r[3]],
              "gain": round(float(np.median(r[2]) / np.median(r[1])), 4),
              "gain_three": round(float(np.median(r[3]) / np.median(r[1])), 4),
              "last_out_equal": bool(torch.equal(outs[(steps - 1) % 3], ref))}
    del arenas, ds, outs
    torch.cuda.empty_cache()
print(json.dumps(res))
