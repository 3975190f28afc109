"""Arenas past 4 GiB (tooling): the same batch timed through K2 on views
under 4 GiB and through the launcher on a large arena across the 4-GiB line (the team kernel with
64-bit loads; variant 78 names it explicitly).  Launches rotate over 2 copies (C2) or 16 (C1) so
no launch reads cached lines.  usage: python tools/big_arena.py [--case NAME]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402
from bench import WORKLOADS, algorithmic_bytes  # noqa: E402

CASE = sys.argv[sys.argv.index("--case") + 1] if "--case" in sys.argv else None   # one case (profiling)
res = {}
for wl, copies in ((("c2", 2),) if CASE else (("c2", 2), ("c1", 16))):
    sid, n, stride, _ = WORKLOADS[wl]
    sz = n * stride
    small = torch.zeros(copies * sz, dtype=torch.uint8, device="cuda")
    d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    V.synth(small[:sz], n, stride, 0, sid, 0x20241020, 0, d)
    for c in range(1, copies):
        small[c * sz:(c + 1) * sz] = small[:sz]
    nbytes = algorithmic_bytes(V.tensor_to_desc(d))
    base = (4 << 30) - copies * sz // 2          # the copies straddle the 4-GiB line
    big = torch.zeros(base + copies * sz + 4096, dtype=torch.uint8, device="cuda")
    big[base:base + copies * sz] = small
    dl = V.tensor_to_desc(d)
    descs_small, descs_big = [], []
    for c in range(copies):
        x = dl.copy()
        x["l3_off"] += c * sz
        descs_small.append(V.desc_to_tensor(x))
        y = dl.copy()
        y["l3_off"] += base + c * sz
        descs_big.append(V.desc_to_tensor(y))
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    ref = torch.zeros(n, dtype=torch.int32, device="cuda")
    V.compute(small, descs_small[0], n, ref)
    e0, e1 = V.Event(), V.Event()
    views = [big[base + c * sz:base + (c + 1) * sz] for c in range(copies)]
    d0 = V.desc_to_tensor(dl)
    runs = (("small_arena_k2", [small] * copies, descs_small, 0),
            # the large allocation's memory through per-copy views under 4 GiB: K2's usual path
            ("big_alloc_views_k2", views, [d0] * copies, 0),
            ("big_arena_k2", [big] * copies, descs_big, 0),
            ("big_arena_team_kernel", [big] * copies, descs_big, 78))
    for name, arenas, descs, var in runs:
        if CASE and name != CASE:
            continue
        for c in range(copies):
            V.compute(arenas[c], descs[c], n, out, None, V.MODE_COMPUTE, var)
            torch.cuda.synchronize()
            assert torch.equal(out, ref), (wl, name, c)
        best = None
        for _ in range(1 if CASE else 3):
            e0.record()
            for i in range(40):
                V.compute(arenas[i % copies], descs[i % copies], n, out, None, V.MODE_COMPUTE, var)
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_ms(e1) / 40
            best = t if best is None else min(best, t)
        res[f"{wl}_{name}"] = {"ms": round(best, 5), "GBps": round(nbytes / (best * 1e-3) / 1e9, 1)}
        print(wl, name, res[f"{wl}_{name}"], flush=True)
    del small, big
    torch.cuda.empty_cache()
print(json.dumps(res))
