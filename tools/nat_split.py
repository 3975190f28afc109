"""Why do two NAT launches side by side beat one? (tooling, round 6).

The one-GPU rehearsals of the C5 bench with two ranks (`profiles/r05z_bench_c5_2rank.json`,
`r06w_bench_c5_2rank.json`) move the 10M NAT'd frames at 20.4-20.5 Gpps in aggregate -- each rank
a 5M-packet half, both kernels resident on the card at once -- against 16.8 Gpps for the same
frames in one launch.  This separates the candidate causes in one process, on one 20.5-GB C5 arena,
rounds alternated (Gpps over the 10M packets, HIP events):
  one        one launch over the 10M packets (the bench's step)
  halves     two launches of 5M one after the other on one stream
  halves2s   the two halves on two streams forked from one and joined back (concurrent)
  quarters4s four quarters on four streams
  half       the first 5M packets alone (a half-size launch; rate over its own packets)
  allocs     the same 10M packets as two separate 10.24-GB allocations (5M each, as the two ranks
             hold them), one launch each, one after the other
  allocs2s   the two allocations' launches on two streams at once
Output: one JSON line."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402
from bench import WORKLOADS, SEED  # noqa: E402

sid, n, stride, _ = WORKLOADS["c5"]
arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
V.synth(arena, n, stride, 0, sid, SEED, 0, d)
V.compute(arena, d, n, None, None, V.MODE_WRITE)
rw_np = np.zeros(n, V.NAT4_DTYPE)
g = np.random.default_rng(SEED)
rw_np.view(np.uint8).reshape(-1, 16)[:, :12] = g.integers(0, 256, (n, 12), dtype=np.uint8)
rw_np["mask"] = V.NAT_SRC | V.NAT_DST | V.NAT_SPORT | V.NAT_DPORT
rw = torch.from_numpy(rw_np.view(np.uint8).copy()).cuda()
h = n // 2
sep = []   # the two ranks' layout: each half its own allocation, frames synthesized in place
for k in range(2):
    a2 = torch.zeros(h * stride, dtype=torch.uint8, device="cuda")
    d2 = torch.zeros(h * 16, dtype=torch.uint8, device="cuda")
    V.synth(a2, h, stride, 0, sid, SEED, k * h, d2)
    V.compute(a2, d2, h, None, None, V.MODE_WRITE)
    sep.append((a2, d2, rw[k * h * 16:(k + 1) * h * 16]))
torch.cuda.synchronize()
main = torch.cuda.current_stream()
side = [torch.cuda.Stream() for _ in range(4)]


def part(k, parts):
    lo, hi = n * k // parts, n * (k + 1) // parts
    return d[lo * 16:hi * 16], rw[lo * 16:hi * 16], hi - lo


def run(form):
    if form == "one":
        V.nat4(arena, d, rw, n, None, V.NAT_RFC1624, stream=main)
    elif form == "half":
        dd, rr, m = part(0, 2)
        V.nat4(arena, dd, rr, m, None, V.NAT_RFC1624, stream=main)
    elif form == "allocs":
        for a2, d2, r2 in sep:
            V.nat4(a2, d2, r2, h, None, V.NAT_RFC1624, stream=main)
    elif form == "allocs2s":
        e = torch.cuda.Event()
        e.record(main)
        for k, (a2, d2, r2) in enumerate(sep):
            side[k].wait_event(e)
            V.nat4(a2, d2, r2, h, None, V.NAT_RFC1624, stream=side[k])
        for k in range(2):
            ev = torch.cuda.Event()
            ev.record(side[k])
            main.wait_event(ev)
    elif form == "halves":
        for k in range(2):
            dd, rr, m = part(k, 2)
            V.nat4(arena, dd, rr, m, None, V.NAT_RFC1624, stream=main)
    else:
        parts = 2 if form == "halves2s" else 4
        e = torch.cuda.Event()
        e.record(main)
        for k in range(parts):
            side[k].wait_event(e)
            dd, rr, m = part(k, parts)
            V.nat4(arena, dd, rr, m, None, V.NAT_RFC1624, stream=side[k])
        for k in range(parts):
            ev = torch.cuda.Event()
            ev.record(side[k])
            main.wait_event(ev)


FORMS = ["one", "halves", "halves2s", "quarters4s", "half", "allocs", "allocs2s"]
res = {f: [] for f in FORMS}
for _ in range(300):   # clocks up
    run("one")
torch.cuda.synchronize()
iters = 30
for r in range(4):
    for f in (FORMS if r % 2 == 0 else FORMS[::-1]):
        run(f)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        for _ in range(iters):
            run(f)
        e1.record(main)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        pk = n // 2 if f == "half" else n
        res[f].append(round(pk / ms / 1e6, 2))
    print(f"round {r} done", file=sys.stderr, flush=True)
print(json.dumps({"Gpps": res, "median": {f: float(np.median(v)) for f, v in res.items()}, "packets": n}))
