"""A mid tier for C3's 576-B class (tooling): K2's default build against the
same build with a third tier for fast-class packets of more than 4 and at most 40 chunks, on C3
and its size classes, C2 and C4, compute and verify, in alternated rounds.  Variants (C3MID_VARIANTS):
88 (8 lanes x 5 loads, one trip), 90 (the same in workgroup-sorted units only); round 6's first
run also had 86 (4 x 10, 5 waves per SIMD), 87 (4 x 5, two trips), 89 (4 x 9).  None was kept
(DESIGN.md §5 "C3"): the variants live in the library of commit 4fada6b ("C3: mid-tier A/B
variants"); build that tree's kernels.hip to re-run this.
Every variant's results are compared with the default build's first.  Output: one JSON line."""
import json, os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402
from bench import WORKLOADS, algorithmic_bytes  # noqa: E402

VARIANTS = [int(v) for v in os.environ.get("C3MID_VARIANTS", "0,88,90").split(",")]
ROUNDS = int(os.environ.get("C3MID_ROUNDS", "3"))


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = V.Event(), V.Event()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    return e0.elapsed_ms(e1) / iters


def batch(cfg):
    sid, n, stride, _ = WORKLOADS[cfg]
    arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    V.synth(arena, n, stride, 0, sid, 0x20241020, 0, d)
    torch.cuda.synchronize()
    return arena, V.tensor_to_desc(d)


cases = []
arena3, desc3 = batch("c3")
for name, sel in (("c3", None), ("c3_576", desc3["l3_len"] == 576), ("c3_1500", desc3["l3_len"] == 1500),
                  ("c3_64", desc3["l3_len"] == 64)):
    sub = desc3 if sel is None else np.ascontiguousarray(desc3[sel])
    cases.append((name, arena3, sub, V.MODE_COMPUTE))
cases.append(("c3_verify", arena3, desc3, V.MODE_VERIFY))
for cfg in ("c2", "c4"):
    a, d = batch(cfg)
    cases.append((cfg, a, d, V.MODE_COMPUTE))

prepared = []
for name, arena, desc, mode in cases:
    m = len(desc)
    ds = V.desc_to_tensor(desc)
    outs = {v: torch.zeros(m, dtype=torch.int32, device="cuda") for v in VARIANTS}
    sts = {v: torch.zeros(m, dtype=torch.uint8, device="cuda") for v in VARIANTS}
    for v in VARIANTS:
        V.compute(arena, ds, m, outs[v], sts[v], mode, v)
    torch.cuda.synchronize()
    for v in VARIANTS[1:]:
        assert torch.equal(outs[v], outs[0]) and torch.equal(sts[v], sts[0]), (name, v)
    prepared.append((name, arena, ds, m, mode, algorithmic_bytes(desc), outs[0], sts[0]))
print("results equal to the default build in every case", file=sys.stderr, flush=True)

res = {name: {str(v): [] for v in VARIANTS} for name, *_ in prepared}
for r in range(ROUNDS):
    order = VARIANTS if r % 2 == 0 else VARIANTS[::-1]
    for name, arena, ds, m, mode, nb, out, st in prepared:
        for v in order:
            ms = timed(lambda: V.compute(arena, ds, m, out, st, mode, v))
            res[name][str(v)].append(round(nb / ms / 1e6, 1))
    print(f"round {r} done", file=sys.stderr, flush=True)
summary = {}
for name in res:
    base = float(np.median(res[name]["0"]))
    summary[name] = {v: {"GBps": res[name][v], "median_vs_default": round(float(np.median(res[name][v])) / base - 1, 4)}
                     for v in res[name]}
names = {"0": "default", "86": "mid tier 4x10 (5 waves/SIMD)", "87": "mid tier 4x5", "88": "mid tier 8x5",
         "89": "mid tier 4x9 (5 waves/SIMD)", "90": "mid tier 8x5, workgroup-sorted units only"}
print(json.dumps({"variants": {str(v): names.get(str(v), "") for v in VARIANTS}, "rounds": ROUNDS, "cases": summary}))
