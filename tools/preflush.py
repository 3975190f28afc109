"""Host-memory egress flush of NAT'd frames: pre-image (VPCSUM_F_PRE) vs full recompute (tooling,
VERDICT r4 "Next round" item 1).

Frames: N C5-like IPv4 TCP / UDP frames of L3 1500 B in a umem-like arena (2-KB chunks, Ethernet at
+384, L3 at +398), valid sums, then the pre-images of their addresses and ports and Java's setters
(new bytes, stale sums: the oracle's restatement, test infrastructure).  One flush = submit + wait
of the whole batch with MODE_WRITE:

* zero_copy (the arena registered: the umem case): the kernels read the frames over PCIe in place;
* staged (pageable arena): the touched 16-B blocks are gathered, copied H2D, sums copied back.

For each: `pre` (vpcsum_ctx_submit_pre, every frame F_PRE: only its header is read) and `full`
(vpcsum_ctx_submit, F_IP | F_L4: the whole segment).  Median microseconds per flush over --reps
flushes after --warmup, and the host-memory bytes each flush reads (by construction: the 16-B
chunks the kernel loads or the staging copies, plus descriptors and pre-images).  The flush
re-applies the pre-images every time (the sums drift; the work does not change); a final flush of
fresh frames is checked against the oracle (setters + full recompute).
usage: python tools/preflush.py [--n 1024] [--reps 200]"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from oracle import oracle as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1024)
ap.add_argument("--reps", type=int, default=200)
ap.add_argument("--warmup", type=int, default=20)
a = ap.parse_args()

import torch  # noqa: E402,F401
from vproxy_amd import vpcsum as V  # noqa: E402
from vproxy_amd import vswitch as S  # noqa: E402

orc = O.Oracle()
n, stride = a.n, 2048


def frames():
    """The same batch on every call: (frames after the setters, descriptors, pre-images, Java's bytes)."""
    rng = np.random.default_rng(11)
    arena, desc = orc.synth(n, stride, 398, O.SYNTH_C5, O.SEED, 7)
    orc.process(arena, desc, O.MODE_COMPUTE, write=True)
    rw = np.zeros(n, O.NAT_DTYPE)
    rw.view(np.uint8).reshape(n, 48)[:, :36] = rng.integers(0, 256, (n, 36), dtype=np.uint8)
    rw["mask"] = S.NAT_FIELDS
    pre = np.zeros(n, O.NAT_DTYPE)
    for i, d in enumerate(desc):
        pre[i] = S.record_pre_image(arena, int(d["l3_off"]), 4, int(d["l4_off"]), int(d["l4_proto"]))
    want = arena.copy()
    orc.nat_java(want, desc, rw)
    orc.nat_setters(arena, desc, rw)
    return arena, desc, pre, want


def chunks(l3_off, need):
    return ((int(l3_off) & 15) + need + 15) // 16 * 16


res = {"frames": n, "l3_len": 1500, "reps": a.reps}
arena_z, desc, pre, want = frames()
d_pre = desc.copy()
d_pre["flags"] |= O.F_PRE
arena_s = arena_z.copy()
# host bytes read per flush, by construction
fld = np.where(desc["l4_proto"] == 6, 16, 6)
need_pre = np.maximum(20, desc["l4_off"].astype(int) + fld + 2)
res["host_bytes_read_per_flush"] = {
    "full": int(sum(chunks(o, 1500) for o in desc["l3_off"]) + 16 * n),
    "pre": int(sum(chunks(o, k) for o, k in zip(desc["l3_off"], need_pre)) + 16 * n + 48 * n),
}
for kind in ("zero_copy", "staged"):
    arena = arena_z if kind == "zero_copy" else arena_s
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=n)
    if kind == "zero_copy":
        ctx.register(arena)
    out = np.zeros(n, np.uint32)
    st = np.zeros(n, np.uint8)
    for mode in ("pre", "full"):
        ts = []
        for k in range(a.warmup + a.reps):
            t0 = time.perf_counter()
            if mode == "pre":
                t = ctx.submit_pre(arena, d_pre, pre, out, st, O.MODE_WRITE)
            else:
                t = ctx.submit(arena, desc, out, st, O.MODE_WRITE)
            ctx.wait(t)
            if k >= a.warmup:
                ts.append((time.perf_counter() - t0) * 1e6)
        res[f"{kind}_{mode}_us"] = round(statistics.median(ts), 2)
        res[f"{kind}_{mode}_us_p90"] = round(float(np.percentile(ts, 90)), 2)
    # the last word: fresh frames through one pre flush equal Java's bytes
    fresh, _, _, _ = frames()
    arena[:] = fresh
    ctx.wait(ctx.submit_pre(arena, d_pre, pre, out, st, O.MODE_WRITE))
    res[f"{kind}_pre_equals_java"] = bool(np.array_equal(arena, want))
    ctx.close()
# the CPU reference point: the oracle's Java restatement (setters + full recompute) of the same
# batch on one thread
b = arena_z.copy()
t0 = time.perf_counter()
for _ in range(20):
    orc.process(b, desc, O.MODE_COMPUTE, write=True)
res["cpu_full_recompute_1thread_us"] = round((time.perf_counter() - t0) / 20 * 1e6, 1)
print(json.dumps(res))
