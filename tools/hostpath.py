"""Host-memory (PCIe-inclusive) rate of the checksum path, for DESIGN.md (tooling).

The vswitch path starts and ends in host memory (tap/tun buffers, AF_XDP umem).  Measured:
  * pipeline: page-locked host arena of C2 frames -> chunked H2D (2-D copy of the 1504 B each
    frame needs) || kernel || D2H of 4-B results, two streams (vpcsum_ctx_pipeline);
  * zero-copy: the kernel reads the page-locked host arena directly over PCIe;
  * submit/wait latency of small batches (the per-completeTx flush of the Java integration),
    with a kernel launch per batch and through the low-latency service grid.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402
from bench import algorithmic_bytes  # noqa: E402

res = {}
n, stride = 1 << 20, 2048
# frames generated on the device, copied once into page-locked host memory
d_arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
d_desc = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
V.synth(d_arena, n, stride, 0, V.SYNTH_C2, 0x20241020, 0, d_desc)
torch.cuda.synchronize()
# the arena as a numpy array registered with the context (page-locked + mapped by
# vpcsum_ctx_register_arena, as a umem would be): the pipeline's MODE_WRITE stores through it
arena_np = d_arena.cpu().numpy().copy()
h_arena = torch.from_numpy(arena_np).pin_memory()   # hipHostMalloc'd copy for the zero-copy kernel
desc = d_desc.cpu().numpy().view(V.DESC_DTYPE).copy()
nbytes = algorithmic_bytes(desc)
ref = torch.zeros(n, dtype=torch.int32, device="cuda")
V.compute(d_arena, d_desc, n, ref, None)
torch.cuda.synchronize()
ref_np = ref.cpu().numpy().view(np.uint32)
del d_arena

ctx = V.Context(0, max_arena=(n // 4) * stride + 4096, max_pkts=n // 4)
ctx.register(arena_np)
out = np.zeros(n, np.uint32)
# the pipeline's descriptors and results are page-locked by the context too (round 6: a context
# copies asynchronously only from memory it locked itself)
ctx.register(desc)
ctx.register(out)

pipe = {}
for chunks in (4, 8, 16, 32):
    out[:] = 0
    ctx.pipeline(arena_np, stride, 1504, desc, out, chunks=chunks)   # warm
    t = time.perf_counter()
    reps = 3
    for _ in range(reps):
        ctx.pipeline(arena_np, stride, 1504, desc, out, chunks=chunks)
    dt = (time.perf_counter() - t) / reps
    assert np.array_equal(out, ref_np)
    pipe[chunks] = {"ms": round(dt * 1e3, 3), "GBps_algorithmic": round(nbytes / dt / 1e9, 2),
                    "Mpps": round(n / dt / 1e6, 2)}
res["pipeline_h2d_kernel_d2h"] = pipe

# the same with the checksum fields written back into the host frames (MODE_WRITE: 2-B posted
# PCIe writes through the registered arena's mapping)
want_arena = arena_np.copy()
pipe = {}
for chunks in (8, 16):
    ctx.pipeline(arena_np, stride, 1504, desc, out, mode=V.MODE_WRITE, chunks=chunks)   # warm
    t = time.perf_counter()
    reps = 3
    for _ in range(reps):
        ctx.pipeline(arena_np, stride, 1504, desc, out, mode=V.MODE_WRITE, chunks=chunks)
    dt = (time.perf_counter() - t) / reps
    assert np.array_equal(out, ref_np)
    pipe[chunks] = {"ms": round(dt * 1e3, 3), "GBps_algorithmic": round(nbytes / dt / 1e9, 2),
                    "Mpps": round(n / dt / 1e6, 2)}
# every frame now carries its sums (verify from the device copy of the written arena)
d_chk = torch.from_numpy(arena_np).cuda()
st = torch.zeros(n, dtype=torch.uint8, device="cuda")
V.compute(d_chk, d_desc, n, None, st, V.MODE_VERIFY)
torch.cuda.synchronize()
assert bool(torch.all((st & 3) == 3))
del d_chk
res["pipeline_h2d_kernel_d2h_write_frames"] = pipe

# zero-copy: kernel reads the page-locked host arena in place (PCIe reads, no staging copy)
zc_out = torch.zeros(n, dtype=torch.int32, device="cuda")
h_desc_dev = d_desc
V.compute(h_arena, h_desc_dev, n, zc_out, None)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(3):
    V.compute(h_arena, h_desc_dev, n, zc_out, None)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 3
assert np.array_equal(zc_out.cpu().numpy().view(np.uint32), ref_np)
res["zero_copy_kernel_reads_host"] = {"ms": round(dt * 1e3, 3), "GBps_algorithmic": round(nbytes / dt / 1e9, 2)}

# small-batch submit/wait latency (per completeTx flush), pageable arena path
lat = {}
small_arena = arena_np[: 8192 * stride].copy()
for b in (32, 128, 1024, 8192):
    dsc = desc[:b].copy()
    o = np.zeros(b, np.uint32)
    for _ in range(5):
        ctx.wait(ctx.submit(small_arena, dsc, o))
    ts = []
    for _ in range(50):
        t = time.perf_counter()
        ctx.wait(ctx.submit(small_arena, dsc, o))
        ts.append(time.perf_counter() - t)
    assert np.array_equal(o, ref_np[:b])
    lat[b] = {"median_us": round(float(np.median(ts)) * 1e6, 1), "p99_us": round(float(np.percentile(ts, 99)) * 1e6, 1),
              "Mpps": round(b / float(np.median(ts)) / 1e6, 3)}
res["submit_wait_latency_pageable"] = lat

# zero-copy flush on a registered (page-locked, mapped) arena: what GpuCsumBatch.flush does on
# an AF_XDP umem -- kernel reads the frames over PCIe and writes the checksum fields in place
zc_arena = np.zeros(64 << 20, np.uint8)
zc_arena[: 8192 * stride] = arena_np[: 8192 * stride]
ctx.register(zc_arena)
lat = {}
for b in (32, 128, 1024, 8192):
    dsc = desc[:b].copy()
    o = np.zeros(b, np.uint32)
    for _ in range(5):
        ctx.wait(ctx.submit(zc_arena, dsc, o, None, V.MODE_WRITE))
    ts = []
    for _ in range(50):
        t = time.perf_counter()
        ctx.wait(ctx.submit(zc_arena, dsc, o, None, V.MODE_WRITE))
        ts.append(time.perf_counter() - t)
    assert np.array_equal(o, ref_np[:b])
    lat[b] = {"median_us": round(float(np.median(ts)) * 1e6, 1), "p99_us": round(float(np.percentile(ts, 99)) * 1e6, 1),
              "Mpps": round(b / float(np.median(ts)) / 1e6, 3)}
res["submit_wait_latency_zero_copy_write"] = lat

# the same flushes through the low-latency service (persistent grid polling a pinned mailbox)
ctx.set_service(200000)
lat = {}
for b in (32, 128, 1024, 8192):
    dsc = desc[:b].copy()
    o = np.zeros(b, np.uint32)
    for _ in range(5):
        ctx.wait(ctx.submit(zc_arena, dsc, o, None, V.MODE_WRITE))
    ts = []
    for _ in range(200):
        t = time.perf_counter()
        ctx.wait(ctx.submit(zc_arena, dsc, o, None, V.MODE_WRITE))
        ts.append(time.perf_counter() - t)
    assert np.array_equal(o, ref_np[:b])
    lat[b] = {"median_us": round(float(np.median(ts)) * 1e6, 1), "p99_us": round(float(np.percentile(ts, 99)) * 1e6, 1),
              "Mpps": round(b / float(np.median(ts)) / 1e6, 3)}
res["submit_wait_latency_service_zero_copy_write"] = lat
res["service_stats"] = ctx.stats()
ctx.set_service(0)
res["config"] = "C2: 1,048,576 x 1500 B IPv4/TCP, stride 2048, 1504 B copied per frame"
print(json.dumps(res))
