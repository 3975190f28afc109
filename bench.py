#!/usr/bin/env python3
"""bench.py -- device-resident batched IPv4+TCP checksum throughput (BASELINE.json metric).

One "step" = one pass of the hot path (libvpcsum's checksum kernel, via the C-ABI) over one
device-resident batch.  Default: BASELINE config C2, 1,048,576 synthetic IPv4/TCP packets of L3
1500 B per GPU (umem-like 2048 B frame stride), IP header + TCP checksums computed for every
packet.  `value` = algorithmic bytes of all ranks (1,520 B/packet: 1500 read + 16 B descriptor
+ 4 B results) / max-over-ranks wall time of the K timed steps.

Multi-GPU: one process per GPU.  `--gpus N` without a launcher starts the N ranks itself (a child
`torch.distributed.run`, before this process touches the GPU); under torchrun the ranks come from
the environment.  Each rank has its own batch and stream; torch.distributed (gloo, CPU) carries only
the start/stop barriers and the max-over-ranks reductions -- the data path has no collective
(SURVEY.md §8e).  Weak scaling by default (a fixed batch per GPU, disjoint splitmix64 sub-streams);
`--strong` splits ONE global batch by bytes (vproxy_amd/shard.py:shard_by_bytes).

Other workloads: c1, c3, c4 (BASELINE configs; `--workload c4 --strong` is C4's 262,144 x 9000 B
batch sharded over the GPUs) and c5 (NAT rewrite, RFC 1624, 10M packets split over the GPUs).

Uncached input: a batch smaller than 1 GiB (C1's 64-MB arena) is measured with the launches
rotating over several batches of the same config, so that the Infinity Cache cannot serve one
launch from the lines of the previous (`config.batches_rotated`).

Correctness gate: rank 0's GPU results are compared word for word with the oracle's on the packets
the cpu_baseline leg processes (the whole batch when its budget allows); every rank also writes its
sums in place and verifies them (size-independent property).

`--workload c5 --preimage`: C5's frames after Java's setters (new addresses and ports, stale sums)
with the 16-B pre-images of the old values; a step is the egress flush that updates their sums
from the pre-images (vpcsum_pre_async, RFC 1624, only the headers read).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c1|c3|c4|c5] [--strong]
       [--preimage] [--share-gpu]   (more ranks than GPUs: a same-card rehearsal, reported as such)
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "device-resident GB/s, batched IPv4+TCP checksum, 1500B pkts, 1/2/4/8 GPU"
SEED = 0x20241020
NAT_BYTES_PER_PKT = 72   # 40 B header read + 16 B rewrite + 12 B rewritten + 4 B sums
# c5 --preimage (the egress flush of NAT'd frames, VPCSUM_F_PRE): 16 B descriptor + 16 B pre-image
# read + 40 B header read + 4 B sums written
PRE_BYTES_PER_PKT = 76
# The timed launches rotate over batches whose arenas hold at least this many bytes together, so
# that no launch reads input the 256-MB Infinity Cache kept from the previous one (C1's whole
# 64-MB batch would otherwise be served from it: +10%)
ROTATE_BYTES = 1 << 30

WORKLOADS = {
    # name: (synth id, packets per GPU (weak) / in the global batch (strong), frame stride, text)
    "c2": (2, 1 << 20, 2048, "C2: 1,048,576 x L3 1500 B IPv4/TCP (IP hdr + TCP csum), stride 2048"),
    "c1": (1, 1 << 20, 64, "C1: 1,048,576 x L3 50 B IPv4/UDP (64 B frames)"),
    "c3": (3, 1 << 20, 2048, "C3: 1,048,576 mixed {64,576,1500} x {UDP,TCP,ICMP}"),
    "c4": (4, 1 << 18, 9216, "C4: 262,144 x L3 9000 B IPv6/TCP"),
    "c5": (6, 10_000_000, 2048, "C5: NAT rewrite (RFC 1624) of 10,000,000 x L3 1500 B IPv4 TCP/UDP, "
                                "src/dst IP + ports"),
}


def algorithmic_bytes(desc: np.ndarray) -> int:
    """sum of L3 bytes read + 16 B descriptor + 2 B per checksum written."""
    nck = ((desc["flags"] & 1) > 0).astype(np.int64) + ((desc["flags"] & 2) > 0).astype(np.int64)
    return int(desc["l3_len"].astype(np.int64).sum() + 16 * len(desc) + 2 * nck.sum())


def host_cores() -> dict:
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota if one is set
    (the GPU box shows the whole machine in the mask but grants a share of it)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    return {"affinity": aff, "cgroup_quota": quota, "usable": min(aff, quota) if quota else aff}


def cpu_baseline(workload: str, synth_id: int, stride: int, first: int, budget_s: float = 6.0) -> tuple[dict, tuple]:
    """Oracle (C restatement of Utils.java:778-801, per-step carry fold, -O2) on the host cores,
    single thread and all usable cores, on a bounded sample of the same workload (rank 0's first
    packets).  Returns the baseline and (n, out, status) of the oracle for the correctness gate."""
    from oracle import oracle as O
    orc = O.Oracle()
    n0 = 20000
    arena, desc = orc.synth(n0, stride, 0, synth_id, SEED, first)
    t = time.perf_counter()
    orc.process(arena, desc)
    dt0 = max(time.perf_counter() - t, 1e-4)
    n1 = int(min(max(n0 * budget_s / dt0, n0), WORKLOADS[workload][1]))
    arena, desc = orc.synth(n1, stride, 0, synth_id, SEED, first)
    nbytes = algorithmic_bytes(desc)
    t = time.perf_counter()
    out, status = orc.process(arena, desc)
    t1 = time.perf_counter() - t
    cores = host_cores()
    threads = cores["usable"]
    reps = max(1, int(budget_s / max(t1 / threads, 1e-3)))
    t = time.perf_counter()
    for _ in range(reps):
        orc.process(arena, desc, threads=threads)
    tn = time.perf_counter() - t
    return {
        "value": round(nbytes * reps / tn / 1e9, 4),
        "unit": "GB/s",
        "cores": threads,
        "cores_visible": cores,
        "kind": "port",
        "sample": f"{n1} packets of {workload} ({nbytes / 1e6:.1f} MB algorithmic), "
                  f"{reps} passes on {threads} threads; Java-algorithm C (oracle/csum_oracle.c, gcc -O2)",
        "single_thread_GBps": round(nbytes / t1 / 1e9, 4),
        "single_thread_Mpps": round(n1 / t1 / 1e6, 3),
    }, (n1, out, status)


def cpu_baseline_nat(rw_np: np.ndarray, budget_s: float = 6.0) -> tuple[dict, tuple]:
    """C5 on the host: the oracle's Java-semantics rewrite (setters + full recompute,
    SwitchUtils.applyNat, SwitchUtils.java:522-542) on a bounded sample, 1 thread and all cores."""
    from oracle import oracle as O
    orc = O.Oracle()
    m = min(1 << 18, len(rw_np))
    a0, d0 = orc.synth(m, 2048, 0, O.SYNTH_C5, SEED, 0)
    orc.process(a0, d0, write=True)                 # valid input checksums
    a = a0.copy()
    t = time.perf_counter()
    orc.nat4_java(a, d0, rw_np[:m], threads=1)
    t1 = time.perf_counter() - t
    cores = host_cores()
    th = cores["usable"]
    reps = max(1, int(budget_s / max(t1 / th, 1e-3)))
    t = time.perf_counter()
    for _ in range(reps):
        b = a0.copy()
        orc.nat4_java(b, d0, rw_np[:m], threads=th)
    tn = time.perf_counter() - t
    return {
        "value": round(m * reps * NAT_BYTES_PER_PKT / tn / 1e9, 4),
        "unit": "GB/s",
        "cores": th,
        "cores_visible": cores,
        "kind": "port",
        "sample": f"{m} C5 packets, {reps} passes on {th} threads (array copy included); strict Java "
                  f"semantics: setters + full recompute (oracle/csum_oracle.c:orc_nat4_java, gcc -O2)",
        "single_thread_Mpps": round(m / t1 / 1e6, 3),
        "all_cores_Mpps": round(m * reps / tn / 1e6, 3),
    }, (m, a0, d0, a)


def oracle_sample_gate(synth_id: int, stride: int, first: int, out_np: np.ndarray, m: int = 4096) -> dict:
    """The checker on every rank: a contiguous block of m packets of this rank's slice (first =
    its first packet's index in the synthetic stream), regenerated on the host and checksummed by
    the oracle, must equal the GPU's words."""
    from oracle import oracle as O
    n = len(out_np)
    m = min(m, n)
    off = (n - m) // 2
    a, d = O.Oracle().synth(m, stride, 0, synth_id, SEED, first + off)
    want, _ = O.Oracle().process(a, d)
    return {"sample_packets": int(m), "sample_first": int(first + off),
            "sample_equal": bool(np.array_equal(out_np[off:off + m], want))}


def pmc_traffic(tag: str, packets: int, profiles: str | None = None, src: str | None = None):
    """HBM bytes per launch of the dominant kernel from a committed rocprofv3 PMC summary
    (profiles/r*_pmc_<tag>/summary.json, tools/save_profiles.py: 2 x FETCH_SIZE + WRITE_SIZE, every
    read request being 128 B), scaled from the summary's packet count to this rank's `packets` (a
    strong shard holds part of the batch).  PMC counters cannot be read from inside this process,
    so the value comes from that separate --pmc run of the same kernel and config.

    Which summary: one measured on the library sources this process runs (`src_hash` equal to
    vproxy_amd/build.py:source_hash, the newest commit of those); when no summary matches, the
    newest by commit time (never by tag name), reported as stale.  Returns (bytes, provenance)."""
    import glob
    if src is None:
        from vproxy_amd.build import source_hash
        src = source_hash()
    cands = []
    for f in glob.glob(os.path.join(profiles or os.path.join(REPO, "profiles"), f"r*_pmc_{tag}", "summary.json")):
        d = json.load(open(f))
        if "hbm_bytes_per_launch" in d and d.get("packets"):
            cands.append((d.get("src_hash") == src, d.get("head_time", 0), f, d))
    if not cands:
        return None, None
    match = [c for c in cands if c[0]]
    same, _, f, d = max(match or cands, key=lambda c: (c[1], c[2]))
    return int(round(d["hbm_bytes_per_launch"] * packets / d["packets"])), {
        "source": os.path.relpath(f, profiles or REPO) if profiles else os.path.relpath(f, REPO),
        "head": d.get("head"), "src_hash": d.get("src_hash"), "stale": not same}


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int) -> int:
    """`--gpus N` without a launcher: run the N ranks as children of torch.distributed.run (this
    process has not touched the GPU) and return their exit code."""
    argv = sys.argv[1:]
    if "--gpus" not in argv and not any(a.startswith("--gpus=") for a in argv):
        argv = argv + ["--gpus", str(n)]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def launch_stats(ms: list[float]) -> dict:
    a = np.array(ms)
    k = min(5, len(a))
    return {"min": round(float(a.min()), 5), "median": round(float(np.median(a)), 5),
            "max": round(float(a.max()), 5), "first5_mean": round(float(a[:k].mean()), 5),
            "last5_mean": round(float(a[-k:].mean()), 5)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE under a launcher, else 1)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="allow more ranks than visible GPUs (ranks share cards: a rehearsal, "
                         "marked so in the line, never a scaling point)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--strong", action="store_true", help="split one global batch over the GPUs (c5: always)")
    ap.add_argument("--preimage", action="store_true",
                    help="c5: time the egress flush of the NAT'd frames from their pre-images (VPCSUM_F_PRE) "
                         "instead of the NAT rewrite")
    ap.add_argument("--team", type=int, default=0, help="kernel variant id (0 = library default)")
    ap.add_argument("--ramp-ms", type=float, default=3000.0,
                    help="run the step kernel this long before the warm-up (clock ramp; reported)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=6.0)
    args = ap.parse_args()

    import torch   # device_count() does not initialise the GPU on this image
    ndev = torch.cuda.device_count()
    under_launcher = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1")) if under_launcher else (args.gpus or 1)
    if args.gpus is not None and args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch with matching counts")
    if world > ndev and not args.share_gpu:
        sys.exit(f"bench.py: {world} ranks but {ndev} visible GPU(s): one rank per GPU "
                 f"(pass --share-gpu for a same-card rehearsal)")
    if not under_launcher and world > 1:
        sys.exit(launch_ranks(world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    # one process per GPU; with --share-gpu the ranks wrap around the visible cards (a rehearsal
    # of the multi-rank path on a small box: devices_distinct in the line says how many cards ran)
    torch.cuda.set_device(local % max(ndev, 1))
    from vproxy_amd import vpcsum as V
    from vproxy_amd.shard import all_ranks_ok, gather_over_ranks, max_over_ranks, shard_by_bytes, sum_over_ranks
    from vproxy_amd.build import source_hash
    V.lib()

    synth_id, n_cfg, stride, desc_text = WORKLOADS[args.workload]
    nat = args.workload == "c5"
    pre = nat and args.preimage
    if args.preimage and not nat:
        sys.exit("bench.py: --preimage is a c5 workload option")
    if pre:
        desc_text = ("C5 egress flush of NAT'd frames from 16-B pre-images (RFC 1624, VPCSUM_F_PRE) of "
                     "10,000,000 x L3 1500 B IPv4 TCP/UDP after Java's setters (src/dst IP + ports)")
    strong = args.strong or nat
    stream = torch.cuda.current_stream()
    if strong:
        # one global batch, cut by bytes: the global descriptors alone give the cut, then this rank
        # generates and holds only its own packets [lo, hi) of the global stream (a rank-sized
        # arena, not the whole batch: C5's 10M x 2 KB would be 20.5 GB on every rank)
        d_glob = torch.zeros(n_cfg * 16, dtype=torch.uint8, device="cuda")
        V.synth(None, n_cfg, stride, 0, synth_id, SEED, 0, d_glob, stream=stream)
        torch.cuda.synchronize()
        lo, hi = shard_by_bytes(V.tensor_to_desc(d_glob)["l3_len"], world)[rank]
        del d_glob
        n_gen, first = hi - lo, lo
    else:
        n_gen, first = n_cfg, rank * n_cfg
    # batches of the rotation, carved from one allocation (each batch its own arena view)
    nb = 1 if (nat or n_gen * stride >= ROTATE_BYTES or n_gen == 0) else min(64, -(-ROTATE_BYTES // (n_gen * stride)))
    arena_all = torch.zeros(max(nb * n_gen * stride, 16), dtype=torch.uint8, device="cuda")
    arenas = [arena_all[b * n_gen * stride:(b + 1) * n_gen * stride] for b in range(nb)]
    d_alls = [torch.zeros(max(n_gen, 1) * 16, dtype=torch.uint8, device="cuda") for _ in range(nb)]
    for b in range(nb):   # batch b > 0: a disjoint sub-stream after every rank's batch 0
        V.synth(arenas[b], n_gen, stride, 0, synth_id, SEED, first + b * world * n_cfg, d_alls[b], stream=stream)
    torch.cuda.synchronize()
    arena, d = arenas[0], d_alls[0]
    n = n_gen
    desc_np = V.tensor_to_desc(d)[:n]
    out = torch.zeros(max(n, 1), dtype=torch.int32, device="cuda")
    status = torch.zeros(max(n, 1), dtype=torch.uint8, device="cuda")

    if nat:
        # valid input checksums, then a per-packet rewrite of src/dst IP and ports (seeded table,
        # regenerable on the host for the gate)
        V.compute(arena, d, n, None, None, V.MODE_WRITE, stream=stream)
        rw_np = np.zeros(n_cfg, V.NAT4_DTYPE)   # the global table; this rank's entries [first, +n)
        g = np.random.default_rng(SEED)
        rw_np.view(np.uint8).reshape(-1, 16)[:, :12] = g.integers(0, 256, (n_cfg, 12), dtype=np.uint8)
        rw_np["mask"] = V.NAT_SRC | V.NAT_DST | V.NAT_SPORT | V.NAT_DPORT
        rw_np = np.ascontiguousarray(rw_np[first:first + n])
        rw = torch.from_numpy(rw_np.view(np.uint8).copy()).cuda()
        bytes_per_step = n * (PRE_BYTES_PER_PKT if pre else NAT_BYTES_PER_PKT)
        pre_img = None

        def prep_pre():
            # the frames as the egress flush receives them: the pre-image of the old addresses and
            # ports (16-B vpcsum_pre4_t), then Java's setters (new bytes, stale sums; plumbing,
            # emulating Ipv4Packet.setSrc / setDst and Tcp/UdpPacket.setSrcPort / setDstPort),
            # then F_PRE on every descriptor.  Synthetic C5: L3 at the frame start, IHL 5.
            fr = arena.view(n, stride)
            p4 = torch.zeros((n, 16), dtype=torch.uint8, device="cuda")
            p4[:, 0:8] = fr[:, 12:20]
            p4[:, 8:12] = fr[:, 20:24]
            p4[:, 12] = V.NAT_SRC | V.NAT_DST | V.NAT_SPORT | V.NAT_DPORT
            rw2 = rw.view(n, 16)
            fr[:, 12:20] = rw2[:, 0:8]
            fr[:, 20:24] = rw2[:, 8:12]
            d.view(n, 16)[:, 14] |= V.F_PRE
            torch.cuda.synchronize()
            return p4

        if pre and n:
            pre_img = prep_pre()

        def step(i=0):
            if pre:
                V.pre(arena, d, pre_img, n, None, None, V.MODE_WRITE, V.PRE_FMT_PRE4, stream=stream)
            else:
                V.nat4(arena, d, rw, n, None, V.NAT_RFC1624, stream=stream)
    else:
        bytes_per_step = algorithmic_bytes(desc_np)
        ds = d_alls
        batch_bytes = [bytes_per_step] + [algorithmic_bytes(V.tensor_to_desc(dd)[:n]) for dd in d_alls[1:]]

        def step(i=0):
            # one pass over batch i mod nb: every IP header + L4 checksum -> out (4 B/packet)
            V.compute(arenas[i % nb], ds[i % nb], n, out, None, V.MODE_COMPUTE, args.team, stream=stream)
    torch.cuda.synchronize()

    # clock ramp: the same kernel for --ramp-ms before the warm-up (a fresh box idles its clocks;
    # 5 warm-up launches of 0.25 ms do not ramp them)
    t_ramp = time.perf_counter()
    ramp_launches = 0
    if n:
        while (time.perf_counter() - t_ramp) * 1e3 < args.ramp_ms:
            for i in range(10):
                step(i)
            ramp_launches += 10
            torch.cuda.synchronize()
    ramp_ms = (time.perf_counter() - t_ramp) * 1e3
    for i in range(args.warmup):
        if n:
            step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the timed region: K launches back to back, HIP events on the kernel's stream at both ends
    # only (an event between launches serialises them: +2.5 us per 16-us C1 launch)
    t_beg, t_end = V.Event(), V.Event()
    t0 = time.perf_counter()
    t_beg.record(stream)
    for i in range(args.steps):
        if n:
            step(i)
    t_end.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    kernel_ms = t_beg.elapsed_ms(t_end) / args.steps
    # per-launch times (spread, warm-up drift) from a second pass of K launches, each between
    # its own events, after the timed region
    evs = [V.Event() for _ in range(args.steps + 1)]
    evs[0].record(stream)
    for i in range(args.steps):
        if n:
            step(i)
        evs[i + 1].record(stream)
    torch.cuda.synchronize()
    per_launch = [evs[i].elapsed_ms(evs[i + 1]) for i in range(args.steps)]
    # The same K steps with two batches in flight, through the library's pipe (vpcsum_pipe_*: the
    # launches alternate between the pipe's two streams, forked from the kernel's stream and joined
    # back into it; each batch with its own out words), so that one launch's ramp and drain overlap
    # its neighbour's -- the rate of a caller that keeps two batches in flight, as the host contexts
    # do with their two slots.  Reported next to `value`, not as it: the roofline prices a launch
    # alone, and overlapped launches have no duration of their own.
    peak_main = int(torch.cuda.max_memory_allocated())   # before the second batch below
    pipe_wall, pipe_bytes = 0.0, 0.0
    if not nat:
        if n:
            if nb >= 2:   # the rotation's batches, as in the timed region
                pb = [(arenas[b], ds[b], batch_bytes[b]) for b in range(nb)]
            else:   # a second batch (the next disjoint sub-stream), so that no two launches share one
                a2 = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
                d2 = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
                V.synth(a2, n, stride, 0, synth_id, SEED, first + world * n_cfg, d2, stream=stream)
                pb = [(arena, d, bytes_per_step), (a2, d2, algorithmic_bytes(V.tensor_to_desc(d2)[:n]))]
            pipe = V.Pipe(stream)
            out2 = torch.zeros_like(out)

            def step2(i):
                a, dd, _ = pb[i % len(pb)]
                pipe.compute(a, dd, n, (out, out2)[i % 2], None, V.MODE_COMPUTE, args.team)
            pipe.begin()
            for i in range(4):
                step2(i)
            pipe.join()
            pipe_bytes = float(sum(pb[i % len(pb)][2] for i in range(args.steps)))
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        if n:
            pipe.begin()
            for i in range(args.steps):
                step2(i)
            pipe.join()
        torch.cuda.synchronize()
        pipe_wall = max_over_ranks(time.perf_counter() - t0)
        pipe_bytes = sum_over_ranks(pipe_bytes)
        pb = a2 = d2 = None
        if n:
            pipe.close()
    wall_max = max_over_ranks(wall)
    # per-rank attribution of a multi-GPU line: every rank's kernel time and the card it ran on
    props = torch.cuda.get_device_properties(torch.cuda.current_device())
    dev_id = str(getattr(props, "uuid", "")) or f"{props.pci_domain_id}:{props.pci_bus_id}:{props.pci_device_id}"
    ranks_info = gather_over_ranks({"rank": rank, "device": torch.cuda.current_device(), "device_id": dev_id,
                                    "kernel_ms": round(t_beg.elapsed_ms(t_end) / args.steps, 5),
                                    "packets": int(n), "first_packet": int(first),
                                    "shard_arena_bytes": int(n) * stride,
                                    "peak_alloc_bytes": peak_main})
    # bytes of the K timed launches (the rotation's batches differ slightly in C3's mix)
    timed_bytes = sum(batch_bytes[i % nb] for i in range(args.steps)) if not nat else bytes_per_step * args.steps
    total_bytes_step = sum_over_ranks(float(timed_bytes)) / args.steps
    if not nat and n and nb > 1:   # `out` must hold batch 0 for the correctness gate
        V.compute(arena, d, n, out, None, V.MODE_COMPUTE, args.team, stream=stream)
        torch.cuda.synchronize()

    # measured read ceilings (context for the roofline fraction)
    sink = torch.zeros(8192, dtype=torch.int32, device="cuda")
    e0, e1 = V.Event(), V.Event()
    read_ceiling = read_bpc = pattern_ceiling = unit_order_ceiling = launch_read = None
    if not nat and n:
        # a reference, not a ceiling: a contiguous streaming read of the whole rotation's arena
        # (every byte, where K2 reads 1504 of every 2048), best of four grids
        span = arena_all[int(desc_np["l3_off"].min()) // 16 * 16:]   # every batch of the rotation
        cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
        best = None
        for bpc in (2, 4, 8, 16):
            for _ in range(3):
                V.read_probe(span, span.numel(), sink, cus * bpc, stream=stream)
            e0.record(stream)
            for _ in range(10):
                V.read_probe(span, span.numel(), sink, cus * bpc, stream=stream)
            e1.record(stream)
            r = span.numel() / (e0.elapsed_ms(e1) / 10 * 1e-3) / 1e9
            if best is None or r > best[0]:
                best = (r, bpc)
        read_ceiling, read_bpc = best
        if desc_np["l3_len"].mean() >= 512 and arena.numel() < (1 << 32):
            # a read-only kernel over exactly this batch's chunks (no checksum work), best of 2
            # and 4 workgroups per CU, plain and with software-pipelined trips (bit 30), in
            # algorithmic bytes like `achieved`
            pms = []
            for bpc in (2, 4):
                for pipe in (0, 1 << 30):
                    for _ in range(3):
                        V.pattern_probe(arena, d, n, sink, (cus * bpc) | pipe, stream=stream)
                    e0.record(stream)
                    for _ in range(10):
                        V.pattern_probe(arena, d, n, sink, (cus * bpc) | pipe, stream=stream)
                    e1.record(stream)
                    pms.append(e0.elapsed_ms(e1) / 10)
            pattern_ceiling = bytes_per_step / (min(pms) * 1e-3) / 1e9
            # the same reads in K2's packet order (a wave walks its own 64 consecutive packets,
            # grid-strided units): a reference order, not a ceiling (K2 beats it on C2 through its
            # rotated slot order; on C3 the order costs ~9% against the grid
            # order above, item 24)
            pus = []
            for bpc in (5, 12):
                for _ in range(3):
                    V.pattern_probe(arena, d, n, sink, (cus * bpc) | (1 << 31), stream=stream)
                e0.record(stream)
                for _ in range(10):
                    V.pattern_probe(arena, d, n, sink, (cus * bpc) | (1 << 31), stream=stream)
                e1.record(stream)
                pus.append(e0.elapsed_ms(e1) / 10)
            unit_order_ceiling = bytes_per_step / (min(pus) * 1e-3) / 1e9
        if nb > 2:
            # small-packet batches (C1): a batch is too small for a launch to reach the streaming
            # rate, so the kernel is also priced against a plain streaming read of the same number
            # of bytes per launch (one batch's frames + descriptors, contiguous), launched back to
            # back over the rotation's batches like the timed region; traffic bytes on both sides
            slab = n * stride + n * 16
            cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
            best = None
            for bpc in (4, 8, 16, 32):
                if cus * bpc > sink.numel():
                    continue
                for rep in range(2):
                    e0.record(stream)
                    for k in range(50):
                        b = k % (nb - 1)
                        V.read_probe(arena_all[b * n * stride:b * n * stride + slab], slab, sink, cus * bpc, stream=stream)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    t = e0.elapsed_ms(e1) / 50
                    if rep and (best is None or t < best[0]):
                        best = (t, bpc)
            if best is not None:
                launch_read = {"bytes_per_launch": slab, "ms_per_launch": round(best[0], 5),
                               "workgroups_per_cu": best[1], "GBps": round(slab / (best[0] * 1e-3) / 1e9, 1)}
    elif nat and n:
        # NAT's own memory operations with no rewrite (vpcsum_nat4_pattern_probe_async: descriptor
        # and entry reads, the header window loads, the one store of [L3+10, checksum end)),
        # priced in the same 72 algorithmic B/packet as `achieved`; --preimage: the pre-image
        # kernel's probe build (vpcsum_pre_async bit 23: the same loads and 4-B stores, the stored
        # sums written back unchanged), at 76 B/packet
        def probe():
            if pre:
                V.pre(arena, d, pre_img, n, None, None, V.MODE_WRITE | 0x800000, V.PRE_FMT_PRE4, stream=stream)
            else:
                V.nat4_pattern_probe(arena, d, rw, n, stream=stream)
        for _ in range(3):
            probe()
        e0.record(stream)
        for _ in range(10):
            probe()
        e1.record(stream)
        pattern_ceiling = bytes_per_step / (e0.elapsed_ms(e1) / 10 * 1e-3) / 1e9

    # correctness: (1) rank 0 against the oracle on the cpu_baseline's packets (2) every rank:
    # sums written in place, then verified on the GPU
    # every line carries the CPU baseline, N > 1 included: rank 0 times it after the timed region
    # (the other ranks wait at the next collective), on rank 0's first packets
    cpu, gate = None, {}
    if pre and n:
        # the timed flushes applied the pre-images again and again: every rank's gate takes a fresh
        # batch through one flush (then the descriptors lose F_PRE, for the verify below)
        V.synth(arena, n, stride, 0, synth_id, SEED, first, d, stream=stream)
        V.compute(arena, d, n, None, None, V.MODE_WRITE, stream=stream)
        pre_img = prep_pre()
        V.pre(arena, d, pre_img, n, None, None, V.MODE_WRITE, V.PRE_FMT_PRE4, stream=stream)
        torch.cuda.synchronize()
        d.view(n, 16)[:, 14] &= 0xFF ^ V.F_PRE
    if rank == 0 and not args.no_cpu_baseline and not nat and n:
        cpu, (m, want_out, want_st) = cpu_baseline(args.workload, synth_id, stride, first, args.cpu_budget)
        m = min(m, n)
        got = out[:m].cpu().numpy().view(np.uint32)
        gate["oracle_packets"] = int(m)
        gate["oracle_equal"] = bool(np.array_equal(got, want_out[:m]))
    elif rank == 0 and not args.no_cpu_baseline and nat and n:
        cpu, (m, a0, d0, want) = cpu_baseline_nat(rw_np, args.cpu_budget)   # rank 0: first == 0
        got = arena[:m * stride].cpu().numpy()
        gate["oracle_packets"] = int(m)
        gate["oracle_equal"] = bool(np.array_equal(got, want))
    if not nat and n:
        gate.update(oracle_sample_gate(synth_id, stride, first, out[:n].cpu().numpy().view(np.uint32)))
    if nat:
        ok = True
        if n:
            V.compute(arena, d, n, None, status, V.MODE_VERIFY, stream=stream)
            torch.cuda.synchronize()
            st = status[:n].cpu().numpy()
            v4 = desc_np["l3_ver"] == 4
            ok = bool(np.all((st[v4] & 3) == 3))
    else:
        ok = True
        if n:
            V.compute(arena, d, n, out, status, V.MODE_WRITE, args.team, stream=stream)
            V.compute(arena, d, n, None, status, V.MODE_VERIFY, args.team, stream=stream)
            torch.cuda.synchronize()
            st = status[:n].cpu().numpy()
            want_ok = np.where(desc_np["flags"] & 1, 1, 0) | np.where(desc_np["flags"] & 2, 2, 0)
            ok = bool(np.all((st & 3) == want_ok))
    ok = ok and gate.get("oracle_equal", True) and gate.get("sample_equal", True)
    all_ok = all_ranks_ok(ok)

    achieved = timed_bytes / args.steps / (kernel_ms * 1e-3) / 1e9 if n else 0.0
    # C5's summary: the 10M-packet pass with the bench's rewrite mask (src|dst|ports = 15)
    traffic, traffic_src = pmc_traffic(("pre15" if pre else "nat15") if nat else args.workload, n) \
        if args.team == 0 else (None, None)
    traffic_src = traffic_src or {}
    if rank == 0:
        value = total_bytes_step * args.steps / wall_max / 1e9
        kname = ("k_pre (RFC 1624 from pre-images)" if pre else "k_natq (RFC 1624)") if nat else "k_csum_d (K2)"
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": desc_text + (" (one global batch, byte-balanced shards)" if strong else " per GPU"),
                "global_batch": n_cfg if strong else n_cfg * world,
                "source_hash": source_hash(),
                "packets_rank0": n,
                "algorithmic_bytes_per_step_rank0": bytes_per_step,
                "algorithmic_bytes_per_step_all_ranks": int(total_bytes_step),
                "parallelism": f"shard-per-GPU x{world} (independent streams, no collective)",
                "verify_all_packets": all_ok,
                "oracle_gate": gate or None,
                "batches_rotated": nb,
                "ramp_ms": round(ramp_ms, 1),
                "ramp_launches": ramp_launches,
                "per_launch_ms_rank0": launch_stats(per_launch) if n else None,
                "devices_distinct": len({r["device_id"] for r in ranks_info}),
                "shared_gpu_rehearsal": len({r["device_id"] for r in ranks_info}) < world,
                "kernel_ms_over_ranks": {"min": min(r["kernel_ms"] for r in ranks_info),
                                         "max": max(r["kernel_ms"] for r in ranks_info)},
                "ranks": ranks_info if world > 1 else None,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kname,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "traffic_unit": "HBM bytes per launch (rocprofv3 PMC, corrected)",
                "traffic_source": traffic_src.get("source"),
                # the tree the PMC summary was measured on; stale: no summary of this tree's sources
                "traffic_head": traffic_src.get("head"),
                "traffic_stale": traffic_src.get("stale"),
                "algorithmic_bytes_per_launch": bytes_per_step,
                "kernel_avg_ms": round(kernel_ms, 5),
                # references (not bounds): a contiguous read of the whole span, and K2's reads in
                # its own unit order without the rotation
                "contiguous_read_GBps": round(read_ceiling, 1) if read_ceiling else None,
                "contiguous_read_workgroups_per_cu": read_bpc,
                "measured_pattern_ceiling_GBps": round(pattern_ceiling, 1) if pattern_ceiling else None,
                "frac_of_pattern_ceiling": round(achieved / pattern_ceiling, 4) if pattern_ceiling else None,
                "reference_order_probe_GBps": round(unit_order_ceiling, 1) if unit_order_ceiling else None,
                "frac_of_reference_order_probe": round(achieved / unit_order_ceiling, 4) if unit_order_ceiling else None,
                "pattern_ceiling_kernel": ("k_pre probe (same loads and stores, no arithmetic)" if pre else
                                           "k_natq probe (same loads and stores, no rewrite)" if nat else
                                           "k_pattern_probe (K2's chunk reads, no checksum work)")
                if pattern_ceiling else None,
                "traffic_over_algorithmic": round(traffic / bytes_per_step, 3) if traffic and bytes_per_step else None,
                # small-packet batches: the same bytes per launch as one contiguous streaming read
                "launch_read_ceiling": launch_read,
                "frac_of_launch_read_ceiling": round(traffic / (kernel_ms * 1e-3) / 1e9 / launch_read["GBps"], 4)
                if launch_read and traffic else None,
            },
            "cpu_baseline": cpu,
        }
        if not nat and pipe_wall > 0:
            pv = pipe_bytes / pipe_wall / 1e9
            line["pipelined_two_streams"] = {"value": round(pv, 2), "unit": "GB/s",
                                             "ms_per_step": round(pipe_wall / args.steps * 1e3, 5),
                                             "over_value": round(pv / value, 4),
                                             "api": "vpcsum_pipe_begin / vpcsum_pipe_compute_async / vpcsum_pipe_join",
                                             "what": "the same K steps with two batches in flight through the "
                                                     "library's pipe; not `value`: the roofline prices one launch alone"}
        if nat:
            line["config"]["Mpps_rank0"] = round(n / kernel_ms / 1e3, 1) if n else 0
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not all_ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
