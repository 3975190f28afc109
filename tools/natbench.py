"""NAT / TTL rewrite throughput (BASELINE config C5 per GPU), RFC 1624 and strict-Java modes."""
import json, os, sys, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vproxy_amd import vpcsum as V  # noqa: E402
n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 10_000_000 // 8
stride = 2048
arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
V.synth(arena, n, stride, 0, V.SYNTH_C5, 0x20241020, 0, d)
# C5: 1500 B IPv4 TCP/UDP (50/50) with valid input checksums, every packet rewritten
V.compute(arena, d, n, None, None, V.MODE_WRITE)
g = torch.Generator(device="cpu").manual_seed(5)
rw = torch.randint(0, 256, (n, 16), dtype=torch.uint8, generator=g)
rw[:, 12] = V.NAT_SRC | V.NAT_DST | V.NAT_SPORT | V.NAT_DPORT
rw[:, 13:] = 0
rw = rw.cuda()
st = torch.zeros(n, dtype=torch.uint8, device="cuda")
res = {"packets": n}
modes = [("rfc1624", V.NAT_RFC1624), ("strict_java", V.NAT_STRICT_JAVA),
         ("rfc1624_bytewise", V.NAT_RFC1624 | 0x100), ("strict_java_bytewise", V.NAT_STRICT_JAVA | 0x100)]
if "--sweep" in sys.argv:   # packets per lane of the wide kernel (nat_mode bits 12..14)
    modes += [(f"rfc1624_w{1 << k}", V.NAT_RFC1624 | ((k + 1) << 12)) for k in range(3)]
if "--probe" in sys.argv:   # the pattern ceiling and the bench's form (no status), interleaved rounds
    for rnd in range(3):
        for name, fn in (("probe", lambda: V.nat4_pattern_probe(arena, d, rw, n)),
                         ("rfc1624_nostatus", lambda: V.nat4(arena, d, rw, n, None, V.NAT_RFC1624))):
            for _ in range(3):
                fn()
            e0, e1 = V.Event(), V.Event()
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_ms(e1) / 10
            res.setdefault(name, []).append({"ms": round(ms, 4), "Mpps": round(n / ms / 1e3, 1)})
for name, mode in modes:
    for _ in range(3):
        V.nat4(arena, d, rw, n, st, mode)
    e0, e1 = V.Event(), V.Event()
    e0.record()
    it = 10
    for _ in range(it):
        V.nat4(arena, d, rw, n, st, mode)
    e1.record()
    ms = e0.elapsed_ms(e1) / it
    res[name] = {"ms": round(ms, 4), "Mpps": round(n / ms / 1e3, 1), "GBps_at_72B": round(n * 72 / ms / 1e6, 1)}

if "--v6" in sys.argv:
    # 48-B entries (vpcsum_nat_async): the same IPv4 batch, and 1M IPv6/TCP packets of 9000 B (C4
    # frames) with 16-B addresses and ports rewritten, RFC 1624
    def timed48(ar, dd, rw48, m, mode):
        s_ = torch.zeros(m, dtype=torch.uint8, device="cuda")
        for _ in range(3):
            V.nat(ar, dd, rw48, m, s_, mode)
        e0, e1 = V.Event(), V.Event()
        e0.record()
        for _ in range(10):
            V.nat(ar, dd, rw48, m, s_, mode)
        e1.record()
        torch.cuda.synchronize()
        ms_ = e0.elapsed_ms(e1) / 10
        assert int((s_ & V.S_BAD_DESC).sum().item()) == 0
        return {"ms": round(ms_, 4), "Mpps": round(m / ms_ / 1e3, 1)}

    def entries48(m, seed):
        g_ = torch.Generator(device="cpu").manual_seed(seed)
        r48 = torch.zeros((m, 48), dtype=torch.uint8)
        r48[:, :36] = torch.randint(0, 256, (m, 36), dtype=torch.uint8, generator=g_)
        r48[:, 36] = V.NAT_SRC | V.NAT_DST | V.NAT_SPORT | V.NAT_DPORT
        return r48.cuda()

    res["v4_48B_entries_rfc1624"] = timed48(arena, d, entries48(n, 6), n, V.NAT_RFC1624)
    del arena
    torch.cuda.empty_cache()
    n6, s6 = 1 << 20, 9216
    a6 = torch.zeros(n6 * s6, dtype=torch.uint8, device="cuda")
    d6 = torch.zeros(n6 * 16, dtype=torch.uint8, device="cuda")
    V.synth(a6, n6, s6, 0, V.SYNTH_C4, 0x20241020, 0, d6)
    V.compute(a6, d6, n6, None, None, V.MODE_WRITE)
    res["v6_c4_frames"] = {"packets": n6, "rfc1624": timed48(a6, d6, entries48(n6, 7), n6, V.NAT_RFC1624)}
    print(json.dumps(res))
    sys.exit(0)

if "--no-cpu" not in sys.argv:
    # CPU baseline (BASELINE C5): the oracle's Java-semantics rewrite (setters + full recompute,
    # SwitchUtils.java:522-542) on a bounded sample of the same workload, 1 and 16 threads
    from oracle import oracle as O  # noqa: E402
    orc = O.Oracle()
    m = 1 << 18
    a_np, d_np = orc.synth(m, stride, 0, O.SYNTH_C5, O.SEED, 0)
    orc.process(a_np, d_np, write=True)
    rw_np = rw[:m].cpu().numpy()
    cpu = {"packets": m, "kind": "port"}
    for th in (1, 16):
        a = a_np.copy()
        t = time.perf_counter()
        orc.nat4_java(a, d_np, rw_np, threads=th)
        dt = time.perf_counter() - t
        cpu[f"strict_java_{th}t_Mpps"] = round(m / dt / 1e6, 2)
    # the GPU's strict-Java result on the same packets must equal the oracle's
    g = torch.from_numpy(a_np.copy()).cuda()
    gd = torch.from_numpy(d_np.view(np.uint8).copy()).cuda()
    gst = torch.zeros(m, dtype=torch.uint8, device="cuda")
    V.nat4(g, gd, rw[:m].contiguous(), m, gst, V.NAT_STRICT_JAVA)
    cpu["gpu_equal"] = bool(np.array_equal(g.cpu().numpy(), a))
    res["cpu_baseline"] = cpu
print(json.dumps(res))
