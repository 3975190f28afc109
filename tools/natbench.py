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
