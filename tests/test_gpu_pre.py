"""GPU parity of the pre-image egress flush (VPCSUM_F_PRE, VERDICT r4 "Next round" items 1 and 6).

A NAT'd frame reaches the egress flush with Java's setters already applied -- new addresses and
ports in the frame, the stored sums stale (SwitchUtils.applyNat, SwitchUtils.java:531-542; e.g.
Ipv4Packet.setSrc writes raw.pktBuf, :433-445) -- and the pre-image the vswitch recorded just
before them (vproxy_amd/vswitch.py:record_pre_image).  The GPU updates the L4 sum by RFC 1624 from
the pre-image and the stored field, and recomputes the IPv4 header sum in full.  The oracle's
answer is Java's: the setters followed by a full recompute of the dirtied sums (getRawPacket(0),
AbstractPacket.java:15-22, 58-65; oracle/csum_oracle.c:orc_nat_java).  They must be byte-equal
whenever the stored L4 sum was correct before the rewrite -- what ingress verify's S_L4_OK proves,
the seam's condition for F_PRE (vswitch.pre_eligible); frames without it take the full recompute.
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAT_FIELDS = O.NAT_SRC | O.NAT_DST | O.NAT_SPORT | O.NAT_DPORT


@pytest.fixture(scope="module")
def V():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vproxy_amd import vpcsum
    vpcsum.lib()
    return vpcsum


def dev(a):
    """A pageable host-to-device copy (torch's plain `.cuda()`), the path round 5's two intermittent
    faults hit; round 6 restores it here (DESIGN_HISTORY.md "Round 6: the intermittent fault")."""
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()


def pre_images(arena, desc, rw):
    """The vswitch's pre-images (old values of the fields each entry rewrites), recorded from the
    frames before the setters run."""
    from vproxy_amd import vswitch as S
    pre = np.zeros(len(desc), O.NAT_DTYPE)
    for i, d in enumerate(desc):
        pre[i] = S.record_pre_image(arena, int(d["l3_off"]), int(d["l3_ver"]), int(d["l4_off"]), int(d["l4_proto"]),
                                    int(rw[i]["mask"]) & NAT_FIELDS)
    return pre


def nat4_of(rw48):
    r4 = np.zeros(len(rw48), O.NAT4_DTYPE)
    r4["src"], r4["dst"] = rw48["src"][:, :4], rw48["dst"][:, :4]
    r4["sport"], r4["dport"], r4["mask"] = rw48["sport"], rw48["dport"], rw48["mask"]
    return r4


def java_dirty_flags(desc, rw):
    """F_IP / F_L4 as Java's setters leave a packet (checksumSkipped): IPv4 addresses and the TTL
    dirty the header (Ipv4Packet.java:401-458); addresses dirty the L4 sum through the pseudo header
    of TCP / UDP, and of ICMP / ICMPv6 under IPv6 (pseudoHeaderChanges, Ipv4Packet.java:236-240,
    Ipv6Packet.java:238-242); ports dirty TCP / UDP; an L4 packet without its checksum field in the
    segment is never dirty.  The egress defers exactly these (SwitchUtils.checksumFlagsFor)."""
    v4 = desc["l3_ver"] == 4
    proto = desc["l4_proto"].astype(int)
    fld = np.array([O.L4_FIELD.get(int(p), -1) for p in proto])
    l4sum = (fld >= 0) & ~(v4 & (proto == 58)) & \
        (desc["l3_len"].astype(int) - desc["l4_off"].astype(int) >= fld + 2)
    m = rw["mask"].astype(int)
    tcpudp = (proto == 6) | (proto == 17)
    addr_dirty = l4sum & (tcpudp | (~v4 & ((proto == 1) | (proto == 58))))
    ip = v4 & ((m & (O.NAT_SRC | O.NAT_DST | O.NAT_SET_TTL | O.NAT_DEC_TTL)) != 0)
    l4 = (((m & (O.NAT_SRC | O.NAT_DST)) != 0) & addr_dirty) | (l4sum & tcpudp & ((m & (O.NAT_SPORT | O.NAT_DPORT)) != 0))
    return (np.where(ip, O.F_IP, 0) | np.where(l4, O.F_L4, 0)).astype(np.uint8)


def assert_frames(got, want, desc, what="", whole=True):
    """Byte equality (whole: of the arrays; else of desc's packets), naming the first packet that
    differs."""
    if whole and np.array_equal(got, want):
        return
    for i, d in enumerate(desc):
        o, L = int(d["l3_off"]), int(d["l3_len"])
        if not np.array_equal(got[o:o + L], want[o:o + L]):
            diff = np.nonzero(got[o:o + L] != want[o:o + L])[0]
            raise AssertionError(f"{what} packet {i}: ver {d['l3_ver']} proto {d['l4_proto']} flags "
                                 f"{d['flags']:#x} l4_off {d['l4_off']} len {L}: bytes {diff[:8].tolist()} "
                                 f"got {got[o + diff[:4]].tolist()} want {want[o + diff[:4]].tolist()}")
    if whole:
        raise AssertionError(f"{what}: bytes outside the packets differ")


def nat_case(orc, rng, n, workload, pad=0, stride=9088, udp_zero=0.1, mask=None):
    """Frames with valid sums (10% UDP stored 0), random 48-B rewrites (every NAT / TTL bit unless
    `mask`), the pre-images, the frames after Java's setters and Java's final bytes.  Returns
    (after_setters, desc, pre, want, java_status): each descriptor carries the sums Java left dirty
    plus F_PRE; packets with none, and those the setters refused (TTL expired: IPInputRoute drops
    them), carry no flags."""
    arena, desc = orc.synth(n, stride, pad, workload, O.SEED, int(rng.integers(0, 1 << 30)))
    orc.process(arena, desc, O.MODE_COMPUTE, write=True)
    for d in desc:
        if d["l4_proto"] == 17 and rng.random() < udp_zero:
            o = int(d["l3_off"]) + int(d["l4_off"])
            arena[o + 6:o + 8] = 0
    rw = np.zeros(n, O.NAT_DTYPE)
    rw.view(np.uint8).reshape(n, 48)[:, :38] = rng.integers(0, 256, (n, 38), dtype=np.uint8)
    rw["mask"] = rng.integers(0, 64, n) if mask is None else mask
    pre = pre_images(arena, desc, rw)
    want = arena.copy()
    wst = orc.nat_java(want, desc, rw)
    after = arena.copy()
    sst = orc.nat_setters(after, desc, rw)
    assert np.array_equal(sst, wst)
    d = desc.copy()
    dirty = java_dirty_flags(desc, rw)
    d["flags"] = np.where(dirty != 0, dirty | O.F_PRE, 0)
    d["flags"][wst != O.S_DONE] = 0
    return after, d, pre, want, wst


def gpu_pre(V, after, desc, pre, mode, fmt):
    import torch
    a = dev(after)
    n = len(desc)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    V.pre(a, dev(desc), dev(pre), n, out, st, mode, pre_fmt=fmt)
    torch.cuda.synchronize()
    return a.cpu().numpy(), out.cpu().numpy().view(np.uint32), st.cpu().numpy()


def expected_out(orc, want, desc):
    """Out words of the F_PRE packets: the sums Java's recompute leaves in the frames."""
    d = desc.copy()
    d["flags"] &= O.F_IP | O.F_L4
    out, _ = orc.process(want, d)
    return out


@pytest.mark.parametrize("pad", [0, 1, 2, 14])
@pytest.mark.parametrize("tune", [0, 0x100, 0x2000, 3 << 18])
def test_pre_v4_v6_equals_java(V, orc, pad, tune):
    """48-B pre-images (IPv4 with options, IPv6; TCP / UDP / ICMP / ICMPv6; every rewrite mask,
    TTL bits included; 10% UDP stored 0): the frames after the flush equal Java's setters + full
    recompute byte for byte, on the LDS-window path, the byte path (bit 8), two packets per lane
    (bits 12..13) and a 3-workgroup-per-CU grid (bits 18..22)."""
    rng = np.random.default_rng(300 + pad)
    after, desc, pre, want, wst = nat_case(orc, rng, 1500, O.SYNTH_FUZZ, pad)
    got, out, st = gpu_pre(V, after, desc, pre, O.MODE_WRITE | tune, 1)
    assert_frames(got, want, desc, f"pad {pad} tune {tune:#x}")
    live = desc["flags"] != 0
    assert np.all(st[live] == O.S_DONE) and np.all(st[~live] == 0xEE)   # flags 0: not the kernel's
    assert np.array_equal(out[live], expected_out(orc, want, desc)[live])
    # compute mode: the same words, the frames untouched
    got, out2, _ = gpu_pre(V, after, desc, pre, O.MODE_COMPUTE | tune, 1)
    assert np.array_equal(got, after) and np.array_equal(out2[live], out[live])


@pytest.mark.parametrize("workload", [O.SYNTH_C1, O.SYNTH_C3, O.SYNTH_C5])
@pytest.mark.parametrize("tune", [0, 0x100, 0x2000, 0x20000, 0x22000, 0x1000000])
def test_pre4_ipv4_equals_java(V, orc, workload, tune):
    """16-B pre-images (vpcsum_pre4_t) on IPv4 batches, 4- and 6-chunk windows, 1 or 2 packets per
    lane: byte-equal to Java; IPv6 descriptors are refused untouched."""
    rng = np.random.default_rng(400 + workload)
    after, desc, pre, want, wst = nat_case(orc, rng, 3000, workload, pad=14, stride=2048)
    got, out, st = gpu_pre(V, after, desc, nat4_of(pre), O.MODE_WRITE | tune, 0)
    assert_frames(got, want, desc, f"workload {workload} tune {tune:#x}")
    live = desc["flags"] != 0
    assert np.all(st[live] == O.S_DONE)
    assert np.array_equal(out[live], expected_out(orc, want, desc)[live])
    a6, d6, p6, w6, s6 = nat_case(orc, rng, 200, O.SYNTH_FUZZ)
    got, _, st = gpu_pre(V, a6, d6, nat4_of(p6), O.MODE_WRITE | tune, 0)
    v6 = (d6["l3_ver"] == 6) & (d6["flags"] != 0)
    assert np.all(st[v6] == O.S_BAD_DESC)
    for i in np.nonzero(v6)[0]:
        o = int(d6[i]["l3_off"])
        assert np.array_equal(got[o:o + int(d6[i]["l3_len"])], a6[o:o + int(d6[i]["l3_len"])])


def test_pre_nat_golden(V, orc):
    """The reference's own checkPartialAndModify rewrites on the TestPacket frames (setSrc / setDst
    1.2.3.4 and ::2, setSrcPort / setDstPort 121, setTtl / setHopLimit 5; tests/golden/nat.json):
    setters applied to the frame, the pre-image of the fields they changed, the flush -> the
    reference's bytes."""
    import torch
    from vproxy_amd import vswitch as S
    d = json.load(open(os.path.join(GOLD, "nat.json")))
    done = 0
    for c in d["cases"]:
        fr = bytes.fromhex(c["before"])
        info, _ = O.parse_l3(fr, c["l3_off"], len(fr) - c["l3_off"])
        rw = np.frombuffer(bytes.fromhex(c["entry"]), O.NAT_DTYPE).copy()
        if rw[0]["mask"] & O.NAT_DEC_TTL and (fr[c["l3_off"] + (8 if info.ver == 4 else 7)] <= 1):
            continue
        desc = np.array([(info.l3_off, info.l3_len, info.l4_off, info.ver, info.proto, 0, 0)], dtype=O.DESC_DTYPE)
        dirty = int(java_dirty_flags(desc, rw)[0])
        if not dirty:
            continue
        desc["flags"] = dirty | O.F_PRE
        a = np.frombuffer(fr, np.uint8).copy()
        pre = np.zeros(1, O.NAT_DTYPE)
        pre[0] = S.record_pre_image(a, info.l3_off, info.ver, info.l4_off, info.proto, int(rw[0]["mask"]) & NAT_FIELDS)
        orc.nat_setters(a, desc, rw)
        for tune in (0, 0x100):
            got, _, st = gpu_pre(V, a, desc, pre, O.MODE_WRITE | tune, 1)
            assert st[0] == O.S_DONE
            assert got.tobytes().hex() == c["after"], (c["kat"], c["rewrite"], tune)
        done += 1
    torch.cuda.synchronize()
    assert done >= 10


def test_pre_edge_packets(V, orc):
    """The crafted edge packets (IPv6 extension headers with odd l4_off: the byte path beyond the
    window; ICMPv4 inside IPv6: no pseudo header; sums of 0; UDP stored 0) under random rewrites."""
    import edgevec as E
    pk = [p for p in E.edge_packets(np.random.default_rng(7)) if p["l3_len"] <= 9000]
    for pad in (0, 3):
        arena, desc = E.pack(pk, pad)
        rng = np.random.default_rng(pad + 40)
        rw = np.zeros(len(desc), O.NAT_DTYPE)
        rw.view(np.uint8).reshape(-1, 48)[:, :38] = rng.integers(0, 256, (len(desc), 38), dtype=np.uint8)
        rw["mask"] = rng.integers(1, 64, len(desc))
        # edge packets carry arbitrary flags: the egress asks for the sums Java left dirty
        desc = desc.copy()
        pre = pre_images(arena, desc, rw)
        want = arena.copy()
        wst = orc.nat_java(want, desc, rw)
        after = arena.copy()
        orc.nat_setters(after, desc, rw)
        dirty = java_dirty_flags(desc, rw)
        ok = (wst == O.S_DONE) & (dirty != 0)
        desc["flags"] = np.where(ok, dirty | O.F_PRE, 0)
        got, _, st = gpu_pre(V, after, desc, pre, O.MODE_WRITE, 1)
        assert np.all(st[ok] == O.S_DONE)
        for i in np.nonzero(ok)[0]:
            o, L = int(desc[i]["l3_off"]), int(desc[i]["l3_len"])
            assert np.array_equal(got[o:o + L], want[o:o + L]), (pad, pk[i]["kind"])


@pytest.mark.parametrize("team", [0, 12, 40, 46, 70, 72, 74, 76, 78, 79, 84])
@pytest.mark.parametrize("mode", [O.MODE_COMPUTE, O.MODE_VERIFY, O.MODE_WRITE])
def test_compute_leaves_pre_descriptors_alone(V, orc, team, mode):
    """vpcsum_compute_async on a batch whose every other descriptor has F_PRE: the others equal
    the oracle, the F_PRE ones get out 0 / S_DONE and their frames are not written, on every
    checksum kernel (K2 builds, the team kernel, the zero-copy wave kernel)."""
    import torch
    arena, desc = orc.synth(2000, 2048, 14, O.SYNTH_C3, O.SEED, 77)
    if mode != O.MODE_COMPUTE:
        orc.process(arena, desc, O.MODE_COMPUTE, write=True)
        arena[2048 + 14 + 40::4096] ^= 0x33     # some stored sums wrong (odd frames: not F_PRE)
    d = desc.copy()
    d["flags"][::2] |= O.F_PRE
    want, want_st = orc.process(arena, np.ascontiguousarray(desc[1::2]), mode & O.MODE_VERIFY)
    a = dev(arena)
    out = torch.full((len(d),), -1, dtype=torch.int32, device="cuda")
    st = torch.zeros(len(d), dtype=torch.uint8, device="cuda")
    V.compute(a, dev(d), len(d), out, st, mode, team)
    torch.cuda.synchronize()
    got, gst, ga = out.cpu().numpy().view(np.uint32), st.cpu().numpy(), a.cpu().numpy()
    assert np.all(got[::2] == 0) and np.all(gst[::2] == O.S_DONE)
    assert np.array_equal(got[1::2], want) and np.array_equal(gst[1::2], want_st)
    for i in range(0, len(d), 2):
        o, L = int(d[i]["l3_off"]), int(d[i]["l3_len"])
        assert np.array_equal(ga[o:o + L], arena[o:o + L]), i


def test_mixed_batch_compute_then_pre(V, orc):
    """One egress batch on the device: NAT'd frames with pre-images (F_PRE) between frames summed in
    full, and NAT'd frames whose stored sums were wrong before the rewrite (no F_PRE: full
    recompute).  vpcsum_compute_async then vpcsum_pre_async on the same stream: every frame equals
    Java's bytes."""
    import torch
    rng = np.random.default_rng(9)
    after, desc, pre, want, wst = nat_case(orc, rng, 4000, O.SYNTH_C3, pad=14, stride=2048)
    full = rng.random(len(desc)) < 0.4
    desc["flags"][full] &= 0xFF ^ O.F_PRE
    # the full-recompute frames may carry anything in their dirty sum fields: Java overwrites them
    for i in np.nonzero(full)[0]:
        o, l4 = int(desc[i]["l3_off"]), int(desc[i]["l4_off"])
        if desc[i]["flags"] & O.F_IP:
            after[o + 10:o + 12] = rng.integers(0, 256, 2, dtype=np.uint8)
        if desc[i]["flags"] & O.F_L4:
            f = o + l4 + O.L4_FIELD[int(desc[i]["l4_proto"])]
            after[f:f + 2] = rng.integers(0, 256, 2, dtype=np.uint8)
    a, d, p = dev(after), dev(desc), dev(nat4_of(pre))
    n = len(desc)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    V.compute(a, d, n, out, st, O.MODE_WRITE)
    V.pre(a, d, p, n, out, st, O.MODE_WRITE, pre_fmt=0)
    torch.cuda.synchronize()
    assert_frames(a.cpu().numpy(), want, desc)
    assert np.all(st.cpu().numpy() == O.S_DONE)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), expected_out(orc, want, desc))


def test_pre_on_invalid_input_diverges(V, orc):
    """Why the seam gates F_PRE on ingress verify: with a stored L4 sum that was wrong before the
    rewrite, RFC 1624 carries the error along and differs from Java's full recompute exactly in
    those frames (the pre-image path is exact only on valid input, like VPCSUM_NAT_RFC1624)."""
    rng = np.random.default_rng(12)
    after, desc, pre, want, wst = nat_case(orc, rng, 1000, O.SYNTH_C5, stride=2048, udp_zero=0.0, mask=NAT_FIELDS)
    bad = rng.random(len(desc)) < 0.3
    for i in np.nonzero(bad)[0]:
        o = int(desc[i]["l3_off"])
        after[o + 700] ^= 0x5A       # the payload changed after the sum was taken: invalid input
        want[o + 700] ^= 0x5A
    want2 = want.copy()
    d = desc.copy()
    d["flags"] &= O.F_IP | O.F_L4
    orc.process(want2, d, O.MODE_COMPUTE, write=True)   # Java: full recompute of the new bytes
    got, _, _ = gpu_pre(V, after, desc, pre, O.MODE_WRITE, 1)
    for i in range(len(desc)):
        o, L = int(desc[i]["l3_off"]), int(desc[i]["l3_len"])
        same = np.array_equal(got[o:o + L], want2[o:o + L])
        assert same != bool(bad[i]), i


@pytest.mark.parametrize("registered", [False, True])
def test_ctx_submit_pre(V, orc, registered):
    """vpcsum_ctx_submit_pre on host frames, staged (pageable: an F_PRE packet's header is all that
    is copied; its whole segment for a UDP stored 0) and zero-copy (registered: in place), 48-B and
    16-B entries, mixed with full-recompute descriptors and rejected ones."""
    rng = np.random.default_rng(20 + registered)
    after, desc, pre, want, wst = nat_case(orc, rng, 1200, O.SYNTH_FUZZ, pad=14)
    full = rng.random(len(desc)) < 0.3
    desc["flags"][full] &= 0xFF ^ O.F_PRE
    desc["l3_ver"][5::97] = 5                                # rejected by both kernels
    live = (desc["l3_ver"] != 5) & (desc["flags"] != 0)
    arena = np.concatenate([after, np.zeros(4096, np.uint8)])
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=len(desc))
    if registered:
        ctx.register(arena)
    base = arena.copy()
    for entries in (pre, None):
        if entries is None:   # 16-B entries: IPv4 only, so the IPv6 ones go the full path
            v6 = desc["l3_ver"] == 6
            d2 = desc.copy()
            d2["flags"][v6] &= 0xFF ^ O.F_PRE
            entries, dd = nat4_of(pre), d2
        else:
            dd = desc
        arena[:] = base
        out, st = ctx.run_pre(arena, dd, entries, O.MODE_WRITE)
        assert_frames(arena[:len(want)], want, dd[live], f"registered {registered}", whole=False)
        assert np.all(st[live] == O.S_DONE) and np.all(st[desc["l3_ver"] == 5] == O.S_BAD_DESC)
        assert np.array_equal(out[live], expected_out(orc, want, dd)[live])
    with pytest.raises(V.VpcsumError, match="bad mode"):
        ctx.run_pre(arena, desc, pre, O.MODE_VERIFY)
    ctx.close()


@pytest.mark.parametrize("idle_us", [5000, 40])
def test_service_submit_pre(V, orc, idle_us):
    """Small zero-copy flushes of NAT'd frames through the service grid (vpcsum_ctx_submit_pre with
    vpcsum_ctx_set_service: kernels.hip svc_pre_packet, one wave per frame), consecutive batches of
    1..512 frames mixing F_PRE frames (48-B and 16-B pre-images, UDP stored 0), full-recompute
    frames and refused descriptors, in WRITE and COMPUTE mode: the umem equals Java's bytes.  With
    idle_us = 40 the grid leaves between most flushes and is relaunched (a batch it left unfinished
    is re-run from the stored sums the host captured, never from the fields already rewritten)."""
    import time
    rng = np.random.default_rng(50 + idle_us)
    after, desc, pre, want, wst = nat_case(orc, rng, 1500, O.SYNTH_FUZZ, pad=14)
    full = rng.random(len(desc)) < 0.3
    desc["flags"][full] &= 0xFF ^ O.F_PRE
    desc["l3_ver"][7::101] = 5                               # refused by both paths
    live = (desc["l3_ver"] != 5) & (desc["flags"] != 0)
    d4 = desc.copy()                                         # 16-B entries: IPv4 only
    d4["flags"][d4["l3_ver"] == 6] &= 0xFF ^ O.F_PRE
    p4 = nat4_of(pre)
    exp48, exp4 = expected_out(orc, want, desc), expected_out(orc, want, d4)
    arena = np.concatenate([after, np.zeros(4096, np.uint8)])
    base = arena.copy()
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=len(desc))
    ctx.register(arena)
    ctx.set_service(idle_us)
    iters = 60
    for it in range(iters):
        b = int(rng.choice([1, 2, 3, 4, 5, 32, 128, 512]))
        lo = int(rng.integers(0, len(desc) - b + 1))
        sl = slice(lo, lo + b)
        fmt48 = it % 2 == 0
        dd, pp, exp = (desc, pre, exp48) if fmt48 else (d4, p4, exp4)
        mode = O.MODE_WRITE if it % 3 else O.MODE_COMPUTE
        arena[:] = base
        out = np.zeros(b, np.uint32)
        st = np.zeros(b, np.uint8)
        ctx.wait(ctx.submit_pre(arena, np.ascontiguousarray(dd[sl]), np.ascontiguousarray(pp[sl]), out, st, mode))
        lv = live[sl]
        what = f"it {it} n {b} fmt48 {fmt48} mode {mode}"
        assert np.all(st[lv] == O.S_DONE) and np.all(st[desc["l3_ver"][sl] == 5] == O.S_BAD_DESC), what
        assert np.array_equal(out[lv], exp[sl][lv]), what
        if mode == O.MODE_WRITE:
            assert_frames(arena[:len(want)], want, dd[sl][lv], what, whole=False)
        else:
            assert np.array_equal(arena, base), what
        t_end = time.perf_counter() + float(rng.integers(0, 3 * idle_us)) * 1e-6
        while time.perf_counter() < t_end:
            pass
    s = ctx.stats()
    assert s["service_batches"] == iters and s["service_launches"] >= 1
    ctx.close()


def test_group_and_default_group_submit_pre(V, orc):
    """vpcsum_group_submit_pre over two contexts on one card, and vpcsum_batch_submit_pre on the
    process-wide group: the same bytes as Java."""
    import ctypes
    rng = np.random.default_rng(33)
    after, desc, pre, want, wst = nat_case(orc, rng, 2000, O.SYNTH_C5, pad=14, stride=2048)
    g = V.Group((0, 0), max_arena=after.nbytes, max_pkts=len(desc))
    a = after.copy()
    out = np.zeros(len(desc), np.uint32)
    g.wait(g.submit_pre(a, desc, pre, out, None, O.MODE_WRITE))
    assert np.array_equal(a, want)
    g.close()
    L = V.lib()
    a = after.copy()
    out[:] = 0
    assert L.vpcsum_init(1, a.nbytes, len(desc)) == 0
    try:
        h = ctypes.c_uint64()
        assert L.vpcsum_batch_submit_pre(a.ctypes.data, a.nbytes, desc.ctypes.data, pre.ctypes.data, V.PRE_FMT_PRE,
                                         len(desc), out.ctypes.data, None, O.MODE_WRITE, ctypes.byref(h)) == 0
        assert L.vpcsum_batch_wait(h.value) == 0
    finally:
        L.vpcsum_shutdown()
    assert np.array_equal(a, want)


def _eth_frames(orc, rng, n):
    """C5-like Ethernet frames in a umem layout (2-KB chunks, L2 at +384): IPv4 TCP / UDP of 1500 B
    with valid sums; 30% get a payload byte changed after their sums were taken (invalid L4 input),
    10% of the UDP ones a stored 0."""
    arena, desc = orc.synth(n, 2048, 398, O.SYNTH_C5, O.SEED, int(rng.integers(0, 1 << 30)))
    orc.process(arena, desc, O.MODE_COMPUTE, write=True)
    offs = np.arange(n) * 2048 + 384
    arena.reshape(n, 2048)[:, 384:396] = rng.integers(0, 256, (n, 12), dtype=np.uint8)
    arena.reshape(n, 2048)[:, 396:398] = (0x08, 0x00)
    for i in range(n):
        o = int(desc[i]["l3_off"])
        if rng.random() < 0.3:
            arena[o + 40 + int(rng.integers(0, 1400))] ^= 0x5A
        elif desc[i]["l4_proto"] == 17 and rng.random() < 0.1:
            arena[o + 26:o + 28] = 0
    return arena, offs, np.full(n, 14 + 1500)


def test_nat_flow_ingress_to_egress(V, orc):
    """The path the vswitch runs for NAT'd frames, on one registered umem:
    ingress verify on the GPU (XDPIface.readable) -> DevInput's csum-recalc "all" policy -> for each
    frame the pre-image, then Java's setters (SwitchUtils.applyNat) -> the egress batch defers it
    with its dirty flags, pre-image and ingress status -> one flush (Iface.completeTx).  Frames:
    10k C5-like frames (30% with invalid L4 sums, UDP stored 0), the reference's pcap frames (12
    CHECKSUM_PARTIAL: invalid as full sums) and KAT frames.  Every frame equals what Java leaves:
    the setters, then every sum recomputed in full (csum-recalc all + the setters' dirty flags).
    Frames with a verified L4 sum took the pre-image path, the others the full recompute."""
    from test_ingress_policy import _rx_batch
    from vproxy_amd import vswitch as S
    rng = np.random.default_rng(2025)
    a1, o1, l1 = _eth_frames(orc, rng, 10000)
    a2, o2, l2 = _rx_batch(orc)
    arena = np.concatenate([a1, a2, np.zeros(4096, np.uint8)])
    offs = np.concatenate([o1, o2 + len(a1)])
    lens = np.concatenate([l1, l2])
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=len(offs))
    ctx.register(arena)
    desc, pst, _ = ctx.parse_frames(arena, offs, lens)
    _, st = ctx.run(arena, desc, V.MODE_VERIFY)
    st = np.where(pst & V.S_BAD_DESC, V.S_BAD_DESC, st).astype(np.uint8)
    parsed = (st & V.S_BAD_DESC) == 0
    dec = S.recalc_policy(st, desc, "all")
    # NAT: a rewrite of addresses and ports for every parsed frame with an L4 sum field
    n = len(offs)
    rw = np.zeros(n, O.NAT_DTYPE)
    rw.view(np.uint8).reshape(n, 48)[:, :36] = rng.integers(0, 256, (n, 36), dtype=np.uint8)
    rw["mask"] = NAT_FIELDS
    nat = parsed & ((desc["flags"] & O.F_L4) != 0)
    pre = pre_images(arena, desc, rw)
    want = arena.copy()
    d_all = desc[nat].copy()
    orc.nat_setters(want, d_all, rw[nat])
    orc.process(want, d_all, O.MODE_COMPUTE, write=True)          # Java: csum-recalc all + setters
    orc.nat_setters(arena, d_all, rw[nat])                        # the vswitch's setters (Java)
    batch = S.EgressBatch(arena, capacity=n, register=False)
    batch.ctx.close()
    batch.ctx = ctx                                               # the umem's context
    for i in np.nonzero(nat)[0]:
        d = desc[i]
        batch.defer(int(d["l3_off"]), int(d["l3_len"]), int(d["l4_off"]), int(d["l3_ver"]), int(d["l4_proto"]),
                    int(d["flags"]), pre=pre[i], rx_status=int(st[i]))
    assert batch.complete_tx() == int(nat.sum())
    for i in np.nonzero(nat)[0]:
        o, L = int(desc[i]["l3_off"]), int(desc[i]["l3_len"])
        assert np.array_equal(arena[o:o + L], want[o:o + L]), i
    assert np.array_equal(arena, want)
    s = batch.stats
    assert s["pre_deferred"] + s["pre_full"] == int(nat.sum())
    assert s["pre_deferred"] > 0.5 * nat.sum() and s["pre_full"] > 0.2 * nat.sum()
    assert s["pre_deferred"] == int(np.count_nonzero(nat & ((st & V.S_L4_OK) != 0)))
    assert dec.stats["rx_csum_bad"] >= 12
    ctx.close()


def test_full_size_c5_preimage(V, orc):
    """BASELINE config C5 at full size through the pre-image flush (the bench's --preimage step):
    10,000,000 x 1500 B IPv4 TCP / UDP with valid sums, 16-B pre-images of their addresses and
    ports, Java's setters applied (new bytes, stale sums), one vpcsum_pre_async over all of them.
    Only the two sum fields are written, so "every packet verifies on the GPU" (stored == full
    recompute of the new bytes, for all 10M) is byte equality with Java's setters + getRawPacket(0);
    a sample of 4096 packets is also regenerated and rewritten by the oracle and compared whole."""
    import torch
    n, stride = 10_000_000, 2048
    arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    V.synth(arena, n, stride, 0, O.SYNTH_C5, O.SEED, 0, d)
    V.compute(arena, d, n, None, None, O.MODE_WRITE)
    g = torch.Generator(device="cpu").manual_seed(57)
    rw = torch.randint(0, 256, (n, 16), dtype=torch.uint8, generator=g)
    rw[:, 12] = NAT_FIELDS
    rw[:, 13:] = 0
    rw_d = rw.cuda()
    fr = arena.view(n, stride)
    p4 = torch.zeros((n, 16), dtype=torch.uint8, device="cuda")
    p4[:, 0:8] = fr[:, 12:20]
    p4[:, 8:12] = fr[:, 20:24]
    p4[:, 12] = NAT_FIELDS
    fr[:, 12:20] = rw_d[:, 0:8]
    fr[:, 20:24] = rw_d[:, 8:12]
    d.view(n, 16)[:, 14] |= O.F_PRE
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    V.pre(arena, d, p4, n, None, st, O.MODE_WRITE, pre_fmt=0)
    torch.cuda.synchronize()
    assert bool((st == O.S_DONE).all())
    d.view(n, 16)[:, 14] &= 0xFF ^ O.F_PRE
    vs = torch.zeros(n, dtype=torch.uint8, device="cuda")
    V.compute(arena, d, n, None, vs, O.MODE_VERIFY)
    torch.cuda.synchronize()
    assert bool(((vs & 3) == 3).all()), "a flushed packet does not verify"
    rng = np.random.default_rng(58)
    i0 = int(rng.integers(0, n - 4096))
    a, dd = orc.synth(4096, stride, 0, O.SYNTH_C5, O.SEED, i0)
    orc.process(a, dd, O.MODE_COMPUTE, write=True)
    orc.nat4_java(a, dd, np.ascontiguousarray(rw.numpy().view(O.NAT4_DTYPE).reshape(-1)[i0:i0 + 4096]))
    assert np.array_equal(arena[i0 * stride:(i0 + 4096) * stride].cpu().numpy(), a)
    del arena, fr


@pytest.mark.parametrize("idle_us", [5000, 40])
def test_service_mixed_forms(V, orc, idle_us):
    """One context with the service grid on, two registered arenas (raw Ethernet frames as the TX /
    RX rings hold them, and NAT'd C5-like frames with pre-images), and a random sequence of every
    batch form the grid takes -- descriptor flushes in all three modes, raw egress frames, RX verify
    with and without sums, RX parse with tuples, pre-image flushes -- of 1..600 frames (above 512:
    launched): after every batch the results and both arenas equal a twin context's without the
    service (the launched kernels, each pinned to the oracle by the tests above).  Catches state
    carried from one form to the next: the command flags, the parameter block switching arenas and
    write modes, the aux buffer shared by pre-images and parse results."""
    import sys
    import time
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import egressvec as E
    rng = np.random.default_rng(70 + idle_us)
    fs = E.frames()
    ea, offs = E.layout(fs)
    flags = [E.want_flags(f["ver"], f["proto"], i) for i, f in enumerate(fs)]
    edesc = E.oracle_descriptors(fs, offs, flags)
    offs = np.array(offs, np.uint64)
    lens = np.array([len(f["frame"]) for f in fs], np.uint32)
    fflags = np.array(flags, np.uint8)
    after, ndesc, pre, _, _ = nat_case(orc, rng, 700, O.SYNTH_C5, pad=14, stride=2048, udp_zero=0.1, mask=NAT_FIELDS)
    full = rng.random(len(ndesc)) < 0.3
    ndesc["flags"][full] &= 0xFF ^ O.F_PRE
    arenas = {"svc": (ea.copy(), after.copy()), "ref": (ea.copy(), after.copy())}
    ctxs = {}
    for k, (a1, a2) in arenas.items():
        c = V.Context(0, max_arena=max(a1.nbytes, a2.nbytes), max_pkts=1024)
        c.register(a1)
        c.register(a2)
        if k == "svc":
            c.set_service(idle_us)
        ctxs[k] = c
    n_svc = 0
    for it in range(60):
        form = str(rng.choice(["submit", "egress", "verify", "verify_st", "parse", "pre"]))
        b = int(rng.choice([1, 3, 5, 32, 200, 512, 600]))
        res = {}
        for k in ("svc", "ref"):
            c, (a1, a2) = ctxs[k], arenas[k]
            r2 = np.random.default_rng(it)                      # the same subset for both contexts
            if form == "pre":
                idx = np.sort(r2.choice(len(ndesc), b, replace=False))
                d = np.ascontiguousarray(ndesc[idx])
                res[k] = c.run_pre(a2, d, np.ascontiguousarray(pre[idx]), O.MODE_WRITE)
            elif form == "submit":
                idx = np.sort(r2.choice(len(edesc), min(b, len(edesc)), replace=False))
                mode = int(r2.choice([O.MODE_COMPUTE, O.MODE_VERIFY, O.MODE_WRITE]))
                out = np.zeros(len(idx), np.uint32)
                st = np.zeros(len(idx), np.uint8)
                c.wait(c.submit(a1, np.ascontiguousarray(edesc[idx]), out, st, mode))
                res[k] = (out, st)
            else:
                idx = r2.choice(len(fs), min(b, len(fs)), replace=False)
                if form == "egress":
                    res[k] = c.egress_frames(a1, offs[idx], lens[idx], fflags[idx])
                elif form == "parse":
                    dd, st, tu = c.parse_frames(a1, offs[idx], lens[idx])
                    res[k] = (dd.tobytes(), st, tu.tobytes())
                else:
                    res[k] = c.verify_frames(a1, offs[idx], lens[idx], sums=form == "verify")
        what = f"it {it} form {form} n {b}"
        for x, y in zip(res["svc"], res["ref"]):
            if x is None or isinstance(x, bytes):
                assert x == y, what
            else:
                assert np.array_equal(x, y), what
        assert np.array_equal(arenas["svc"][0], arenas["ref"][0]) and np.array_equal(arenas["svc"][1], arenas["ref"][1]), what
        n_svc += b <= 512 if form == "pre" else min(b, len(fs)) <= 512
        t_end = time.perf_counter() + float(rng.integers(0, 3 * idle_us)) * 1e-6
        while time.perf_counter() < t_end:
            pass
    assert ctxs["svc"].stats()["service_batches"] == n_svc and ctxs["ref"].stats()["service_batches"] == 0
    for c in ctxs.values():
        c.close()


def test_service_grids_of_four_contexts_in_threads(V, orc):
    """Four switches' contexts in four threads (one context per event loop, thread-safe
    across them), each with its own service grid resident at once, each flushing its own umem:
    descriptor flushes (WRITE), NAT'd flushes from pre-images and RX verifies of random sizes.  Every
    result equals the oracle's (Java's bytes for the NAT'd frames)."""
    import threading
    ctxs, errors = [], []

    def work(k):
        try:
            rng = np.random.default_rng(90 + k)
            after, desc, pre, want, wst = nat_case(orc, rng, 400, O.SYNTH_C5, pad=14, stride=2048, mask=NAT_FIELDS)
            arena = after.copy()
            c = V.Context(0, max_arena=arena.nbytes, max_pkts=512)
            ctxs.append(c)
            c.register(arena)
            c.set_service(5000)
            live = desc["flags"] != 0
            for it in range(25):
                b = int(rng.choice([1, 4, 32, 200, 400]))
                idx = np.sort(rng.choice(len(desc), b, replace=False))
                arena[:] = after
                d = np.ascontiguousarray(desc[idx])
                out, st = c.run_pre(arena, d, np.ascontiguousarray(pre[idx]), O.MODE_WRITE)
                for j, i in enumerate(idx):
                    if live[i]:
                        o, L = int(desc[i]["l3_off"]), int(desc[i]["l3_len"])
                        if not np.array_equal(arena[o:o + L], want[o:o + L]) or st[j] != O.S_DONE:
                            errors.append((k, it, int(i)))
                            return
                # the same frames, now Java's bytes, verified: every live packet's stored sums are right
                vd = np.ascontiguousarray(desc[idx])
                vd["flags"] = np.where(vd["flags"] != 0, vd["flags"] & (O.F_IP | O.F_L4), O.F_IP | O.F_L4)
                _, vst = c.run(arena, vd, O.MODE_VERIFY)
                for j, i in enumerate(idx):
                    if live[i] and ((vst[j] & O.S_L4_OK) == 0 or ((vd[j]["flags"] & O.F_IP) and (vst[j] & O.S_IP_OK) == 0)):
                        errors.append((k, it, int(i), "verify"))
                        return
        except Exception as e:   # reported by the main thread
            errors.append((k, repr(e)))

    ts = [threading.Thread(target=work, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    try:
        assert not errors, errors[:4]
        assert len(ctxs) == 4 and all(c.stats()["service_batches"] == 50 for c in ctxs)
    finally:
        for c in ctxs:
            c.close()


def test_service_one_context_two_threads(V, orc):
    """Two threads sharing ONE context with its service grid on (the C-ABI is thread-safe: the
    context's mutex orders the submissions): each thread flushes NAT'd frames from
    pre-images and verifies them, on its own half of one registered umem, submitting and waiting on
    its own tickets while the other's batches come and go.  A submission that finds the other
    thread's batch still on the grid completes it first (its results go to that thread's buffers);
    every result equals the oracle's (Java's bytes), and every batch the grid took is counted."""
    import threading
    rng = np.random.default_rng(95)
    after, desc, pre, want, _ = nat_case(orc, rng, 800, O.SYNTH_C5, pad=14, stride=2048, mask=NAT_FIELDS)
    arena = after.copy()
    c = V.Context(0, max_arena=arena.nbytes, max_pkts=512)
    c.register(arena)
    c.set_service(5000)
    live = desc["flags"] != 0
    errors, posted = [], [0, 0]

    def frames(i):
        o, L = int(desc[i]["l3_off"]), int(desc[i]["l3_len"])
        return slice(o, o + L)

    def work(k):
        try:
            r = np.random.default_rng(200 + k)
            mine = np.arange(k, len(desc), 2)                 # disjoint frames per thread
            for it in range(40):
                b = int(r.choice([1, 5, 32, 200, 400]))
                idx = np.sort(r.choice(mine, b, replace=False))
                for i in idx:
                    arena[frames(i)] = after[frames(i)]
                out = np.zeros(b, np.uint32)
                st = np.zeros(b, np.uint8)
                t = c.submit_pre(arena, np.ascontiguousarray(desc[idx]), np.ascontiguousarray(pre[idx]), out, st,
                                 O.MODE_WRITE)
                c.wait(t)
                vd = np.ascontiguousarray(desc[idx])
                vd["flags"] = O.F_IP | O.F_L4
                vst = np.zeros(b, np.uint8)
                c.wait(c.submit(arena, vd, None, vst, O.MODE_VERIFY))
                posted[k] += 2
                for j, i in enumerate(idx):
                    if not live[i]:
                        continue
                    if st[j] != O.S_DONE or not np.array_equal(arena[frames(i)], want[frames(i)]):
                        errors.append((k, it, int(i), "flush"))
                        return
                    if (vst[j] & (O.S_IP_OK | O.S_L4_OK)) != (O.S_IP_OK | O.S_L4_OK):
                        errors.append((k, it, int(i), "verify", int(vst[j])))
                        return
        except Exception as e:   # reported by the main thread
            errors.append((k, repr(e)))

    ts = [threading.Thread(target=work, args=(k,)) for k in range(2)]
    try:
        for t in ts:
            t.start()
        for t in ts:
            t.join(120)
        assert not any(t.is_alive() for t in ts), "a thread did not finish"
        assert not errors, errors[:4]
        assert c.stats()["service_batches"] == sum(posted) == 160
    finally:
        c.close()
