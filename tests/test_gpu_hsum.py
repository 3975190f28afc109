"""GPU parity of the ingress-header-sum flush (VPCSUM_PRE_HSUM; VERDICT r5 "Next round" item 1).

The RX verify records each received TCP / UDP frame's header sum (vpcsum_ctx_verify_frames_hsum,
vpcsum_parse_ether_hsum_async); the egress flush updates the L4 sum of a frame the vswitch changed
in place from that record and the header words now in the frame (vpcsum_pre_async /
vpcsum_ctx_submit_pre with VPCSUM_PRE_HSUM entries).  The oracle is Java's: the setters' bytes,
then getRawPacket(0)'s full recompute of every dirty sum (oracle.l4_csum / Oracle.process).

* the records the GPU writes equal oracle.hsum_record, frame for frame (launched parse, the
  service grid's RX verify);
* any in-place change of the summed words -- NAT, the PROXY-protocol SYN / SYN-ACK rewrite, an MSS
  option clamped in place -- is flushed to Java's bytes, on the device API (both entry formats) and
  through the host seam (launched, service grid, staged);
* a record that does not describe the packet (lengths, data offset, protocol, version, no record)
  is refused: S_BAD_DESC, nothing written;
* the whole vswitch flow (tests/hsumvec.py scenarios: NAT, MSS clamp in place, MSS added (rebuilt),
  PROXY-protocol SYN / SYN-ACK, TcpReset replacement, rebuilt payload, TTL only) with verify ->
  csum-recalc "all" -> the setters -> EgressBatch.defer_rx -> one flush: every frame equals Java's;
  only in-place frames with S_L4_OK take F_PRE.
"""
import numpy as np
import pytest

from oracle import oracle as O

import hsumvec as H

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def V():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vproxy_amd import vpcsum
    vpcsum.lib()
    return vpcsum


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).pin_memory().cuda()


def _ld16(a, o):
    return (int(a[o]) << 8) | int(a[o + 1])


def _records(fs):
    return np.array([O.hsum_record(f["frame"]) for f in fs], O.HSUM_DTYPE)


def _pcap_eth():
    import os
    from pcaputil import read_pcap
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pcap")
    out = []
    for name in sorted(os.listdir(here)):
        if name.endswith(".pcap"):
            lt, pkts = read_pcap(os.path.join(here, name))
            if lt == 1:
                out += [dict(frame=p) for p in pkts if len(p) <= H.CHUNK - H.HEADROOM]
    return out


def test_parse_ether_hsum_matches_oracle(V):
    """vpcsum_parse_ether_hsum_async: the hsumvec frames, the egress frames (padding, IPv4 options,
    802.1Q, IPv6 extension headers and trailers) and the reference's Ethernet pcap frames; every
    record equals oracle.hsum_record, descriptors and status equal vpcsum_parse_ether_async's."""
    import torch
    import egressvec as E
    fs = H.received(31, 700) + [dict(frame=f["frame"]) for f in E.frames()] + _pcap_eth()
    arena, offs, _ = H.layout(fs, 0)
    lens = np.array([len(f["frame"]) for f in fs], np.uint32)
    n = len(fs)
    a = dev(arena)
    fo = torch.from_numpy(np.array(offs, np.uint64)).cuda()
    fl = torch.from_numpy(lens).cuda()
    d1 = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    s1 = torch.zeros(n, dtype=torch.uint8, device="cuda")
    d2 = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    s2 = torch.zeros(n, dtype=torch.uint8, device="cuda")
    hs = torch.full((n * 8,), 0xEE, dtype=torch.uint8, device="cuda")
    V.parse_ether(a, fo, fl, n, d1, s1)
    V.parse_ether(a, fo, fl, n, d2, s2, hsum=hs)
    torch.cuda.synchronize()
    assert torch.equal(d1, d2) and torch.equal(s1, s2)
    got = hs.cpu().numpy().view(O.HSUM_DTYPE)
    want = _records(fs)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (len(bad), bad[:5], got[bad[:3]], want[bad[:3]])
    assert np.count_nonzero(want["l2_len"]) > 600


@pytest.mark.parametrize("service", [False, True])
def test_ctx_verify_frames_hsum(V, service):
    """vpcsum_ctx_verify_frames_hsum on a registered umem: launched (1,200 frames) and, with the
    service grid on, small batches (1..512 frames): status bytes equal vpcsum_ctx_verify_frames',
    records equal the oracle's."""
    fs = H.received(32, 1200)
    arena, offs, _ = H.layout(fs, 0)
    lens = np.array([len(f["frame"]) for f in fs], np.uint32)
    offs = np.array(offs, np.uint64)
    want = _records(fs)
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=len(fs))
    ctx.register(arena)
    if service:
        ctx.set_service(5000)
        cuts = [0, 1, 3, 35, 547, 1059, 1200]
    else:
        cuts = [0, 1200]
    sts = []
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        _, st_ref = ctx.verify_frames(arena, offs[lo:hi], lens[lo:hi], sums=False)
        st, hs = ctx.verify_frames_hsum(arena, offs[lo:hi], lens[lo:hi])
        assert np.array_equal(st, st_ref), (lo, hi)
        assert np.array_equal(hs, want[lo:hi]), (lo, hi)
        sts.append(st)
    if service:
        assert ctx.stats()["service_batches"] >= 8
    ok = (np.concatenate(sts) & O.S_L4_OK) != 0
    assert 0.6 * len(fs) < ok.sum() < len(fs)
    ctx.close()


def _edit_headers(rng, arena, offs, fs, recs):
    """Random in-place edits of the summed words (addresses, ports, seq / ack, flags, window,
    options: what the in-place setters reach) of every frame; returns the egress descriptors
    (F_L4 | F_PRE, F_IP too for IPv4: the address setters dirty it) and Java's bytes."""
    from vproxy_amd import vswitch as S
    n = len(fs)
    desc = np.zeros(n, O.DESC_DTYPE)
    for i, (f, off) in enumerate(zip(fs, offs)):
        d = S.egress_descriptor(arena[off:off + 512], off, 0)
        l3, l4o, proto = int(d["l3_off"]), int(d["l4_off"]), int(d["l4_proto"])
        hlen = int(recs[i]["hlen"]) or 8
        fld = O.L4_FIELD[proto]
        alen, a0 = (4, 12) if f["ver"] == 4 else (16, 8)
        cand = list(range(l3 + a0, l3 + a0 + 2 * alen)) + \
            [l3 + l4o + k for k in range(hlen) if k not in (fld, fld + 1) and not (proto == 6 and k == 12)]
        for b in rng.choice(cand, size=int(rng.integers(1, min(12, len(cand)) + 1)), replace=False):
            arena[b] = rng.integers(0, 256)
        d["flags"] = O.F_L4 | O.F_PRE | (O.F_IP if f["ver"] == 4 else 0)
        desc[i] = d
    want = arena.copy()
    d2 = desc.copy()
    d2["flags"] &= O.F_IP | O.F_L4
    O.Oracle().process(want, d2, O.MODE_COMPUTE, write=True)
    return desc, want


def _entries(recs, fmt):
    """Pre-image entries carrying the records: 48-B vpcsum_pre_t (fmt 1) or 16-B vpcsum_pre4_t."""
    if fmt == 1:
        e = np.zeros(len(recs), O.NAT_DTYPE)
        raw = e.view(np.uint8).reshape(len(recs), 48)
        raw[:, :8] = recs.view(np.uint8).reshape(len(recs), 8)
        raw[:, 36] = O.PRE_HSUM
    else:
        e = np.zeros(len(recs), O.NAT4_DTYPE)
        raw = e.view(np.uint8).reshape(len(recs), 16)
        raw[:, :8] = recs.view(np.uint8).reshape(len(recs), 8)
        raw[:, 12] = O.PRE_HSUM
    return e


@pytest.mark.parametrize("fmt", [1, 0])
@pytest.mark.parametrize("tune", [0, 0x100, 0x2000])
def test_pre_async_hsum_any_header_edit(V, fmt, tune):
    """vpcsum_pre_async with VPCSUM_PRE_HSUM entries (48-B; 16-B for IPv4 only) after random
    in-place edits of every summed word class: Java's bytes and out words on every packet, through
    the LDS window, the byte path (tune 0x100) and two packets per lane (0x2000)."""
    import torch
    rng = np.random.default_rng(40 + fmt)
    fs = [f for f in H.received(33 + fmt, 1500) if not f["corrupt"] and not f["udp0"]]
    if fmt == 0:
        fs = [f for f in fs if f["ver"] == 4]
    arena, offs, _ = H.layout(fs, 0)
    recs = _records(fs)
    desc, want = _edit_headers(rng, arena, offs, fs, recs)
    a = dev(arena)
    n = len(fs)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    V.pre(a, dev(desc), dev(_entries(recs, fmt)), n, out, st, O.MODE_WRITE | tune, pre_fmt=fmt)
    torch.cuda.synchronize()
    got = a.cpu().numpy()
    assert np.all(st.cpu().numpy() == O.S_DONE)
    bad = [i for i, d in enumerate(desc)
           if not np.array_equal(got[int(d["l3_off"]):int(d["l3_off"]) + int(d["l3_len"])],
                                 want[int(d["l3_off"]):int(d["l3_off"]) + int(d["l3_len"])])]
    assert not bad, (len(bad), [fs[i]["scenario"] for i in bad[:5]])
    assert np.array_equal(got, want)
    d2 = desc.copy()
    d2["flags"] &= O.F_IP | O.F_L4
    exp, _ = O.Oracle().process(want, d2)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), exp)


def test_pre_async_hsum_refuses_other_shapes(V):
    """A record that does not describe the packet -- another segment length, header length (the
    data offset now in the frame), protocol or version, or no record at all -- is refused:
    S_BAD_DESC, out 0, the frame untouched; the good neighbours are written."""
    import torch
    rng = np.random.default_rng(77)
    fs = [f for f in H.received(35, 600) if not f["corrupt"] and not f["udp0"]]
    arena, offs, _ = H.layout(fs, 0)
    recs = _records(fs)
    desc, want = _edit_headers(rng, arena, offs, fs, recs)
    n = len(fs)
    kind = np.arange(n) % 6
    r2 = recs.copy()
    r2["l4_len"][kind == 1] += 4
    r2["hlen"][kind == 2] += 4
    r2["l4_proto"][kind == 3] ^= 6 ^ 17
    r2["l3_ver"][kind == 4] ^= 4 ^ 6
    r2["l2_len"][kind == 5] = 0
    a = dev(arena)
    out = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    V.pre(a, dev(desc), dev(_entries(r2, 1)), n, out, st, O.MODE_WRITE, pre_fmt=1)
    torch.cuda.synchronize()
    got, st, out = a.cpu().numpy(), st.cpu().numpy(), out.cpu().numpy()
    for i, d in enumerate(desc):
        o, L = int(d["l3_off"]), int(d["l3_len"])
        if kind[i] == 0:
            assert st[i] == O.S_DONE and np.array_equal(got[o:o + L], want[o:o + L]), i
        else:
            assert st[i] == O.S_BAD_DESC and out[i] == 0 and np.array_equal(got[o:o + L], arena[o:o + L]), (i, kind[i])


@pytest.mark.parametrize("path", ["launched", "service", "staged"])
def test_hsum_flow_ingress_to_egress(V, path):
    """The vswitch path for received frames on a registered umem: GPU verify
    with header sums (XDPIface.readable) -> csum-recalc "all" (DevInput) -> each frame's scenario
    through the Java setters' byte effects (vswitch.RxPacket: NAT, MSS clamped in place or added by
    a rebuild, the PROXY-protocol SYN / SYN-ACK rewrite, a TcpReset replacement, a rebuilt payload,
    a TTL) -> EgressBatch.defer_rx (GpuCsumBatch.defer's rule) -> flushes (Iface.completeTx):
    launched (one flush of every frame), on the service grid (flushes of <= 512), or staged (a
    context without the umem registered).  Every frame -- in place or rebuilt into another chunk --
    equals Java's bytes: the same setters, then every dirty sum recomputed in full.  F_PRE went to
    exactly the in-place frames with S_L4_OK and an L4 sum to update, never to a rebuilt or
    replaced one."""
    from vproxy_amd import vswitch as S
    rng = np.random.default_rng({"launched": 1, "service": 2, "staged": 3}[path])
    fs = H.received(36, 1600)
    arena, offs, free = H.layout(fs, 700)
    lens = np.array([len(f["frame"]) for f in fs], np.uint32)
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=len(fs))
    ctx.register(arena)
    st, hs = ctx.verify_frames_hsum(arena, np.array(offs, np.uint64), lens)
    assert np.array_equal(hs, _records(fs))
    pkts = []
    for i, (f, off) in enumerate(zip(fs, offs)):
        rx = S.RxPacket(arena, off, int(st[i]), hs[i])
        rx.ip_dirty = rx.ver == 4 and not st[i] & O.S_IP_OK     # csum-recalc "all" (recalc_policy)
        rx.l4_dirty = not st[i] & O.S_L4_OK
        H.apply(rx, f, rng, free)
        pkts.append(rx)
    # Java's bytes: every frame as the setters left it, its dirty sums recomputed in full
    want = arena.copy()
    jd = []
    for rx in pkts:
        fl = S.checksum_flags_for(rx.ver == 4, rx.ip_dirty, rx.proto, rx.l4_dirty)
        if fl:
            jd.append(S.egress_descriptor(arena[rx.frame_off:rx.frame_off + 512], rx.frame_off, fl))
    jd = np.array(jd, O.DESC_DTYPE)
    O.Oracle().process(want, jd, O.MODE_COMPUTE, write=True)
    if path == "staged":
        fctx = V.Context(0, max_arena=arena.nbytes, max_pkts=len(fs))
    else:
        fctx = ctx
        if path == "service":
            ctx.set_service(5000)
    batch = S.EgressBatch(arena, capacity=512 if path == "service" else len(fs), register=False)
    batch.ctx.close()
    batch.ctx = fctx
    expect_pre = 0
    for rx, f in zip(pkts, fs):
        flags = S.checksum_flags_for(rx.ver == 4, rx.ip_dirty, rx.proto, rx.l4_dirty)
        if flags & O.F_L4 and rx.in_place and rx.csum_status & O.S_L4_OK:
            expect_pre += 1
        batch.defer_rx(rx)
        if f["scenario"] in ("nat_mss_add", "tcp_reset", "payload") and not rx.in_place:
            assert not batch.desc[batch.n - 1]["flags"] & O.F_PRE, f["scenario"]
    batch.complete_tx()
    assert batch.stats["rejected"] == 0
    bad = [j for j, d in enumerate(jd)
           if not np.array_equal(arena[int(d["l3_off"]):int(d["l3_off"]) + int(d["l3_len"])],
                                 want[int(d["l3_off"]):int(d["l3_off"]) + int(d["l3_len"])])]
    assert not bad, (path, len(bad), bad[:5])
    assert np.array_equal(arena, want)
    s = batch.stats
    assert s["pre_deferred"] == expect_pre and expect_pre > 500, (s, expect_pre)
    assert s["pre_full"] > 50
    if path == "service":
        assert ctx.stats()["service_batches"] >= 3
    if fctx is not ctx:
        fctx.close()
    ctx.close()
