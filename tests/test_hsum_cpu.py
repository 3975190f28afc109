"""The ingress-header-sum flush on the CPU (no GPU): the record, the arithmetic and the seam's rule.

A received TCP / UDP frame's ingress header sum (vpcsum_hsum_t, oracle.hsum_record) sums every word
of the L4 sum that the vswitch's in-place setters can reach -- addresses, ports, sequence and
acknowledgement numbers, flags, window, options.  At egress the L4 sum is updated from it as RFC 1624
eqn. 3 with the header as one word (pre_common.h:pre_sums, restated below as `hsum_update`).  This
file pins:

* the record against an independent word-by-word sum (and the reference's own fixtures: the pcap
  frames and the egress frames);
* the update against Java's full recompute (oracle.l4_csum: TcpPacket / UdpPacket.updateChecksumWith*,
  getRawPacket(0)) after ANY in-place edit of those words, on frames whose stored sum was correct;
  and its divergence when a payload byte changes (why the seam requires the frame in place);
* the seam's rule (vswitch.hsum_eligible / RxPacket / EgressBatch.defer_rx, mirrored by
  GpuCsumBatch.defer) on every scenario of tests/hsumvec.py: whenever it grants F_PRE, the update
  equals Java's bytes; MSS options added, replaced packets (TcpReset) and rebuilt payloads are
  never granted it.
"""
import numpy as np
import pytest

from oracle import oracle as O

import hsumvec as H


def _fold(x):
    while x >> 16:
        x = (x & 0xFFFF) + (x >> 16)
    return x


def _ld16(a, o):
    return (int(a[o]) << 8) | int(a[o + 1])


def hsum_update(arena, d, rec):
    """pre_common.h:pre_sums for a VPCSUM_PRE_HSUM entry: the L4 sum the flush writes for
    descriptor d, None for a refused record, "udp_full" for a UDP stored 0 (summed in full)."""
    l3, ver, proto = int(d["l3_off"]), int(d["l3_ver"]), int(d["l4_proto"])
    l3_len, l4o = int(d["l3_len"]), int(d["l4_off"])
    hlen = int(rec["hlen"])
    cur = (int(arena[l3 + l4o + 12]) >> 4) * 4 if proto == 6 else 8
    if (int(rec["l2_len"]) == 0 or int(rec["l3_ver"]) != ver or int(rec["l4_proto"]) != proto
            or int(rec["l4_len"]) != l3_len - l4o or hlen != cur or proto not in (6, 17)):
        return None
    w = O.hdr_words(bytes(arena[l3:l3 + l3_len]), ver, l4o, hlen, proto)
    now = _fold(sum(_ld16(w, k) for k in range(0, len(w), 2)))
    hc = _ld16(arena, l3 + l4o + O.L4_FIELD[proto])
    if proto == 17 and hc == 0:
        return "udp_full"
    c = ~_fold((~hc & 0xFFFF) + _fold((~int(rec["sum"]) & 0xFFFF) + now)) & 0xFFFF
    return 0xFFFF if proto == 17 and c == 0 else c


def _pcap_frames():
    import os
    from pcaputil import read_pcap
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pcap")
    out = []
    for name in sorted(os.listdir(here)):
        if name.endswith(".pcap"):
            lt, pkts = read_pcap(os.path.join(here, name))
            if lt == 1:   # Ethernet captures (the others are not frames the vswitch receives)
                out += pkts
    return out


def test_hsum_record_is_the_header_word_sum():
    """oracle.hsum_record on the reference's pcap frames, the egress frames and the hsumvec frames
    equals a plain end-around sum of the pseudo-header addresses and the L4 header words (checksum
    field excluded); frames that are not TCP / UDP, or whose TCP data offset leaves the segment,
    get no record (l2_len 0)."""
    import egressvec as E
    frames = _pcap_frames() + [f["frame"] for f in E.frames()] + [f["frame"] for f in H.received(5, 300)]
    recorded = 0
    for fr in frames:
        r = O.hsum_record(fr)
        info, _ = O.parse_ether(fr)
        if info is None or info.proto not in (6, 17):
            assert int(r["l2_len"]) == 0
            continue
        l3 = bytes(fr)[info.l3_off:info.l3_off + info.l3_len]
        seg = info.l3_len - info.l4_off
        hlen = (l3[info.l4_off + 12] >> 4) * 4 if info.proto == 6 and seg >= 20 else 8
        if seg < 8 or (info.proto == 6 and (seg < 20 or hlen < 20 or hlen > seg)):
            assert int(r["l2_len"]) == 0
            continue
        a = (12, 20) if info.ver == 4 else (8, 40)
        words = [_ld16(l3, k) for k in range(a[0], a[1], 2)]
        words += [_ld16(l3, info.l4_off + k) for k in range(0, hlen, 2) if k != O.L4_FIELD[info.proto]]
        assert int(r["sum"]) == _fold(sum(words))
        assert (int(r["l4_len"]), int(r["hlen"]), int(r["l4_proto"]), int(r["l3_ver"]), int(r["l2_len"])) == \
            (seg, hlen, info.proto, info.ver, info.l3_off)
        recorded += 1
    assert recorded > 300


def _desc_of(arena, off):
    from vproxy_amd import vswitch as S
    return S.egress_descriptor(arena[off:off + 512], off, O.F_L4)


def test_hsum_update_equals_java_after_any_header_edit():
    """Frames with correct sums; random in-place edits of any subset of the words the record sums
    (addresses, ports, seq, ack, flags / data offset byte kept, window, urgent pointer, option
    bytes); the update from the record equals Java's full recompute of the edited frame, for IPv4
    (with options) and IPv6 (with an extension header), TCP and UDP, 802.1Q or not."""
    rng = np.random.default_rng(17)
    fs = [f for f in H.received(8, 2000) if not f["corrupt"] and not f["udp0"]]
    arena, offs, _ = H.layout(fs, 0)
    checked = 0
    for f, off in zip(fs, offs):
        rec = O.hsum_record(f["frame"])
        assert int(rec["l2_len"])
        d = _desc_of(arena, off)
        l3, l4o, proto = int(d["l3_off"]), int(d["l4_off"]), int(d["l4_proto"])
        hlen = int(rec["hlen"])
        fld = O.L4_FIELD[proto]
        alen, a0 = (4, 12) if f["ver"] == 4 else (16, 8)
        # candidate bytes: addresses and the L4 header, not the checksum field, not the data offset
        cand = list(range(l3 + a0, l3 + a0 + 2 * alen)) + \
            [l3 + l4o + k for k in range(hlen) if k not in (fld, fld + 1) and not (proto == 6 and k == 12)]
        for b in rng.choice(cand, size=int(rng.integers(1, min(12, len(cand)) + 1)), replace=False):
            arena[b] = rng.integers(0, 256)
        want = O.l4_csum(bytes(arena[l3:l3 + int(d["l3_len"])]), int(d["l3_len"]), l4o, f["ver"], proto)
        got = hsum_update(arena, d, rec)
        assert got == want, (f["scenario"], f["ver"], proto, hex(got), hex(want))
        checked += 1
    assert checked > 1500


def test_hsum_update_diverges_when_the_payload_changes():
    """A payload byte changed after receipt: the update carries the old payload's sum, Java's
    recompute does not.  This is why the seam grants F_PRE only to a frame still in place (never
    rebuilt: TcpPacket / UdpPacket.setData and every other rebuild clear the PacketBuffer's
    buffers)."""
    fs = [f for f in H.received(9, 600) if not f["corrupt"] and not f["udp0"]]
    arena, offs, _ = H.layout(fs, 0)
    differ = compared = 0
    for f, off in zip(fs, offs):
        rec = O.hsum_record(f["frame"])
        d = _desc_of(arena, off)
        l3, l4o, L = int(d["l3_off"]), int(d["l4_off"]), int(d["l3_len"])
        if L - l4o - int(rec["hlen"]) < 2:
            continue
        arena[l3 + l4o + int(rec["hlen"])] ^= 0x33
        want = O.l4_csum(bytes(arena[l3:l3 + L]), L, l4o, f["ver"], int(d["l4_proto"]))
        compared += 1
        differ += hsum_update(arena, d, rec) != want
    assert compared > 300 and differ == compared


def test_hsum_update_refuses_a_record_of_another_shape():
    """The kernel's own check: a record whose version, protocol, segment length or header length
    differs from the packet's is refused (nothing written) -- e.g. an MSS option added in place of a
    rebuild, a truncated packet."""
    fs = [f for f in H.received(10, 200) if not f["corrupt"] and not f["udp0"]]
    arena, offs, _ = H.layout(fs, 0)
    for f, off in zip(fs, offs):
        rec = O.hsum_record(f["frame"])
        d = _desc_of(arena, off)
        assert hsum_update(arena, d, rec) is not None
        for field, delta in (("l4_len", 4), ("hlen", 4), ("l3_ver", 2), ("l4_proto", 11)):
            r2 = rec.copy()
            r2[field] = int(r2[field]) + delta
            assert hsum_update(arena, d, r2) is None, field
        r2 = rec.copy()
        r2["l2_len"] = 0
        assert hsum_update(arena, d, r2) is None


@pytest.mark.parametrize("seed", [21, 22])
def test_seam_rule_on_every_scenario(seed):
    """The whole seam on the CPU: each frame is verified (the oracle's recompute stands in for the
    GPU verify), marked by csum-recalc "all", changed by its scenario through the RxPacket setters
    (vswitch.py, the Java setters' byte effects), and deferred by EgressBatch.defer_rx's rule
    (hsum_eligible).  Every frame granted F_PRE gets Java's bytes from the header-sum update; none
    of the rebuilt or replaced frames is granted it; every in-place scenario on a verified frame
    is."""
    from vproxy_amd import vswitch as S
    fs = H.received(seed, 800)
    arena, offs, free = H.layout(fs, 800)
    rng = np.random.default_rng(seed)
    granted = {s: 0 for s in H.SCENARIOS}
    for f, off in zip(fs, offs):
        d = _desc_of(arena, off)
        l3, L, l4o = int(d["l3_off"]), int(d["l3_len"]), int(d["l4_off"])
        proto, ver = int(d["l4_proto"]), int(d["l3_ver"])
        pkt_bytes = bytes(arena[l3:l3 + L])
        st = O.S_DONE
        fld = l3 + l4o + O.L4_FIELD[proto]
        if proto == 17 and _ld16(arena, fld) == 0:
            st |= O.S_UDP_NOCSUM
        elif O.l4_csum(pkt_bytes, L, l4o, ver, proto) == _ld16(arena, fld):
            st |= O.S_L4_OK
        if ver == 4 and O.ipv4_header_csum(pkt_bytes, l4o) == _ld16(arena, l3 + 10):
            st |= O.S_IP_OK
        rx = S.RxPacket(arena, off, st, O.hsum_record(f["frame"]))
        rx.ip_dirty = ver == 4 and not st & O.S_IP_OK          # csum-recalc "all" (recalc_policy)
        rx.l4_dirty = not st & O.S_L4_OK
        H.apply(rx, f, rng, free)
        flags = S.checksum_flags_for(rx.ver == 4, rx.ip_dirty, rx.proto, rx.l4_dirty)
        d2 = S.egress_descriptor(arena[rx.frame_off:rx.frame_off + 512], rx.frame_off, flags)
        ok = bool(flags & O.F_L4) and S.hsum_eligible(
            rx.csum_status, rx.csum_hsum, rx.csum_l3, rx.in_place, int(d2["l3_off"]), int(d2["l3_ver"]),
            int(d2["l4_proto"]), int(d2["l3_len"]), int(d2["l4_off"]), rx.tcp_hlen())
        if f["scenario"] in ("nat_mss_add", "tcp_reset", "payload") and not rx.in_place:
            assert not ok, f["scenario"]
        if not ok:
            continue
        granted[f["scenario"]] += 1
        l3b, Lb, l4b = int(d2["l3_off"]), int(d2["l3_len"]), int(d2["l4_off"])
        got = hsum_update(arena, d2, rx.csum_hsum)
        want = O.l4_csum(bytes(arena[l3b:l3b + Lb]), Lb, l4b, rx.ver, rx.proto)
        assert got == want, f["scenario"]
    for s in ("nat", "nat_mss_clamp", "proxy_syn", "proxy_synack"):
        assert granted[s] > 20, (s, granted)
    assert granted["nat_mss_add"] == granted["payload"] == 0


def test_hsum_eligible_rule_table():
    """Each condition of the rule on its own."""
    from vproxy_amd import vswitch as S
    rec = np.zeros((), O.HSUM_DTYPE)
    rec["sum"], rec["l4_len"], rec["hlen"], rec["l4_proto"], rec["l3_ver"], rec["l2_len"] = 0x1234, 1480, 20, 6, 4, 14
    base = dict(rx_status=O.S_DONE | O.S_IP_OK | O.S_L4_OK, rec=rec, l3_rx=398, in_place=True, l3_now=398, ver=4,
                proto=6, l3_len=1500, l4_off=20, tcp_hlen=20)
    assert S.hsum_eligible(**base)
    for k, v in (("rx_status", O.S_DONE | O.S_IP_OK), ("rx_status", O.S_BAD_DESC | O.S_L4_OK), ("in_place", False),
                 ("l3_now", 402), ("ver", 6), ("proto", 17), ("l3_len", 1504), ("l4_off", 24), ("tcp_hlen", 24)):
        assert not S.hsum_eligible(**{**base, k: v}), k
    r0 = rec.copy()
    r0["l2_len"] = 0
    assert not S.hsum_eligible(**{**base, "rec": r0})
    # the 48-B entry: the record in its first 8 bytes, mask PRE_HSUM
    e = np.frombuffer(S.hsum_entry(rec).tobytes(), np.uint8)
    assert e[36] == O.PRE_HSUM and e[:8].tobytes() == rec.tobytes() and not e[8:36].any() and not e[37:].any()
