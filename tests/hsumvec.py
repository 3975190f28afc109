"""Received frames and the vswitch operations that change them between ingress and egress, for the
ingress-header-sum flush (VPCSUM_PRE_HSUM).  Test infrastructure: tests/ only.

Each scenario is something the reference does to a received TCP / UDP frame after
XDPIface.readable and before XDPIface.sendPacket:

* ``nat``            SwitchUtils.applyNat (SwitchUtils.java:531-542): addresses and ports, in place.
* ``nat_mss_clamp``  applyNat, then SwitchUtils.checkAndUpdateMss on a SYN whose MSS option is above
                     the egress port's maxMss: TcpOption.setData of the 2 MSS bytes, in place
                     (SwitchUtils.java:69-77, TcpPacket.java:561-569).
* ``nat_mss_add``    applyNat, then checkAndUpdateMss on a SYN without an MSS option: the option is
                     added and the TCP packet rebuilt (SwitchUtils.java:83-94; clearRawPacket) --
                     the frame leaves through sendPacket's copying branch from another chunk.
* ``proxy_syn``      SwitchUtils.buildSynPacketForProxyProtocol (:461-465): the sequence number
                     lowered by the PROXY v2 header length, in place, before applyNat.
* ``proxy_synack``   buildSynAckPacketForProxyProtocol (:467-473): seq - 1, ack, flags SYN|ACK, in
                     place, before applyNat.
* ``tcp_reset``      TcpReset (TcpReset.java:45-82): a new RST packet put into the same
                     PacketBuffer (replacePacket), sent from another chunk.
* ``payload``        TcpPacket / UdpPacket.setData with a new payload of the same length: a rebuild
                     (clearRawPacket), sent from another chunk.
* ``ttl``            IPInputRoute's setTtl alone (IP header dirty only; no L4 sum to update).

Frames: IPv4 (IHL 5 and with options) and IPv6 (with and without an extension header), with and
without an 802.1Q tag, TCP SYNs with and without an MSS option and data segments with other
options, UDP; 15% with a payload byte corrupted after their sums were taken (not S_L4_OK) and 5% of
the UDP ones with a stored 0.  Layout: 2048-B umem chunks, frames at chunk + 384 (XDPIface).
"""
from __future__ import annotations

import numpy as np

from oracle import oracle as O

CHUNK, HEADROOM = 2048, 384
SCENARIOS = ("nat", "nat_mss_clamp", "nat_mss_add", "proxy_syn", "proxy_synack", "tcp_reset", "payload", "ttl")
MAX_MSS = 1400          # the egress port's maxMss (baseMTU - overhead - 40)
PP_V2_LEN = 28          # a PROXY protocol v2 header for IPv4 (ProxyProtocolHelper.getV2HeaderLength)
TCP_SYN, TCP_ACK, TCP_RST, TCP_PSH = 0x02, 0x10, 0x04, 0x08


def _put16(b, off, v):
    b[off] = (v >> 8) & 0xFF
    b[off + 1] = v & 0xFF


def _tcp(rng, payload: int, syn: bool, mss: int | None, extra_opts: int) -> bytearray:
    """A TCP segment: 20-B header, an MSS option when `mss`, `extra_opts` NOP words, payload."""
    opts = bytearray()
    if mss is not None:
        opts += bytes([2, 4]) + mss.to_bytes(2, "big")
    opts += bytes([1, 1, 1, 1]) * extra_opts
    h = bytearray(rng.integers(0, 256, 20, dtype=np.uint8).tobytes())
    h[12] = ((20 + len(opts)) // 4) << 4
    h[13] = (TCP_SYN if syn else TCP_ACK | TCP_PSH) | (h[13] & 0x40)
    return h + opts + bytearray(rng.integers(0, 256, payload, dtype=np.uint8).tobytes())


def _udp(rng, payload: int) -> bytearray:
    u = bytearray(rng.integers(0, 256, 8 + payload, dtype=np.uint8).tobytes())
    _put16(u, 4, 8 + payload)
    return u


def _l3(rng, ver: int, seg: bytes, proto: int, ihl: int = 5, ext: int | None = None) -> bytearray:
    if ver == 4:
        hl = ihl * 4
        p = bytearray(rng.integers(0, 256, hl, dtype=np.uint8).tobytes())
        p[0] = 0x40 | ihl
        _put16(p, 2, hl + len(seg))
        p[8] = 64
        p[9] = proto
        return p + seg
    xl = 0 if ext is None else 8 + ext
    p = bytearray(rng.integers(0, 256, 40 + xl, dtype=np.uint8).tobytes())
    p[0] = 0x60
    _put16(p, 4, xl + len(seg))
    p[7] = 64
    if ext is None:
        p[6] = proto
    else:
        p[6], p[40], p[41] = 60, proto, ext
    return p + seg


def ether(rng, l3: bytes, ver: int, vlan: bool) -> bytes:
    et = b"\x08\x00" if ver == 4 else b"\x86\xdd"
    l2 = bytes(rng.integers(0, 256, 12, dtype=np.uint8)) + ((b"\x81\x00\x00\x64" + et) if vlan else et)
    f = l2 + bytes(l3)
    return f + bytes(rng.integers(1, 256, max(60 - len(f), 0), dtype=np.uint8))


def frame_l3(frame: bytes):
    info, err = O.parse_ether(frame)
    assert info is not None, err
    return info


def with_sums(frame: bytes) -> bytes:
    """The frame with correct IPv4 header and L4 sums (what a well-behaved sender put there)."""
    f = bytearray(frame)
    info = frame_l3(f)
    l3 = info.l3_off
    pkt = bytes(f[l3:l3 + info.l3_len])
    if info.ver == 4:
        f[l3 + 10:l3 + 12] = O.ipv4_header_csum(pkt, info.l4_off).to_bytes(2, "big")
        pkt = bytes(f[l3:l3 + info.l3_len])
    fld = O.L4_FIELD[info.proto]
    c = O.l4_csum(pkt, info.l3_len, info.l4_off, info.ver, info.proto)
    f[l3 + info.l4_off + fld:l3 + info.l4_off + fld + 2] = c.to_bytes(2, "big")
    return bytes(f)


def received(seed: int, n: int) -> list[dict]:
    """n received frames, each {frame, ver, proto, scenario, syn, mss, corrupt, udp0}."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        sc = SCENARIOS[i % len(SCENARIOS)]
        ver = 4 if rng.random() < 0.6 else 6
        vlan = rng.random() < 0.25
        ihl = 5 if rng.random() < 0.7 else int(rng.integers(6, 16))
        ext = None if rng.random() < 0.7 else int(rng.integers(0, 5))
        tcp = sc not in ("nat", "payload", "ttl") or rng.random() < 0.6
        syn = sc in ("nat_mss_clamp", "nat_mss_add", "proxy_syn", "proxy_synack") or (tcp and rng.random() < 0.2)
        mss = None
        if tcp and syn and sc != "nat_mss_add":
            mss = int(rng.integers(MAX_MSS + 1, 9000)) if sc == "nat_mss_clamp" or rng.random() < 0.5 \
                else int(rng.integers(500, MAX_MSS + 1))
        payload = int(rng.integers(0, 1200)) if not syn else int(rng.integers(0, 16))
        if tcp:
            seg = _tcp(rng, payload, syn, mss, int(rng.integers(0, 4)) if sc != "nat_mss_clamp" else 0)
        else:
            seg = _udp(rng, int(rng.integers(0, 1200)))
        proto = 6 if tcp else 17
        l3 = _l3(rng, ver, seg, proto, ihl=ihl, ext=ext)
        f = bytearray(with_sums(ether(rng, l3, ver, vlan)))
        info = frame_l3(f)
        corrupt = rng.random() < 0.15 and info.l3_len - info.l4_off > 60
        if corrupt:   # a payload byte changed after the sum was taken: fails verify
            f[info.l3_off + info.l4_off + 60 + int(rng.integers(0, info.l3_len - info.l4_off - 60))] ^= 0x5A
        udp0 = not tcp and rng.random() < 0.05
        if udp0:
            o = info.l3_off + info.l4_off + 6
            f[o:o + 2] = b"\x00\x00"
        out.append(dict(frame=bytes(f), ver=ver, proto=proto, scenario=sc, syn=syn, mss=mss, corrupt=corrupt,
                        udp0=udp0, vlan=vlan))
    return out


def layout(fs: list[dict], spare: int) -> tuple[np.ndarray, list[int], list[int]]:
    """(arena, frame offsets, offsets of `spare` free chunks for rebuilt frames)."""
    arena = np.zeros(CHUNK * (len(fs) + spare), np.uint8)
    offs = []
    for i, f in enumerate(fs):
        o = i * CHUNK + HEADROOM
        arena[o:o + len(f["frame"])] = np.frombuffer(f["frame"], np.uint8)
        offs.append(o)
    free = [(len(fs) + k) * CHUNK + HEADROOM for k in range(spare)]
    return arena, offs, free


def _tcp_opt_offset(arena, l4: int, kind: int) -> int | None:
    """Offset (from the TCP header) of the first option of `kind` (TcpPacket.from's walk)."""
    doff = (int(arena[l4 + 12]) >> 4) * 4
    o = 20
    while o < doff:
        k = int(arena[l4 + o])
        if k == 0:
            return None
        if k == 1:
            o += 1
            continue
        if k == kind:
            return o
        o += max(int(arena[l4 + o + 1]), 2)
    return None


def rebuilt_with_mss(frame: bytes, mss: int) -> bytes:
    """checkAndUpdateMss's rebuild (SwitchUtils.java:83-94): the TCP options with an MSS option
    appended, data offset and IP length grown by 4; the sums are left for the egress recompute."""
    f = bytearray(frame)
    info = frame_l3(f)
    l3, l4 = info.l3_off, info.l3_off + info.l4_off
    doff = (f[l4 + 12] >> 4) * 4
    opt = bytes([2, 4]) + mss.to_bytes(2, "big")
    g = f[:l4 + doff] + opt + f[l4 + doff:l3 + info.l3_len]
    g[l4 + 12] = (g[l4 + 12] & 0x0F) | (((doff + 4) // 4) << 4)
    if info.ver == 4:
        _put16(g, l3 + 2, info.l3_len + 4)
    else:
        _put16(g, l3 + 4, info.l3_len + 4 - 40)
    return bytes(g)


def reset_for(frame: bytes) -> bytes:
    """TcpReset's answer to a TCP frame (TcpReset.java:45-82): addresses and ports swapped, seq =
    the received ack, ack = seq + 1, flags RST | ACK, no options, no payload, a fresh IP header."""
    f = bytearray(frame)
    info = frame_l3(f)
    l3, l4 = info.l3_off, info.l3_off + info.l4_off
    l2 = bytes(f[6:12]) + bytes(f[0:6]) + bytes(f[12:l3])
    if info.ver == 4:
        ip = bytearray(20)
        ip[0], ip[8], ip[9] = 0x45, 64, 6
        _put16(ip, 2, 40)
        ip[12:16], ip[16:20] = f[l3 + 16:l3 + 20], f[l3 + 12:l3 + 16]
    else:
        ip = bytearray(40)
        ip[0], ip[6], ip[7] = 0x60, 6, 64
        _put16(ip, 4, 20)
        ip[8:24], ip[24:40] = f[l3 + 24:l3 + 40], f[l3 + 8:l3 + 24]
    seq = int.from_bytes(f[l4 + 4:l4 + 8], "big")
    tcp = bytearray(20)
    tcp[0:2], tcp[2:4] = f[l4 + 2:l4 + 4], f[l4:l4 + 2]
    tcp[4:8] = f[l4 + 8:l4 + 12]
    tcp[8:12] = ((seq + 1) & 0xFFFFFFFF).to_bytes(4, "big")
    tcp[12], tcp[13] = 0x50, TCP_RST | TCP_ACK
    return l2 + bytes(ip) + bytes(tcp)


def apply(pkt, sc: dict, rng, free: list[int]):
    """Run scenario sc["scenario"] on RxPacket pkt (vproxy_amd.vswitch.RxPacket) the way the
    reference's code does it.  `free` hands out spare chunks for rebuilt frames."""
    s = sc["scenario"]
    a = pkt.arena

    def nat():
        alen = 4 if pkt.ver == 4 else 16
        pkt.set_src(bytes(rng.integers(0, 256, alen, dtype=np.uint8)))
        pkt.set_dst(bytes(rng.integers(0, 256, alen, dtype=np.uint8)))
        pkt.set_ports(int(rng.integers(0, 65536)), int(rng.integers(0, 65536)))

    if s == "ttl":
        pkt.set_ttl(int(rng.integers(2, 255)))
        return
    if s == "payload":
        info = frame_l3(bytes(a[pkt.frame_off:pkt.frame_off + 1600]))
        f = bytearray(a[pkt.frame_off:pkt.frame_off + info.l3_off + info.l3_len])
        hl = (f[info.l3_off + info.l4_off + 12] >> 4) * 4 if pkt.proto == 6 else 8
        body = info.l3_off + info.l4_off + hl
        f[body:] = rng.integers(0, 256, len(f) - body, dtype=np.uint8).tobytes()
        pkt.rebuild(free.pop(), bytes(f))
        return
    if s == "tcp_reset":
        if pkt.proto == 6:
            pkt.replace(free.pop(), reset_for(bytes(a[pkt.frame_off:pkt.frame_off + 1600])))
        else:
            nat()
        return
    if s == "proxy_syn" and pkt.proto == 6:
        seq = int.from_bytes(bytes(a[pkt.l4 + 4:pkt.l4 + 8]), "big")
        pkt.set_seq(seq - PP_V2_LEN)
    if s == "proxy_synack" and pkt.proto == 6:
        seq = int.from_bytes(bytes(a[pkt.l4 + 4:pkt.l4 + 8]), "big")
        ack = int.from_bytes(bytes(a[pkt.l4 + 8:pkt.l4 + 12]), "big")
        pkt.set_seq(seq - 1)
        pkt.set_ack(ack)
        pkt.set_tcp_flags(TCP_SYN | TCP_ACK)
    nat()
    if s in ("nat_mss_clamp", "nat_mss_add") and pkt.proto == 6:
        o = _tcp_opt_offset(a, pkt.l4, 2)
        if o is not None:
            if int.from_bytes(bytes(a[pkt.l4 + o + 2:pkt.l4 + o + 4]), "big") > MAX_MSS:
                pkt.set_option_data(o, MAX_MSS.to_bytes(2, "big"))
        else:
            info = frame_l3(bytes(a[pkt.frame_off:pkt.frame_off + 1600]))
            f = bytes(a[pkt.frame_off:pkt.frame_off + info.l3_off + info.l3_len])
            pkt.rebuild(free.pop(), rebuilt_with_mss(f, MAX_MSS))
