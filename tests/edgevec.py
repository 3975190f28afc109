"""Crafted edge vectors for the checksum path (test infrastructure: tests/ only).

Every vector is built so that the edge it targets is hit by construction, not by chance:

* L4 result 0x0000 -- one payload word is set to the one's-complement of the rest of the sum,
  so Java's intermediate sum (Utils.java:783-797) is exactly 0xffff and DoFinal gives 0
  (Utils.java:799-801).  For UDP the reference then stores 0xffff (UdpPacket.java:87-89,
  111-113, 142-144, 157-159); TCP (TcpPacket.java:475-485, 508-518) and ICMP / ICMPv6
  (IcmpPacket.java:64-74, 124-135) keep 0x0000.
* IPv4 header result 0x0000 -- the identification word is set the same way
  (Ipv4Packet.java:209-217).
* ICMPv4 carried in IPv6 -- next header 1: Ipv6Packet.__updateChildrenChecksum falls through to
  packet.updateChecksum() (Ipv6Packet.java:232-234), the v4 ICMP sum without a pseudo header.
* IPv6 with one extension header -- l4_off = 40 + 8 + hdrExtLen (the reference's ExtHeader rule,
  Ipv6Packet.java ExtHeader.from), so l4_off may be odd; the pseudo-header length is the L4
  length without the extension header (Ipv6Packet.java:184-242).
* UDP with stored checksum 0 (RFC 768 "no checksum"): verify reports UDP_NOCSUM.

Each packet's expected values are pinned twice: by the C oracle and by the pure-Python
restatement in oracle/oracle.py, which the builder checks before returning.
"""
from __future__ import annotations

import numpy as np

from oracle import oracle as O

V6_EXT_TYPES = (0, 60, 43, 44)   # hop-by-hop, destination options, routing, fragment


def _put16(buf, off, v):
    buf[off] = (v >> 8) & 0xFF
    buf[off + 1] = v & 0xFF


def _l4_adjust_off(proto: int) -> int:
    # an even L4 offset that is neither the checksum field nor a length the parse depends on:
    # TCP / UDP source port, ICMP identifier
    return 0 if proto in (6, 17) else 4


def l4_value(l3: bytes, l3_len: int, l4_off: int, ver: int, proto: int) -> int:
    """Pure-Python Java L4 checksum (UdpPacket's 0 -> 0xffff included)."""
    return O.l4_csum(l3, l3_len, l4_off, ver, proto)


def force_l4_zero(pkt: bytearray, l3_len: int, l4_off: int, ver: int, proto: int):
    """Rewrite one L4 word so that Java's DoFinal of the L4 sum is 0."""
    a = l4_off + _l4_adjust_off(proto)
    _put16(pkt, a, 0)
    c = l4_value(bytes(pkt), l3_len, l4_off, ver, proto)
    if proto == 17 and c == 0xFFFF:
        c = 0          # the substituted value: the true sum was already 0xffff
    _put16(pkt, a, c)  # s + (0xffff - s) = 0xffff, no carry: DoFinal 0


def force_ip_zero(pkt: bytearray, ihl_bytes: int):
    _put16(pkt, 4, 0)
    c = O.ipv4_header_csum(bytes(pkt), ihl_bytes)
    _put16(pkt, 4, c)


def _v4(rng, proto: int, l4len: int, ihl: int = 5) -> tuple[bytearray, int]:
    hl = ihl * 4
    total = hl + l4len
    p = bytearray(rng.integers(0, 256, total, dtype=np.uint8).tobytes())
    p[0] = 0x40 | ihl
    _put16(p, 2, total)
    p[9] = proto
    _put16(p, 10, 0)
    if proto == 6:
        p[hl + 12] = 0x50
    elif proto == 17:
        _put16(p, hl + 4, l4len)
    return p, hl


def _v6(rng, proto: int, l4len: int, ext: int | None = None, ext_type: int = 0) -> tuple[bytearray, int]:
    xl = 0 if ext is None else 8 + ext
    total = 40 + xl + l4len
    p = bytearray(rng.integers(0, 256, total, dtype=np.uint8).tobytes())
    p[0] = 0x60
    _put16(p, 4, total - 40)
    if ext is None:
        p[6] = proto
    else:
        p[6] = ext_type
        p[40] = proto
        p[41] = ext
    l4 = 40 + xl
    if proto == 6:
        p[l4 + 12] = 0x50
    elif proto == 17:
        _put16(p, l4 + 4, l4len)
    return p, l4


def edge_packets(rng, big: bool = True) -> list[dict]:
    """The edge packets as dicts {bytes, l3_len, l4_off, ver, proto, flags, kind, want_ip, want_l4}.
    want_* is the pinned Java value (None: not pinned beyond the oracle)."""
    lens = [8, 9, 10, 31, 44, 63, 64, 65, 556, 1480] + ([4000, 8960] if big else [])
    pk = []

    def add(p, l4_off, ver, proto, kind, want_ip=None, want_l4=None, flags=None):
        if flags is None:
            flags = (O.F_IP if ver == 4 else 0) | O.F_L4
        pk.append(dict(bytes=bytes(p), l3_len=len(p), l4_off=l4_off, ver=ver, proto=proto, flags=flags,
                       kind=kind, want_ip=want_ip, want_l4=want_l4))

    for L in lens:
        for proto in (17, 6, 1):
            minl4 = 20 if proto == 6 else 8
            l4len = max(L, minl4)
            # IPv4, L4 forced to 0 (UDP -> 0xffff); also with IPv4 options
            for ihl in (5, 7):
                p, hl = _v4(rng, proto, l4len, ihl)
                force_l4_zero(p, len(p), hl, 4, proto)
                force_ip_zero(p, hl)
                add(p, hl, 4, proto, f"v4_{proto}_zero", want_ip=0, want_l4=0xFFFF if proto == 17 else 0)
            # IPv6, L4 forced to 0 (ICMP -> ICMPv6 with its pseudo header)
            p6 = {17: 17, 6: 6, 1: 58}[proto]
            p, l4 = _v6(rng, p6, l4len)
            force_l4_zero(p, len(p), l4, 6, p6)
            add(p, l4, 6, p6, f"v6_{p6}_zero", want_l4=0xFFFF if p6 == 17 else 0)
            # ICMPv4 in IPv6: the sum is the segment's alone
            if proto == 1:
                p, l4 = _v6(rng, 1, l4len)
                seg = bytearray(p[l4:])
                seg[2:4] = b"\x00\x00"
                add(p, l4, 6, 1, "icmp_in_v6", want_l4=O.csum(bytes(seg)))
                p, l4 = _v6(rng, 1, l4len)
                force_l4_zero(p, len(p), l4, 6, 1)
                add(p, l4, 6, 1, "icmp_in_v6_zero", want_l4=0)
    # IPv6 with one extension header: hdrExtLen odd and even, every L4 kind
    for h in (0, 1, 2, 3, 5, 6, 8, 13, 17, 40, 255):
        for proto in (6, 17, 58, 1):
            L = int(rng.choice(lens))
            l4len = max(L, 20 if proto == 6 else 8)
            p, l4 = _v6(rng, proto, l4len, ext=h, ext_type=V6_EXT_TYPES[h % 4])
            add(p, l4, 6, proto, "v6_ext")
            p, l4 = _v6(rng, proto, l4len, ext=h, ext_type=V6_EXT_TYPES[(h + 1) % 4])
            force_l4_zero(p, len(p), l4, 6, proto)
            add(p, l4, 6, proto, "v6_ext_zero", want_l4=0xFFFF if proto == 17 else 0)
    # UDP with stored 0: verify says UDP_NOCSUM (sum computed normally)
    for ver in (4, 6):
        p, l4 = _v4(rng, 17, 100) if ver == 4 else _v6(rng, 17, 100)
        add(p, l4, ver, 17, "udp_nocsum")
    return pk


def pack(packets: list[dict], pad: int, stride: int | None = None, fill=None):
    """Lay the packets out one per frame (L3 at frame + pad) and build descriptors.  Frames hold
    the packets with their checksum fields already set to the Java values ("valid input"), except
    kind udp_nocsum, whose UDP field is 0."""
    stride = stride or ((pad + max(len(p["bytes"]) for p in packets) + 64 + 63) // 64) * 64
    arena = np.zeros(stride * len(packets), np.uint8) if fill is None else fill(stride * len(packets))
    desc = np.zeros(len(packets), O.DESC_DTYPE)
    for i, p in enumerate(packets):
        b = bytearray(p["bytes"])
        fld = p["l4_off"] + O.L4_FIELD[p["proto"]]
        if p["ver"] == 4:
            _put16(b, 10, O.ipv4_header_csum(bytes(b), p["l4_off"]))
        _put16(b, fld, 0 if p["kind"] == "udp_nocsum" else
               l4_value(bytes(b), p["l3_len"], p["l4_off"], p["ver"], p["proto"]))
        base = i * stride + pad
        arena[base:base + len(b)] = np.frombuffer(bytes(b), np.uint8)
        desc[i] = (base, p["l3_len"], p["l4_off"], p["ver"], p["proto"], p["flags"], 0)
    return arena, desc


def check_pins(packets: list[dict]):
    """The constructions above hit their edges (pure-Python restatement)."""
    for p in packets:
        b = p["bytes"]
        if p["want_ip"] is not None:
            assert O.ipv4_header_csum(b, p["l4_off"]) == p["want_ip"], p["kind"]
        if p["want_l4"] is not None:
            assert l4_value(b, p["l3_len"], p["l4_off"], p["ver"], p["proto"]) == p["want_l4"], p["kind"]


def ether_frames(packets: list[dict]) -> list[bytes]:
    """The packets behind a 14-B Ethernet header, checksum fields set (as pack())."""
    out = []
    for p in packets:
        a, d = pack([p], 0, stride=len(p["bytes"]) + 64)
        eth = bytes(12) + (b"\x08\x00" if p["ver"] == 4 else b"\x86\xdd")
        out.append(eth + a[:len(p["bytes"])].tobytes())
    return out


def parse_cases() -> list[tuple[bytes, bool, str]]:
    """Ethernet frames at the edges of the reference's parse rules, each with whether vproxy's
    vswitch accepts it as an IP packet (EthernetPacket.from(raw, allowPartial=true)):
    (frame, accepted, reason)."""
    rng = np.random.default_rng(77)
    eth4, eth6 = bytes(12) + b"\x08\x00", bytes(12) + b"\x86\xdd"
    cases = []

    def v4(proto, l4: bytes, nibble=4, ihl=5):
        p, hl = _v4(rng, proto, len(l4), ihl)
        p[0] = (nibble << 4) | ihl
        p[hl:] = l4
        return bytes(p)

    def v6(proto, l4: bytes, ext=None, nibble=6, ext_type=0):
        p, o = _v6(rng, proto, len(l4), ext=ext, ext_type=ext_type)
        p[0] = nibble << 4
        p[o:] = l4
        return bytes(p)

    def tcp(n, doff=5, opts=b""):
        b = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        if n > 12:
            b[12] = doff << 4
        b[20:20 + len(opts)] = opts
        return bytes(b[:n])

    def udp(n, length=None):
        b = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        if n >= 6:
            _put16(b, 4, n if length is None else length)
        return bytes(b)

    rnd = lambda n: rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    # Ipv4Packet.initPartial: the EtherType decides, the version nibble is not read (:29-63)
    cases.append((eth4 + v4(6, tcp(40), nibble=6), True, "ipv4 ethertype, version nibble 6"))
    cases.append((eth4 + v4(6, tcp(40), nibble=0), True, "ipv4 ethertype, version nibble 0"))
    # TcpPacket.initPartial >= 20 B (TcpPacket.java:187-199)
    for n, ok in ((18, False), (19, False), (20, True), (21, True)):
        cases.append((eth4 + v4(6, tcp(n)), ok, f"ipv4 tcp {n} B"))
        cases.append((eth6 + v6(6, tcp(n)), ok, f"ipv6 tcp {n} B"))
    # UdpPacket.initPartial >= 8 B, the length field is not read (UdpPacket.java:17-27)
    for n, ok in ((7, False), (8, True), (30, True)):
        cases.append((eth4 + v4(17, udp(n)), ok, f"ipv4 udp {n} B"))
    cases.append((eth4 + v4(17, udp(30, length=31)), True, "ipv4 udp length field != buffer (partial)"))
    cases.append((eth6 + v6(17, udp(30, length=29)), True, "ipv6 udp length field != buffer (partial)"))
    # IcmpPacket.initPartial reads byte 0 (IcmpPacket.java:22-26): 0 B throws
    for n, ok in ((0, False), (1, True), (3, True), (8, True)):
        cases.append((eth4 + v4(1, rnd(n)), ok, f"ipv4 icmp {n} B"))
    cases.append((eth6 + v6(58, rnd(1)), True, "ipv6 icmpv6 1 B"))
    cases.append((eth6 + v6(1, rnd(2)), True, "ipv6 icmpv4 2 B"))
    # ICMPv6 number inside IPv4 is PacketBytes: accepted, no L4 sum
    cases.append((eth4 + v4(58, rnd(0)), True, "ipv4 proto 58 (PacketBytes)"))
    # Ipv6Packet.initPartial: no version check without extension headers (:26-59)
    cases.append((eth6 + v6(6, tcp(20), nibble=4), True, "ipv6 ethertype, version nibble 4"))
    # with an extension header the full Ipv6Packet.from runs: version, then the L4 from()
    cases.append((eth6 + v6(6, tcp(20), ext=0, nibble=4), False, "ipv6 ext, version nibble 4"))
    cases.append((eth6 + v6(17, udp(30, length=31), ext=2), False, "ipv6 ext, udp length != buffer"))
    cases.append((eth6 + v6(17, udp(30), ext=2), True, "ipv6 ext, udp length == buffer"))
    cases.append((eth6 + v6(17, udp(7), ext=2), False, "ipv6 ext, udp 7 B"))
    for n, ok in ((7, False), (8, True)):
        cases.append((eth6 + v6(58, rnd(n), ext=1), ok, f"ipv6 ext, icmpv6 {n} B"))
        cases.append((eth6 + v6(1, rnd(n), ext=1), ok, f"ipv6 ext, icmpv4 {n} B"))
    # TcpPacket.from: dataOffset and the option walk (TcpPacket.java:223-287, :602-640)
    good_opts = bytes([2, 4, 5, 0xB4, 1, 3, 3, 7, 1, 1, 0, 0])        # MSS, NOP, WS, NOP NOP END
    for opts, doff, ok, why in (
            (good_opts, 8, True, "mss nop ws nop nop end"),
            (bytes([1] * 8), 7, True, "nops"),
            (bytes([8, 10]) + bytes(8) + bytes([1, 1]), 8, True, "timestamps + nops"),
            (bytes([2, 3, 0, 1]), 6, False, "mss length 3"),
            (bytes([3, 4, 0, 0]), 6, False, "window scale length 4"),
            (bytes([5, 0, 0, 0]), 6, False, "option length 0 (reference loops)"),
            (bytes([5, 1, 0, 0]), 6, False, "option length 1 (reference throws)"),
            (bytes([5, 9, 0, 0]), 6, False, "option past dataOffset"),
            (bytes([1, 1, 1, 5]), 6, False, "option kind on the last byte"),
            (bytes([0, 9, 9, 9]), 6, True, "end then garbage")):
        cases.append((eth6 + v6(6, tcp(40, doff, opts), ext=3), ok, f"ipv6 ext, tcp options: {why}"))
        cases.append((eth6 + v6(6, tcp(40, doff, opts)), True, f"ipv6 tcp options not parsed (partial): {why}"))
    cases.append((eth6 + v6(6, tcp(24, 7), ext=0), False, "ipv6 ext, tcp dataOffset > length"))
    cases.append((eth6 + v6(6, tcp(24, 2), ext=0), True, "ipv6 ext, tcp dataOffset < 20"))
    # IPv6_NEXT_HEADER_NO_NEXT_HEADER behind an extension header
    cases.append((eth6 + v6(59, b"", ext=4), True, "ipv6 ext, no next header, empty"))
    cases.append((eth6 + v6(59, rnd(4), ext=4), False, "ipv6 ext, no next header, 4 B"))
    cases.append((eth6 + v6(59, rnd(4)), True, "ipv6 no next header, 4 B (partial: PacketBytes)"))
    # extension header length and chains
    p = bytearray(v6(6, tcp(20), ext=8))
    _put16(p, 4, 40 + 8 + 8 - 40 + 3)      # payload ends inside the extension header
    cases.append((eth6 + bytes(p[:40 + 8 + 3]), False, "ipv6 ext header truncated"))
    p = bytearray(v6(17, udp(8), ext=0))
    p[40] = 60                              # a second extension header
    cases.append((eth6 + bytes(p), False, "ipv6 two ext headers (reference loops)"))
    # EtherIP (EtherIPPacket.java:32-48): >= 2 B and an inner Ethernet header; inner ARP checked
    inner_arp = bytes(12) + b"\x08\x06" + bytes([0, 1, 8, 0, 6, 4, 0, 1]) + rnd(20)
    for l4, ok, why in ((rnd(1), False, "1 B"), (bytes(2) + rnd(13), False, "inner frame 13 B"),
                        (bytes(2) + bytes(12) + b"\x81\x00" + rnd(2), False, "inner vlan 16 B"),
                        (bytes(2) + inner_arp, True, "inner arp"),
                        (bytes(2) + inner_arp[:30], False, "inner arp truncated"),
                        (bytes(2) + bytes(12) + b"\x08\x00" + rnd(10), True, "inner ipv4 garbage")):
        cases.append((eth4 + v4(97, l4), ok, f"etherip {why}"))
    # L3 header rules, IPv4 (Ipv4Packet.initPartial, Ipv4Packet.java:29-63): the buffer, IHL and
    # totalLength; a shorter totalLength cuts the Ethernet padding off
    p4 = v4(6, tcp(20))
    cases.append((eth4 + p4[:19], False, "ipv4 19 B"))
    for ihl, ok in ((4, False), (0, False), (6, True)):
        q = bytearray(v4(6, tcp(40)))
        q[0] = 0x40 | ihl
        cases.append((eth4 + bytes(q), ok, f"ipv4 ihl {ihl} (tcp at 4*ihl)"))
    q = bytearray(v4(6, tcp(40)))
    q[0] = 0x4F                                 # 60-B header in a 60-B packet: no room for TCP
    _put16(q, 2, 60)
    cases.append((eth4 + bytes(q), False, "ipv4 ihl 15, totalLength 60"))
    q = bytearray(p4)
    q[0] = 0x4F
    _put16(q, 2, 40)
    cases.append((eth4 + bytes(q), False, "ipv4 ihl 15 > 40-B buffer"))
    for total, ok, why in ((24, False, "totalLength < 4*ihl + tcp"), (19, False, "totalLength < 4*ihl"),
                           (41, False, "totalLength > buffer"), (40, True, "totalLength == buffer")):
        q = bytearray(p4)
        _put16(q, 2, total)
        cases.append((eth4 + bytes(q), ok, f"ipv4 {why}"))
    cases.append((eth4 + p4 + rnd(6), True, "ipv4 + 6 B ethernet padding"))
    cases.append((eth4 + v4(17, udp(8)) + bytes(18), True, "ipv4 udp 8 B + 18 B padding"))
    # IPv6 (Ipv6Packet.initPartial, Ipv6Packet.java:26-59): payloadLength 0 is a jumbogram,
    # refused; a payload past the buffer refused; padding cut
    p6 = v6(6, tcp(20))
    cases.append((eth6 + p6[:39], False, "ipv6 39 B"))
    for pl, ok, why in ((0, False, "payloadLength 0 (jumbo)"), (21, False, "payloadLength > buffer"),
                        (19, False, "payloadLength < tcp header")):
        q = bytearray(p6)
        _put16(q, 4, pl)
        cases.append((eth6 + bytes(q), ok, f"ipv6 {why}"))
    cases.append((eth6 + p6 + rnd(4), True, "ipv6 + 4 B padding"))
    q = bytearray(v6(17, udp(30), ext=2))
    _put16(q, 4, 0)
    cases.append((eth6 + bytes(q), False, "ipv6 ext, payloadLength 0 (jumbo)"))
    # L2: Ethernet / 802.1Q lengths, non-IP types
    cases.append((eth4[:13], False, "ethernet 13 B"))
    cases.append((bytes(12) + b"\x81\x00" + b"\x00\x05", False, "802.1q 16 B"))
    cases.append((bytes(12) + b"\x81\x00\x00\x05\x08\x00" + v4(6, tcp(20)), True, "802.1q ipv4"))
    cases.append((bytes(12) + b"\x08\x06" + inner_arp[14:], False, "arp"))
    return cases
