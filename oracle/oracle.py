"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the vswitch checksum path.

Two restatements of vproxy's Java checksum code, used only by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg:

* :func:`csum_intermediate` / :func:`csum` ... pure-Python, line-by-line restatement of
  ``Utils.calculateChecksumIntermediate`` / ``calculateChecksumDoFinal``
  (base/src/main/java/io/vproxy/base/util/Utils.java:778-801) for the small known-answer cases.
* :class:`Oracle` ... ctypes binding of ``oracle/csum_oracle.c`` (same algorithm in C) for
  batches and for the timed CPU baseline.
* :func:`parse_ether` / :func:`parse_l3` ... restatement of the parse rules that decide the
  checksum inputs (EthernetPacket.from, EthernetPacket.java:25-94; Ipv4Packet.from,
  Ipv4Packet.java:73-145; Ipv6Packet.from, Ipv6Packet.java:69-159) producing descriptors, and
  :func:`flow_tuple`, the conntrack key the L4 input nodes read (TcpInput.java:47-51,
  UdpInput.java:45-47).

Parity pin: tests/test_oracle_golden.py checks this module against every TestPacket.java
known-answer vector and the reference's pcap fixtures (tests/golden/).
The product (``vproxy_amd``) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liborc.so")

F_IP, F_L4, F_RAW, F_L4P, F_PRE = 0x01, 0x02, 0x04, 0x08, 0x10   # F_PRE: Java recomputes in full
S_IP_OK, S_L4_OK, S_UDP_NOCSUM, S_DONE, S_BAD_DESC = 0x01, 0x02, 0x04, 0x40, 0x80
S_TTL_EXPIRED = 0x20
MODE_COMPUTE, MODE_VERIFY, MODE_WRITE = 0x00, 0x01, 0x10
NAT_SRC, NAT_DST, NAT_SPORT, NAT_DPORT, NAT_DEC_TTL, NAT_SET_TTL = 0x01, 0x02, 0x04, 0x08, 0x10, 0x20

DESC_DTYPE = np.dtype([("l3_off", "<u8"), ("l3_len", "<u2"), ("l4_off", "<u2"), ("l3_ver", "u1"),
                       ("l4_proto", "u1"), ("flags", "u1"), ("rsv", "u1")])
NAT4_DTYPE = np.dtype([("src", "u1", 4), ("dst", "u1", 4), ("sport", "u1", 2), ("dport", "u1", 2),
                       ("mask", "u1"), ("rsv", "u1", 3)])
NAT_DTYPE = np.dtype([("src", "u1", 16), ("dst", "u1", 16), ("sport", "u1", 2), ("dport", "u1", 2),
                      ("mask", "u1"), ("ttl", "u1"), ("rsv", "u1", 10)])
# vpcsum_hsum_t: the ingress header sum of a received TCP / UDP frame (include/vpcsum.h)
HSUM_DTYPE = np.dtype([("sum", "<u2"), ("l4_len", "<u2"), ("hlen", "u1"), ("l4_proto", "u1"), ("l3_ver", "u1"),
                       ("l2_len", "u1")])
PRE_HSUM = 0x80   # VPCSUM_PRE_HSUM: a pre-image entry holding a vpcsum_hsum_t
assert DESC_DTYPE.itemsize == 16 and NAT4_DTYPE.itemsize == 16 and NAT_DTYPE.itemsize == 48
assert HSUM_DTYPE.itemsize == 8

# Consts.java:24-31
IP_PROTOCOL_ICMP, IP_PROTOCOL_TCP, IP_PROTOCOL_UDP, IP_PROTOCOL_ICMPv6 = 1, 6, 17, 58
IPv6_needs_next_header = {0, 60, 43, 44, 51, 50, 135, 139, 140, 253, 254}
ETHER_TYPE_IPv4, ETHER_TYPE_IPv6, ETHER_TYPE_8021Q = 0x0800, 0x86DD, 0x8100


# ----------------------------------------------------------------------------------------
# Pure-Python restatement (Utils.java:778-801)
# ----------------------------------------------------------------------------------------
def csum_intermediate(s: int, a: bytes, limit: int) -> int:
    """Utils.calculateChecksumIntermediate, Utils.java:783-797."""
    for i in range(limit // 2):
        s += (a[i * 2] << 8) | a[i * 2 + 1]
        while s > 0xFFFF:
            s = (s & 0xFFFF) + 1
    if limit % 2 != 0:
        s += a[limit - 1] << 8
        while s > 0xFFFF:
            s = (s & 0xFFFF) + 1
    return s


def csum_final(s: int) -> int:
    """Utils.calculateChecksumDoFinal, Utils.java:799-801."""
    return 0xFFFF - s


def csum(a: bytes, limit: int | None = None) -> int:
    """Utils.calculateChecksum, Utils.java:778-781."""
    return csum_final(csum_intermediate(0, a, len(a) if limit is None else limit))


def pseudo_ipv4(l3: bytes, proto: int, upper_len: int) -> bytes:
    """Utils.buildPseudoIPv4Header, Utils.java:758-766."""
    return bytes(l3[12:16]) + bytes(l3[16:20]) + bytes([0, proto]) + (upper_len & 0xFFFF).to_bytes(2, "big")


def pseudo_ipv6(l3: bytes, proto: int, upper_len: int) -> bytes:
    """Utils.buildPseudoIPv6Header, Utils.java:768-776."""
    return bytes(l3[8:24]) + bytes(l3[24:40]) + (upper_len & 0xFFFFFFFF).to_bytes(4, "big") + bytes([0, 0, 0, proto])


L4_FIELD = {IP_PROTOCOL_TCP: 16, IP_PROTOCOL_UDP: 6, IP_PROTOCOL_ICMP: 2, IP_PROTOCOL_ICMPv6: 2}


def ipv4_header_csum(l3: bytes, ihl_bytes: int) -> int:
    """Ipv4Packet.__updateChecksum, Ipv4Packet.java:209-217."""
    b = bytearray(l3[:ihl_bytes])
    b[10:12] = b"\x00\x00"
    return csum(bytes(b), ihl_bytes)


def l4_csum(l3: bytes, l3_len: int, l4_off: int, ver: int, proto: int) -> int:
    """TcpPacket/UdpPacket/IcmpPacket checksum update (TcpPacket.java:475-518,
    UdpPacket.java:136-164, IcmpPacket.java:64-74,124-135)."""
    fld = L4_FIELD[proto]
    seg = bytearray(l3[l4_off:l3_len])
    seg[fld:fld + 2] = b"\x00\x00"
    if proto == IP_PROTOCOL_ICMP:
        c = csum(bytes(seg))
    else:
        ph = pseudo_ipv4(l3, proto, len(seg)) if ver == 4 else pseudo_ipv6(l3, proto, len(seg))
        c = csum(ph + bytes(seg))
    if proto == IP_PROTOCOL_UDP and c == 0:
        c = 0xFFFF
    return c


# ----------------------------------------------------------------------------------------
# Parse rules (what bytes a checksum covers)
# ----------------------------------------------------------------------------------------
@dataclass
class L3Info:
    l3_off: int      # offset of L3 inside the given buffer
    l3_len: int      # totalLength / 40+payloadLength
    l4_off: int      # relative to l3_off
    ver: int
    proto: int


IP_PROTOCOL_ETHERIP, IPv6_NO_NEXT_HEADER = 97, 59            # Consts.java:29-30
ETHER_TYPE_ARP = 0x0806
TCP_OPTION_END, TCP_OPTION_NOP, TCP_OPTION_MSS, TCP_OPTION_WINDOW_SCALE = 0, 1, 2, 3


def _u16(b, o):
    return (b[o] << 8) | b[o + 1]


def _arp_from(b: bytes) -> str | None:
    """ArpPacket.from (ArpPacket.java:22-70): the length checks (extra bytes are cut, not refused)."""
    if len(b) < 8:
        return "input packet length too short for an arp packet"
    hs, ps = b[4], b[5]
    if len(b) < 8 + 2 * (hs + ps):
        return "input packet length too short for an arp packet"
    return None


def _etherip(b: bytes) -> str | None:
    """EtherIPPacket.initPartial / from (EtherIPPacket.java:32-71): >= 2 B, then the inner
    Ethernet frame.  Its own errors propagate; an inner IP packet that fails to parse is kept as
    PacketBytes (EthernetPacket.java:60-64), an inner ARP that fails does propagate."""
    if len(b) < 2:
        return "input packet length too short for an etherip packet"
    inner = b[2:]
    if len(inner) < 14:
        return "input packet length too short for a ethernet packet"
    typ, hl = _u16(inner, 12), 14
    if typ == ETHER_TYPE_8021Q:
        if len(inner) < 18:
            return "input packet length too short for 802.1q ethernet packet"
        typ, hl = _u16(inner, 16), 18
    if typ == ETHER_TYPE_ARP:
        return _arp_from(inner[hl:])
    return None


def _l4_init_partial(ver: int, proto: int, seg: bytes) -> str | None:
    """Ipv4/Ipv6Packet.initUpperLayerPacket(.., raw) (Ipv4Packet.java:146-163, Ipv6Packet.java:
    161-180) -> the L4 PartialPacket.initPartial: TcpPacket.java:187-199 (>= 20 B),
    UdpPacket.java:17-27 (>= 8 B), IcmpPacket.java:22-26 (reads byte 0: a 0-byte ICMP message
    throws in the reference -- refused here), EtherIPPacket.java:32-48."""
    if proto == IP_PROTOCOL_TCP:
        return "input packet length too short for a tcp packet" if len(seg) < 20 else None
    if proto == IP_PROTOCOL_UDP:
        return "input packet length too short for an udp packet" if len(seg) < 8 else None
    if proto == IP_PROTOCOL_ICMP or (ver == 6 and proto == IP_PROTOCOL_ICMPv6):
        return "icmp packet with no bytes (IndexOutOfBounds in the reference)" if len(seg) < 1 else None
    if proto == IP_PROTOCOL_ETHERIP:
        return _etherip(seg)
    return None   # PacketBytes


def _tcp_from(seg: bytes) -> str | None:
    """TcpPacket.from (TcpPacket.java:223-287) incl. the option walk and TcpOption.from/check
    (:602-640).  An option of length 0 re-reads itself forever in the reference and one of
    length 1 throws (bytes.uint8(1) of a 1-byte view): both refused."""
    if len(seg) < 20:
        return "input packet length too short for a tcp packet"
    data_off = ((seg[12] >> 4) & 0xF) * 4
    if data_off > len(seg):
        return "dataOffset too big"
    off = 20
    while data_off > 20 and off < data_off:
        kind = seg[off]
        if kind in (TCP_OPTION_END, TCP_OPTION_NOP):
            off += 1
            if kind == TCP_OPTION_END:
                break
            continue
        if off + 1 >= data_off:
            return "invalid tcp option, reaches dataOffset"
        ln = seg[off + 1]
        if off + ln > data_off:
            return "invalid tcp option, length is too long"
        if ln == 0:
            return "tcp option of length 0 (the reference loops forever)"
        if ln == 1:
            return "tcp option of length 1 (IndexOutOfBounds in the reference)"
        if kind == TCP_OPTION_WINDOW_SCALE and ln != 3:
            return "invalid tcp option length for kind=window_scale"
        if kind == TCP_OPTION_MSS and ln != 4:
            return "invalid tcp option length for kind=mss"
        off += ln
    return None


def _l4_from(ver: int, proto: int, seg: bytes) -> str | None:
    """The L4 full parse (AbstractPacket.from): TcpPacket.from, UdpPacket.from (UdpPacket.java:
    40-60: >= 8 B and the length field equal to the buffer), IcmpPacket.from (IcmpPacket.java:
    33-45: >= 8 B), EtherIPPacket.from."""
    if proto == IP_PROTOCOL_TCP:
        return _tcp_from(seg)
    if proto == IP_PROTOCOL_UDP:
        if len(seg) < 8:
            return "input packet length too short for an udp packet"
        return "udp packet length not matching the input bytes length" if _u16(seg, 4) != len(seg) else None
    if proto == IP_PROTOCOL_ICMP or (ver == 6 and proto == IP_PROTOCOL_ICMPv6):
        return "input packet length too short for a icmp packet" if len(seg) < 8 else None
    if proto == IP_PROTOCOL_ETHERIP:
        return _etherip(seg)
    return None


def _ipv6_from(b: bytes, off: int) -> tuple[L3Info | None, str | None]:
    """Ipv6Packet.from(raw, mustParse) (Ipv6Packet.java:69-159)."""
    if len(b) < 40:
        return None, "input packet length too short for an ipv6 packet"
    if b[0] >> 4 != 6:
        return None, f"invalid version for ipv6 packet: {b[0] >> 4}"
    pl, nh = _u16(b, 4), b[6]
    if pl == 0:
        return None, "we do not support Jumbo Payload for now"
    if 40 + pl > len(b):
        return None, f"40+payloadLength({pl}) > input.length({len(b)})"
    total = 40 + pl                     # setPktBufLen: L2 padding is cut
    skip, proto = 0, nh
    if nh in IPv6_needs_next_header:
        # ExtHeader.from (Ipv6Packet.java ExtHeader): an ext header occupies 8 + hdrExtLen bytes
        # (the reference's rule, not RFC 8200's (len+1)*8).  A chain of two or more re-parses the
        # first one forever (xhBuf = xhBuf.sub(0, len)): refused.
        xh = b[40:total]
        if len(xh) < 8 or len(xh) < 8 + xh[1]:
            return None, "input packet length too short for an ipv6 ext hdr packet"
        if xh[0] in IPv6_needs_next_header:
            return None, "multiple ipv6 ext headers (the reference loops forever)"
        skip, proto = 8 + xh[1], xh[0]
    seg = b[40 + skip:total]
    if proto == IPv6_NO_NEXT_HEADER and len(seg) != 0:
        return None, "NO_NEXT_HEADER with bytes for a next packet"
    err = _l4_from(6, proto, seg)
    if err:
        return None, err
    return L3Info(off, total, 40 + skip, 6, proto), None


def _ipv4_from(b: bytes, off: int) -> tuple[L3Info | None, str | None]:
    """Ipv4Packet.from (Ipv4Packet.java:73-145)."""
    if len(b) < 20:
        return None, "input packet length too short for an ip packet"
    if b[0] >> 4 != 4:
        return None, f"invalid version for ipv4 packet: {b[0] >> 4}"
    ihl = b[0] & 0x0F
    if len(b) < ihl * 4:
        return None, f"input packet smaller than ihl({ihl}) specified"
    if ihl < 5:
        return None, f"input packet ihl({ihl}) < 5"
    total = _u16(b, 2)
    if total < ihl * 4:
        return None, f"input ihl({ihl}) > totalLength({total})"
    if total > len(b):
        return None, f"totalLength({total}) > input.length({len(b)})"
    err = _l4_from(4, b[9], b[ihl * 4:total])
    if err:
        return None, err
    return L3Info(off, total, ihl * 4, 4, b[9]), None


def parse_l3(buf: bytes, off: int, avail: int) -> tuple[L3Info | None, str | None]:
    """An IP packet without L2 (tun / FLAG_IP, PacketBuffer.init, PacketBuffer.java:156-174): the
    version nibble picks Ipv4Packet.from / Ipv6Packet.from, full parse down to L4.  Returns
    (info, err); err means vproxy refuses the packet (no checksum)."""
    b = bytes(buf[off:off + avail])
    if len(b) < 1:
        return None, "empty"
    ver = b[0] >> 4
    if ver == 4:
        return _ipv4_from(b, off)
    if ver == 6:
        return _ipv6_from(b, off)
    return None, f"receiving packet with unknown ip version: {ver}"


def _ipv4_init_partial(b: bytes, off: int) -> tuple[L3Info | None, str | None]:
    """Ipv4Packet.initPartial (Ipv4Packet.java:29-63): no version check (the EtherType chose
    IPv4), the L4 part only through initPartial."""
    if len(b) < 20:
        return None, "input packet length too short for an ip packet"
    ihl = b[0] & 0x0F
    if len(b) < ihl * 4:
        return None, f"input packet smaller than ihl({ihl}) specified"
    if ihl < 5:
        return None, f"input packet ihl({ihl}) < 5"
    total = _u16(b, 2)
    if total < ihl * 4:
        return None, f"input ihl({ihl}) > totalLength({total})"
    if total > len(b):
        return None, f"totalLength({total}) > input.length({len(b)})"
    err = _l4_init_partial(4, b[9], b[ihl * 4:total])
    if err:
        return None, err
    return L3Info(off, total, ihl * 4, 4, b[9]), None


def _ipv6_init_partial(b: bytes, off: int) -> tuple[L3Info | None, str | None]:
    """Ipv6Packet.initPartial (Ipv6Packet.java:26-59): no version check, unless the next header
    is an extension header -- then the full Ipv6Packet.from runs (L4 included)."""
    if len(b) < 40:
        return None, "input packet length too short for an ipv6 packet"
    nh = b[6]
    if nh in IPv6_needs_next_header:
        return _ipv6_from(b, off)
    pl = _u16(b, 4)
    if pl == 0:
        return None, "we do not support Jumbo Payload for now"
    if 40 + pl > len(b):
        return None, f"40+payloadLength({pl}) > input.length({len(b)})"
    err = _l4_init_partial(6, nh, b[40:40 + pl])
    if err:
        return None, err
    return L3Info(off, 40 + pl, 40, 6, nh), None


def parse_ether(frame: bytes) -> tuple[L3Info | None, str | None]:
    """An Ethernet frame as the vswitch receives it (tap / XDP: PacketBuffer.init ->
    EthernetPacket.from(raw, allowPartial=true), EthernetPacket.java:25-94): 14 B header, 18 B
    with an 802.1Q tag, then Ipv4Packet/Ipv6Packet.initPartial by EtherType.  An IP packet that
    fails to parse becomes PacketBytes (:60-64): no checksum, reported here as an error."""
    frame = bytes(frame)
    if len(frame) < 14:
        return None, "input packet length too short for a ethernet packet"
    typ, hl = _u16(frame, 12), 14
    if typ == ETHER_TYPE_8021Q:
        if len(frame) < 18:
            return None, "input packet length too short for 802.1q ethernet packet"
        typ, hl = _u16(frame, 16), 18
    if typ == ETHER_TYPE_IPv4:
        return _ipv4_init_partial(frame[hl:], hl)
    if typ == ETHER_TYPE_IPv6:
        return _ipv6_init_partial(frame[hl:], hl)
    return None, "not ip"


def desc_flags_for(info: L3Info, want_ip=True, want_l4=True) -> int:
    f = 0
    if want_ip and info.ver == 4:
        f |= F_IP
    if want_l4 and info.proto in L4_FIELD and not (info.ver == 4 and info.proto == IP_PROTOCOL_ICMPv6):
        if info.l3_len - info.l4_off >= L4_FIELD[info.proto] + 2:
            f |= F_L4
    return f


def flow_tuple(frame: bytes) -> dict:
    """The flow tuple the L4 input nodes read before their conntrack lookup, for one Ethernet
    frame: TcpInput.java:47-51 (tcpPkt.getSrc(ipPkt) / getDst(ipPkt) -> conntrack.lookupTcp;
    getFlags() == SYN -> lookupTcpListen), UdpInput.java:45-47 (ipPkt.getDst(), udpPkt.getDstPort()).
    Fields as the parsers set them: Ipv4Packet.initPartial src/dst at 12 / 16 (Ipv4Packet.java:51-54),
    Ipv6Packet at 8 / 24 (Ipv6Packet.java:47-50), Tcp/UdpPacket.initPartial ports at 0 / 2 and TCP
    flags = uint16(12) & 0x3f (TcpPacket.java:192-195, UdpPacket.java:22-23).  Bytes in network order,
    an IPv4 address in the first 4 of 16; a frame the parser refuses gives all zeros (l3_ver 0)."""
    t = {"src": bytes(16), "dst": bytes(16), "sport": bytes(2), "dport": bytes(2), "l3_ver": 0, "l4_proto": 0,
         "tcp_flags": 0}
    info, err = parse_ether(frame)
    if info is None:
        return t
    l3 = bytes(frame)[info.l3_off:info.l3_off + info.l3_len]
    if info.ver == 4:
        t["src"], t["dst"] = l3[12:16] + bytes(12), l3[16:20] + bytes(12)
    else:
        t["src"], t["dst"] = l3[8:24], l3[24:40]
    t["l3_ver"], t["l4_proto"] = info.ver, info.proto
    if info.proto in (IP_PROTOCOL_TCP, IP_PROTOCOL_UDP):
        l4 = l3[info.l4_off:]
        t["sport"], t["dport"] = l4[0:2], l4[2:4]
        if info.proto == IP_PROTOCOL_TCP:
            t["tcp_flags"] = _u16(l4, 12) & 0x3F
    return t


def hdr_words(l3: bytes, ver: int, l4_off: int, hlen: int, proto: int) -> bytes:
    """The words of the L4 sum an in-place setter of the vswitch can reach, as one byte string:
    the pseudo-header addresses (Utils.buildPseudoIPv4Header / IPv6Header, Utils.java:758-776) and
    the L4 header [0, hlen) with its checksum field as zeros -- TcpPacket.setSrcPort / setDstPort /
    setSeqNum / setAckNum / setFlags and TcpOption.setData (TcpPacket.java:31-110, 561-569),
    UdpPacket.setSrcPort / setDstPort (UdpPacket.java:188-209), Ipv4Packet / Ipv6Packet.setSrc /
    setDst (Ipv4Packet.java:433-458, Ipv6Packet.java:374-396) all write inside it."""
    addr = bytes(l3[12:20]) if ver == 4 else bytes(l3[8:40])
    h = bytearray(l3[l4_off:l4_off + hlen])
    f = L4_FIELD[proto]
    h[f:f + 2] = b"\x00\x00"
    return addr + bytes(h)


def hsum_record(frame: bytes) -> np.void:
    """The ingress header sum (vpcsum_hsum_t) of one received Ethernet frame, as the RX verify
    records it: the frame parsed with the vswitch's rules (parse_ether); for TCP (data offset 20..
    segment length) and UDP (8-B header in the segment) the per-step Java fold
    (Utils.calculateChecksumIntermediate, Utils.java:783-797) of :func:`hdr_words`, the segment length,
    the header length, protocol, version and the L3 header's offset in the frame; all zeros for
    any other frame."""
    r = np.zeros(1, HSUM_DTYPE)[0]
    info, _ = parse_ether(frame)
    if info is None or info.proto not in (IP_PROTOCOL_TCP, IP_PROTOCOL_UDP):
        return r
    l3 = bytes(frame)[info.l3_off:info.l3_off + info.l3_len]
    seg = info.l3_len - info.l4_off
    if info.proto == IP_PROTOCOL_TCP:
        if seg < 20:
            return r
        hlen = (l3[info.l4_off + 12] >> 4) * 4
        if hlen < 20 or hlen > seg:
            return r
    else:
        if seg < 8:
            return r
        hlen = 8
    w = hdr_words(l3, info.ver, info.l4_off, hlen, info.proto)
    r["sum"] = csum_intermediate(0, w, len(w))
    r["l4_len"], r["hlen"], r["l4_proto"], r["l3_ver"], r["l2_len"] = seg, hlen, info.proto, info.ver, info.l3_off
    return r


def pseudo_partial(l3: bytes, info: L3Info) -> int:
    """VPCSUM_F_L4P (checksum offload, XDPConsts.VP_CSUM_UP_PSEUDO): the folded, uncomplemented
    pseudo-header sum the L4 field holds for CHECKSUM_PARTIAL; Utils.calculateChecksumIntermediate
    over Utils.buildPseudoIPv4/IPv6Header (Utils.java:758-797)."""
    seg = info.l3_len - info.l4_off
    ph = pseudo_ipv4(l3, info.proto, seg) if info.ver == 4 else pseudo_ipv6(l3, info.proto, seg)
    return csum_intermediate(0, ph, len(ph))


def pure_process(l3: bytes, info: L3Info, flags: int) -> tuple[int, int]:
    """Pure-Python (ip_csum, l4_csum) for one parsed L3 packet."""
    ipc = ipv4_header_csum(l3, info.l4_off) if flags & F_IP else 0
    l4c = l4_csum(l3, info.l3_len, info.l4_off, info.ver, info.proto) if flags & F_L4 else 0
    if flags & F_L4P:
        l4c = pseudo_partial(l3, info)
    return ipc, l4c


def nat_java_pure(l3: bytearray, ver: int, proto: int, l3_len: int, l4_off: int, rw) -> None:
    """NAT / TTL rewrite as Java does it, in place on one L3 packet: the setters
    (Ipv4Packet.setSrc/setDst/setTtl, Ipv4Packet.java:401-407, 433-458; Ipv6Packet.setSrc/setDst/
    setHopLimit, Ipv6Packet.java:354-396; TcpPacket/UdpPacket.setSrcPort/setDstPort) mark the sums
    dirty (pseudoHeaderChanges: Ipv4Packet.java:236-240, Ipv6Packet.java:238-242) and
    getRawPacket(0) recomputes them in full.  rw: one NAT_DTYPE record.  Returns the status:
    S_DONE, or S_BAD_DESC | S_TTL_EXPIRED (nothing written) for a TTL decrement of a TTL / hop
    limit <= 1, which IPInputRoute drops instead (IPInputRoute.java:81-88)."""
    m = int(rw["mask"])
    t = 8 if ver == 4 else 7
    if m & NAT_DEC_TTL and (int(rw["ttl"]) if m & NAT_SET_TTL else l3[t]) <= 1:
        return S_BAD_DESC | S_TTL_EXPIRED
    fld = L4_FIELD.get(proto, -1)
    l4sum = fld >= 0 and not (ver == 4 and proto == IP_PROTOCOL_ICMPv6) and l3_len - l4_off >= fld + 2
    addr_dirty = l4sum and (proto in (IP_PROTOCOL_TCP, IP_PROTOCOL_UDP) or
                            (ver == 6 and proto in (IP_PROTOCOL_ICMP, IP_PROTOCOL_ICMPv6)))
    ip_dirty = l4_dirty = False
    a = 12 if ver == 4 else 8
    alen = 4 if ver == 4 else 16
    if m & NAT_SRC:
        l3[a:a + alen] = bytes(rw["src"][:alen])
        ip_dirty, l4_dirty = ver == 4, l4_dirty or addr_dirty
    if m & NAT_DST:
        l3[a + alen:a + 2 * alen] = bytes(rw["dst"][:alen])
        ip_dirty, l4_dirty = ver == 4, l4_dirty or addr_dirty
    if m & NAT_SET_TTL:
        l3[t] = int(rw["ttl"])
        ip_dirty = ip_dirty or ver == 4
    if m & NAT_DEC_TTL:
        l3[t] = (l3[t] - 1) & 0xFF
        ip_dirty = ip_dirty or ver == 4
    if l4sum and proto in (IP_PROTOCOL_TCP, IP_PROTOCOL_UDP):
        if m & NAT_SPORT:
            l3[l4_off:l4_off + 2] = bytes(rw["sport"])
            l4_dirty = True
        if m & NAT_DPORT:
            l3[l4_off + 2:l4_off + 4] = bytes(rw["dport"])
            l4_dirty = True
    if ip_dirty:
        l3[10:12] = ipv4_header_csum(bytes(l3), l4_off).to_bytes(2, "big")
    if l4_dirty:
        l3[l4_off + fld:l4_off + fld + 2] = l4_csum(bytes(l3), l3_len, l4_off, ver, proto).to_bytes(2, "big")
    return S_DONE


# ----------------------------------------------------------------------------------------
# C oracle (same algorithm, for batches and the timed CPU baseline)
# ----------------------------------------------------------------------------------------
def build(force: bool = False) -> str:
    src = os.path.join(HERE, "csum_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


class Oracle:
    def __init__(self):
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, U32, U64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        L.orc_process_batch.argtypes = [P, U64, P, U32, U32, P, P, P]
        L.orc_process_batch_mt.argtypes = [P, U64, P, U32, U32, P, P, ctypes.c_int]
        L.orc_process_batch_mt.restype = ctypes.c_int
        L.orc_csum.argtypes = [P, U32]
        L.orc_csum.restype = U32
        L.orc_csum_intermediate.argtypes = [U32, P, U32]
        L.orc_csum_intermediate.restype = U32
        L.orc_synth_batch.argtypes = [P, U32, U32, U32, U32, U64, U64, P]
        L.orc_synth_batch_mt.argtypes = [P, U32, U32, U32, U32, U64, U64, P, ctypes.c_int]
        L.orc_synth_batch_mt.restype = ctypes.c_int
        L.orc_process_batch_mt_w.argtypes = [P, U64, P, U32, U32, P, P, P, ctypes.c_int]
        L.orc_process_batch_mt_w.restype = ctypes.c_int
        L.orc_nat4_java.argtypes = [P, U64, P, P, P]
        L.orc_nat4_java_batch.argtypes = [P, U64, P, P, U32, P, ctypes.c_int]
        L.orc_nat4_java_batch.restype = ctypes.c_int
        L.orc_nat_java_batch.argtypes = [P, U64, P, P, ctypes.c_int, U32, P, ctypes.c_int]
        L.orc_nat_java_batch.restype = ctypes.c_int
        L.orc_nat_setters_batch.argtypes = [P, U64, P, P, U32, P]
        L.orc_rng.argtypes = [U64, U64, U64]
        L.orc_rng.restype = U64
        self.L = L

    @staticmethod
    def _p(a):
        return None if a is None else a.ctypes.data_as(ctypes.c_void_p)

    def csum(self, b: bytes) -> int:
        arr = np.frombuffer(b, dtype=np.uint8) if len(b) else np.zeros(1, np.uint8)
        return int(self.L.orc_csum(self._p(arr), len(b)))

    def process(self, arena: np.ndarray, desc: np.ndarray, mode: int = MODE_COMPUTE,
                write: bool = False, threads: int = 1):
        n = len(desc)
        out = np.zeros(n, np.uint32)
        status = np.zeros(n, np.uint8)
        if write:
            mode |= MODE_WRITE
        if threads > 1:   # with write: the packets must not overlap
            desc = np.ascontiguousarray(desc)
            rc = self.L.orc_process_batch_mt_w(self._p(arena), arena.nbytes, self._p(desc), n, mode,
                                               self._p(out), self._p(status), self._p(arena) if write else None,
                                               threads)
            assert rc == 0
        else:
            self.L.orc_process_batch(self._p(arena), arena.nbytes, self._p(desc), n, mode,
                                     self._p(out), self._p(status), self._p(arena) if write else None)
        return out, status

    def synth(self, n: int, stride: int, l3_pad: int, workload: int, seed: int, first_index: int = 0,
              threads: int = 1):
        arena = np.zeros(n * stride, np.uint8)
        desc = np.zeros(n, DESC_DTYPE)
        if threads > 1:
            assert self.L.orc_synth_batch_mt(self._p(arena), n, stride, l3_pad, workload, seed, first_index,
                                             self._p(desc), threads) == 0
        else:
            self.L.orc_synth_batch(self._p(arena), n, stride, l3_pad, workload, seed, first_index, self._p(desc))
        return arena, desc

    def nat4_java(self, arena: np.ndarray, desc: np.ndarray, rw: np.ndarray, threads: int = 1):
        """In order on one thread; threads > 1 needs frames that do not overlap."""
        status = np.zeros(len(desc), np.uint8)
        desc = np.ascontiguousarray(desc)
        rw = np.ascontiguousarray(rw)
        rc = self.L.orc_nat4_java_batch(self._p(arena), arena.nbytes, self._p(desc), self._p(rw), len(desc),
                                        self._p(status), threads)
        assert rc == 0
        return status

    def nat_java(self, arena: np.ndarray, desc: np.ndarray, rw: np.ndarray, threads: int = 1):
        """48-B vpcsum_nat_t entries (IPv4 and IPv6), Java semantics; in order on one thread."""
        status = np.zeros(len(desc), np.uint8)
        desc = np.ascontiguousarray(desc)
        rw = np.ascontiguousarray(rw)
        assert rw.dtype == NAT_DTYPE
        rc = self.L.orc_nat_java_batch(self._p(arena), arena.nbytes, self._p(desc), self._p(rw), 1, len(desc),
                                       self._p(status), threads)
        assert rc == 0
        return status

    def nat_setters(self, arena: np.ndarray, desc: np.ndarray, rw: np.ndarray):
        """Java's setters alone (48-B entries): the new bytes written, the stored sums left stale --
        the frames a pre-image flush (VPCSUM_F_PRE) receives.  Returns the status per packet."""
        status = np.zeros(len(desc), np.uint8)
        desc = np.ascontiguousarray(desc)
        rw = np.ascontiguousarray(rw)
        assert rw.dtype == NAT_DTYPE
        self.L.orc_nat_setters_batch(self._p(arena), arena.nbytes, self._p(desc), self._p(rw), len(desc),
                                     self._p(status))
        return status

    def rng(self, seed: int, pkt: int, word: int) -> int:
        return int(self.L.orc_rng(seed, pkt, word))


SYNTH_C1, SYNTH_C2, SYNTH_C3, SYNTH_C4, SYNTH_FUZZ, SYNTH_C5 = 1, 2, 3, 4, 5, 6
SEED = 0x20241020
