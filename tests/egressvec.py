"""Egress frames as vproxy holds them at Iface.sendPacket (test infrastructure: tests/ only).

An XDP or tap frame is parsed with EthernetPacket.from(raw, allowPartial=true) (PacketBuffer.java:
177 -> EthernetPacket.java:52-56), i.e. Ipv4Packet / Ipv6Packet.initPartial.  Such a packet keeps
the frame's Ethernet padding in its buffer (initPartial does not cut to totalLength,
Ipv4Packet.java:29-63; from() would, :100-103) and leaves `options` empty, so
getRawPacket().length() includes the padding and getHeaderSize() is 20 for any IHL.  Java's own
recompute covers exactly [ihl*4, totalLength) (:55, TcpPacket.java:475-485).

The frames below hit those cases by construction:

* 60-B Ethernet frames holding a 40-B IPv4/TCP ACK (6 B of padding) or a short UDP / ICMP
  message (the NIC minimum frame), padding bytes random and non-zero;
* IPv4 with options, IHL 6..15, TCP / UDP / ICMP;
* 802.1Q-tagged frames (L3 at +18);
* IPv6 with one extension header (Java's 8 + hdrExtLen rule), and IPv6 frames with trailing
  bytes past 40 + payloadLength (an FCS left in the buffer).

Frames lie in a umem-like arena: 2048-B chunks, the frame at chunk + 384 (UMem headroom,
XDPIface.java:144-147), so L3 is 2-B aligned (+398 / +402).
"""
from __future__ import annotations

import numpy as np

from oracle import oracle as O

CHUNK, HEADROOM = 2048, 384


def _put16(b, off, v):
    b[off] = (v >> 8) & 0xFF
    b[off + 1] = v & 0xFF


def _ipv4(rng, proto: int, l4len: int, ihl: int) -> bytearray:
    hl = ihl * 4
    p = bytearray(rng.integers(0, 256, hl + l4len, dtype=np.uint8).tobytes())
    p[0] = 0x40 | ihl
    _put16(p, 2, hl + l4len)
    p[9] = proto
    if proto == 6:
        p[hl + 12] = 0x50
    elif proto == 17:
        _put16(p, hl + 4, l4len)
    return p


def _ipv6(rng, proto: int, l4len: int, ext: int | None) -> bytearray:
    xl = 0 if ext is None else 8 + ext
    p = bytearray(rng.integers(0, 256, 40 + xl + l4len, dtype=np.uint8).tobytes())
    p[0] = 0x60
    _put16(p, 4, xl + l4len)
    if ext is None:
        p[6] = proto
    else:
        p[6], p[40], p[41] = 60, proto, ext   # destination options
    l4 = 40 + xl
    if proto == 6:
        p[l4 + 12] = 0x50
    elif proto == 17:
        _put16(p, l4 + 4, l4len)
    return p


def _ether(rng, l3: bytes, ver: int, vlan: bool, min_frame: int = 60, trailer: int = 0) -> bytes:
    et = b"\x08\x00" if ver == 4 else b"\x86\xdd"
    l2 = bytes(rng.integers(0, 256, 12, dtype=np.uint8)) + ((b"\x81\x00" + bytes([0x00, 0x64]) + et) if vlan else et)
    f = l2 + bytes(l3)
    pad = max(min_frame - len(f), 0) + trailer
    return f + bytes(rng.integers(1, 256, pad, dtype=np.uint8))   # non-zero padding


def frames(seed: int = 11) -> list[dict]:
    """[{frame, ver, proto, kind}]: each frame as the Java side holds it."""
    rng = np.random.default_rng(seed)
    out = []

    def add(l3, ver, proto, kind, vlan=False, trailer=0):
        out.append(dict(frame=_ether(rng, l3, ver, vlan, trailer=trailer), ver=ver, proto=proto, kind=kind,
                        vlan=vlan))

    for vlan in (False, True):
        # the bare TCP ACK: 14 + 40 = 54 B -> padded to 60
        add(_ipv4(rng, 6, 20, 5), 4, 6, "v4_tcp_ack_padded", vlan)
        for l4len in (8, 9, 12, 18, 25):                      # short UDP / ICMP in a padded frame
            add(_ipv4(rng, 17, l4len, 5), 4, 17, "v4_udp_padded", vlan)
            add(_ipv4(rng, 1, l4len, 5), 4, 1, "v4_icmp_padded", vlan)
        for ihl in range(6, 16):                              # IPv4 options
            for proto, l4len in ((6, 20), (6, 1460 - ihl * 4), (17, 8), (17, 333), (1, 8), (1, 61)):
                add(_ipv4(rng, proto, l4len, ihl), 4, proto, f"v4_opt_ihl{ihl}", vlan)
        for ext in (0, 1, 7, 8, 13, 40):                      # IPv6 with one extension header
            for proto, l4len in ((6, 20), (17, 8), (17, 101), (58, 8), (58, 77), (1, 30)):
                add(_ipv6(rng, proto, l4len, ext), 6, proto, f"v6_ext{ext}", vlan)
        for proto, l4len in ((6, 20), (17, 8), (58, 8)):      # IPv6 with a 4-B trailer
            add(_ipv6(rng, proto, l4len, None), 6, proto, "v6_trailer", vlan, trailer=4)
    return out


def want_flags(ver: int, proto: int, kind: int) -> int:
    """Dirty flags per frame, cycling through what checksumFlagsFor yields: IP + L4, L4 alone, IP
    alone, L4 pseudo (offload; not for ICMPv4)."""
    f4 = O.F_IP if ver == 4 else 0
    choices = [f4 | O.F_L4, O.F_L4, f4 or O.F_L4]
    if proto in (6, 17) or (ver == 6 and proto == 58):
        choices.append(f4 | O.F_L4P)
    return choices[kind % len(choices)]


def layout(fs: list[dict]) -> tuple[np.ndarray, list[int]]:
    """The frames in a umem-like arena: (arena, frame offsets)."""
    arena = np.zeros(CHUNK * len(fs), np.uint8)
    offs = []
    for i, f in enumerate(fs):
        o = i * CHUNK + HEADROOM
        arena[o:o + len(f["frame"])] = np.frombuffer(f["frame"], np.uint8)
        offs.append(o)
    return arena, offs


def oracle_descriptors(fs: list[dict], offs: list[int], flags: list[int]) -> np.ndarray:
    """The bytes Java's recompute covers, from the oracle's restatement of the reference parser
    (oracle.parse_ether: EthernetPacket.from(allowPartial) -> Ipv4/Ipv6Packet.initPartial)."""
    d = np.zeros(len(fs), O.DESC_DTYPE)
    for i, (f, o, fl) in enumerate(zip(fs, offs, flags)):
        info, err = O.parse_ether(f["frame"])
        assert info is not None, (f["kind"], err)
        d[i] = (o + info.l3_off, info.l3_len, info.l4_off, info.ver, info.proto, fl, 0)
    return d


def buffer_length_descriptors(fs: list[dict], offs: list[int], flags: list[int]) -> np.ndarray:
    """Round 2's GpuCsumBatch.defer: l3_len = getRawPacket().length() (the buffer: padding
    included), l4_off = getHeaderSize() (20 + empty options for IPv4).  Kept to show the frames
    above tell the two apart."""
    d = oracle_descriptors(fs, offs, flags)
    for i, f in enumerate(fs):
        hl = 18 if f["vlan"] else 14
        d[i]["l3_len"] = len(f["frame"]) - hl
        if f["ver"] == 4:
            d[i]["l4_off"] = 20
    return d
