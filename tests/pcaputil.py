"""Minimal pcap reader for the reference's fixtures (test tooling).

Link types as handled by the reference's PcapParser (base/.../vpacket/PcapParser.java):
1 = Ethernet (EthernetPacket), 113 = Linux cooked SLL (LinuxCookedPacket, 16-byte header,
protocol at bytes 14..15), 0 = BSD loopback (BSDLoopbackEncapsulation, 4-byte family)."""
from __future__ import annotations

import struct


def read_pcap(path: str) -> tuple[int, list[bytes]]:
    data = open(path, "rb").read()
    magic = struct.unpack("<I", data[:4])[0]
    end = "<" if magic == 0xA1B2C3D4 else ">"
    _, _, _, _, _, _, linktype = struct.unpack(end + "IHHiIII", data[:24])
    off = 24
    pkts = []
    while off + 16 <= len(data):
        _, _, incl, _ = struct.unpack(end + "IIII", data[off:off + 16])
        off += 16
        pkts.append(data[off:off + incl])
        off += incl
    return linktype, pkts


def l3_offset(linktype: int, pkt: bytes) -> int | None:
    """Offset of the IP header inside a captured packet, or None if not IP."""
    if linktype == 1:
        typ = (pkt[12] << 8) | pkt[13]
        if typ == 0x8100:
            typ = (pkt[16] << 8) | pkt[17]
            return 18 if typ in (0x0800, 0x86DD) else None
        return 14 if typ in (0x0800, 0x86DD) else None
    if linktype == 113:
        typ = (pkt[14] << 8) | pkt[15]
        return 16 if typ in (0x0800, 0x86DD) else None
    if linktype == 0:
        return 4
    return None
