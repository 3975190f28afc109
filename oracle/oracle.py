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
  Ipv4Packet.java:73-145; Ipv6Packet.from, Ipv6Packet.java:69-159) producing descriptors.

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

F_IP, F_L4, F_RAW, F_L4P = 0x01, 0x02, 0x04, 0x08
S_IP_OK, S_L4_OK, S_UDP_NOCSUM, S_DONE, S_BAD_DESC = 0x01, 0x02, 0x04, 0x40, 0x80
MODE_COMPUTE, MODE_VERIFY, MODE_WRITE = 0x00, 0x01, 0x10
NAT_SRC, NAT_DST, NAT_SPORT, NAT_DPORT, NAT_DEC_TTL = 0x01, 0x02, 0x04, 0x08, 0x10

DESC_DTYPE = np.dtype([("l3_off", "<u8"), ("l3_len", "<u2"), ("l4_off", "<u2"), ("l3_ver", "u1"),
                       ("l4_proto", "u1"), ("flags", "u1"), ("rsv", "u1")])
NAT4_DTYPE = np.dtype([("src", "u1", 4), ("dst", "u1", 4), ("sport", "u1", 2), ("dport", "u1", 2),
                       ("mask", "u1"), ("rsv", "u1", 3)])
assert DESC_DTYPE.itemsize == 16 and NAT4_DTYPE.itemsize == 16

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


def parse_l3(buf: bytes, off: int, avail: int) -> tuple[L3Info | None, str | None]:
    """Ipv4Packet.from (Ipv4Packet.java:73-145) / Ipv6Packet.from (Ipv6Packet.java:69-159)
    reduced to the fields the checksum needs. Returns (info, err)."""
    b = buf[off:off + avail]
    if len(b) < 1:
        return None, "empty"
    ver = b[0] >> 4
    if ver == 4:
        if len(b) < 20:
            return None, "input packet length too short for an ip packet"
        ihl = b[0] & 0x0F
        if len(b) < ihl * 4:
            return None, f"input packet smaller than ihl({ihl}) specified"
        if ihl < 5:
            return None, f"input packet ihl({ihl}) < 5"
        total = (b[2] << 8) | b[3]
        if total < ihl * 4:
            return None, f"input ihl({ihl}) > totalLength({total})"
        if total > len(b):
            return None, f"totalLength({total}) > input.length({len(b)})"
        return L3Info(off, total, ihl * 4, 4, b[9]), None
    if ver == 6:
        if len(b) < 40:
            return None, "input packet length too short for an ipv6 packet"
        pl = (b[4] << 8) | b[5]
        nh = b[6]
        if pl == 0:
            return None, "we do not support Jumbo Payload for now"
        if 40 + pl > len(b):
            return None, f"40+payloadLength({pl}) > input.length({len(b)})"
        total = 40 + pl
        skip = 0
        proto = nh
        if nh in IPv6_needs_next_header:
            # Ipv6Packet.java:121-139 / ExtHeader.from :199-211: an ext header occupies
            # 8 + hdrExtLen bytes (the reference's rule, not RFC 8200's (len+1)*8).  A chain
            # of more than one ext header re-parses the first one forever in the reference
            # (xhBuf = xhBuf.sub(0, len)), so only single-ext-header packets are defined.
            xh = b[40:total]
            if len(xh) < 8:
                return None, "input packet length too short for an ipv6 ext hdr packet"
            nxt, hlen = xh[0], xh[1]
            if len(xh) < 8 + hlen:
                return None, "input packet length too short for an ipv6 ext hdr packet"
            if nxt in IPv6_needs_next_header:
                return None, "multiple ipv6 ext headers (reference loops forever)"
            skip = 8 + hlen
            proto = nxt
        return L3Info(off, total, 40 + skip, 6, proto), None
    return None, f"invalid version {ver}"


def parse_ether(frame: bytes) -> tuple[L3Info | None, str | None]:
    """EthernetPacket.from (EthernetPacket.java:25-94): 14 B header, 18 B with an 802.1Q tag."""
    if len(frame) < 14:
        return None, "input packet length too short for a ethernet packet"
    typ = (frame[12] << 8) | frame[13]
    hl = 14
    if typ == ETHER_TYPE_8021Q:
        if len(frame) < 18:
            return None, "input packet length too short for 802.1q ethernet packet"
        typ = (frame[16] << 8) | frame[17]
        hl = 18
    if typ not in (ETHER_TYPE_IPv4, ETHER_TYPE_IPv6):
        return None, "not ip"
    info, err = parse_l3(frame, hl, len(frame) - hl)
    if info is not None and ((typ == ETHER_TYPE_IPv4) != (info.ver == 4)):
        return None, "version mismatch"
    return info, err


def desc_flags_for(info: L3Info, want_ip=True, want_l4=True) -> int:
    f = 0
    if want_ip and info.ver == 4:
        f |= F_IP
    if want_l4 and info.proto in L4_FIELD and not (info.ver == 4 and info.proto == IP_PROTOCOL_ICMPv6):
        if info.l3_len - info.l4_off >= L4_FIELD[info.proto] + 2:
            f |= F_L4
    return f


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
        L.orc_nat4_java.argtypes = [P, U64, P, P, P]
        L.orc_nat4_java_batch.argtypes = [P, U64, P, P, U32, P, ctypes.c_int]
        L.orc_nat4_java_batch.restype = ctypes.c_int
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
        if threads > 1 and not write:
            rc = self.L.orc_process_batch_mt(self._p(arena), arena.nbytes, self._p(desc), n, mode,
                                             self._p(out), self._p(status), threads)
            assert rc == 0
        else:
            self.L.orc_process_batch(self._p(arena), arena.nbytes, self._p(desc), n, mode,
                                     self._p(out), self._p(status), self._p(arena) if write else None)
        return out, status

    def synth(self, n: int, stride: int, l3_pad: int, workload: int, seed: int, first_index: int = 0):
        arena = np.zeros(n * stride, np.uint8)
        desc = np.zeros(n, DESC_DTYPE)
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

    def rng(self, seed: int, pkt: int, word: int) -> int:
        return int(self.L.orc_rng(seed, pkt, word))


SYNTH_C1, SYNTH_C2, SYNTH_C3, SYNTH_C4, SYNTH_FUZZ, SYNTH_C5 = 1, 2, 3, 4, 5, 6
SEED = 0x20241020
