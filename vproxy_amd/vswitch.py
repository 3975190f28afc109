"""Host-side mirror of the vswitch seam that drives the GPU checksum (tests / tooling / Python
callers).  Same contract as java/io/vproxy/vpcsum/GpuCsumBatch.java:

* :func:`checksum_flags_for` -- SwitchUtils.checksumFlagsFor (core/.../vswitch/util/
  SwitchUtils.java:297-316): IP dirty -> F_IP (VP_CSUM_IP), upper layer dirty -> F_L4 (VP_CSUM_UP).
* :class:`EgressBatch` -- defer dirty frames at Iface.sendPacket, compute every deferred sum at
  Iface.completeTx in one GPU launch, written into the frames (XDPIface.java:100-178, 227-243).
* :func:`egress_descriptor` -- the descriptor GpuCsumBatch.defer builds from the parsed Java
  packet of a frame vproxy holds (partially parsed: Ethernet padding and IPv4 options included in
  the buffer, so the lengths come from the IP header fields, not from the buffer).
* :func:`descriptors_for_frames` -- build descriptors for received Ethernet frames on the GPU
  (EthernetPacket/Ipv4Packet/Ipv6Packet.from rules) for ingress verify.
* :func:`recalc_policy` -- the verify status -> DevInput csum-recalc decision (which frames get
  their sums marked dirty, which are dropped), INTEGRATION.md §4.

No checksum is computed on the CPU here: everything goes through libvpcsum.so.
"""
from __future__ import annotations

import numpy as np

from . import vpcsum as V

ETHER_TYPE_IPv4, ETHER_TYPE_IPv6, ETHER_TYPE_8021Q = 0x0800, 0x86DD, 0x8100
L4_WITH_CSUM = {6, 17, 1, 58}


def checksum_flags_for(is_ipv4: bool, ip_dirty: bool, upper_proto: int, upper_dirty: bool,
                       offload: bool = False) -> int:
    """SwitchUtils.checksumFlagsFor: which sums a frame needs recomputed.  IPv6 has no header
    checksum (Ipv6Packet.__updateChecksum only recurses, Ipv6Packet.java:214-217).  With
    ``offload`` (checksum offload on the TX queue: VP_CSUM_UP_PSEUDO | VP_CSUM_XDP_OFFLOAD) the
    upper layer gets only its pseudo-header sum (F_L4P); ICMPv4 has none and is summed in full."""
    f = 0
    if is_ipv4 and ip_dirty:
        f |= V.F_IP
    if upper_dirty and upper_proto in L4_WITH_CSUM and not (is_ipv4 and upper_proto == 58):
        f |= V.F_L4P if offload and upper_proto != 1 else V.F_L4
    return f


# IPv6 next-header values Java parses as extension headers (Consts.IPv6_needs_next_header,
# base/src/main/java/io/vproxy/base/util/Consts.java:31)
IPV6_EXT_HEADERS = frozenset({0, 60, 43, 44, 51, 50, 135, 139, 140, 253, 254})


def _u16(b, o: int) -> int:
    return (int(b[o]) << 8) | int(b[o + 1])


def egress_descriptor(frame, frame_off: int, flags: int):
    """The descriptor GpuCsumBatch.defer fills for one frame, from what the Java packet objects
    report (java/io/vproxy/vpcsum/GpuCsumBatch.java: defer):

    * L3 at frame + 14, or + 18 with an 802.1Q tag (EthernetPacket.getVlan(), EthernetPacket.java:
      32-37);
    * IPv4: l3_len = Ipv4Packet.getTotalLength() and l4_off = getIhl() * 4 (:334, :361).  A frame
      parsed with allowPartial (every XDP / tap frame: PacketBuffer.java:177 -> EthernetPacket.java:
      52-56) keeps its Ethernet padding in pktBuf and leaves `options` empty (initPartial,
      Ipv4Packet.java:29-63), so neither the buffer length nor getHeaderSize() may be used;
      Java's own recompute covers raw.sub(ihl*4, totalLength - ihl*4) (:55);
    * IPv6: l3_len = 40 + getPayloadLength() (:332), l4_off = getHeaderSize() (:427-435: 40 +
      8 + hdrExtLen per extension header, which from() fills whenever the next header is one,
      :33-35), l4_proto = getProtocol() (the last header's next header, :363-367).

    An IPv6 chain of two or more extension headers never reaches the seam in vproxy (Ipv6Packet.from
    loops on it), and the GPU parser refuses it: here the descriptor names the second
    extension header as l4_proto, which the kernel refuses with F_L4 (S_BAD_DESC), so such a frame is
    handed back to the native path.

    `frame` holds the frame's bytes from its first byte (at least its headers: a frame near the end
    of the arena may be shorter than 64 B): the header fields the Java object exposes are read from
    it (no checksum is computed here).  Returns a DESC_DTYPE record, or None for a frame that is not
    IP or too short to hold its IP header."""
    b = frame
    if len(b) < 14:
        return None
    typ, hl = _u16(b, 12), 14
    if typ == ETHER_TYPE_8021Q:
        if len(b) < 18:
            return None
        typ, hl = _u16(b, 16), 18
    d = np.zeros(1, V.DESC_DTYPE)[0]
    d["l3_off"] = frame_off + hl
    d["flags"] = flags
    if typ == ETHER_TYPE_IPv4:
        if len(b) < hl + 20:
            return None
        d["l3_len"] = _u16(b, hl + 2)
        d["l4_off"] = (int(b[hl]) & 0x0F) * 4
        d["l3_ver"], d["l4_proto"] = 4, int(b[hl + 9])
    elif typ == ETHER_TYPE_IPv6:
        if len(b) < hl + 40:
            return None
        nh, off = int(b[hl + 6]), 40
        if nh in IPV6_EXT_HEADERS:   # one extension header (a chain makes Java's parser loop)
            if len(b) < hl + 42:
                return None
            nh, off = int(b[hl + 40]), 40 + 8 + int(b[hl + 41])
        d["l3_len"] = 40 + _u16(b, hl + 4)
        d["l4_off"] = off
        d["l3_ver"], d["l4_proto"] = 6, nh
    else:
        return None
    return d


NAT_FIELDS = V.NAT_SRC | V.NAT_DST | V.NAT_SPORT | V.NAT_DPORT


def record_pre_image(arena, l3_off: int, ver: int, l4_off: int, proto: int, mask: int = NAT_FIELDS):
    """The pre-image the vswitch records just before SwitchUtils.applyNat runs the setters
    (SwitchUtils.java:531-542): the old source / destination address and, for
    TCP / UDP, the old ports -- what ipPkt.getSrc() / getDst() and pkt.getSrcPort() / getDstPort()
    return at that moment (the cached fields equal the frame's bytes: Ipv4Packet.from reads them
    from the buffer, :73-145).  Returns one NAT_DTYPE record (vpcsum_pre_t) holding the old values,
    mask = the fields recorded.  No checksum arithmetic happens here."""
    e = np.zeros(1, V.NAT_DTYPE)[0]
    a, alen = (l3_off + 12, 4) if ver == 4 else (l3_off + 8, 16)
    if mask & V.NAT_SRC:
        e["src"][:alen] = arena[a:a + alen]
    if mask & V.NAT_DST:
        e["dst"][:alen] = arena[a + alen:a + 2 * alen]
    m = mask & (V.NAT_SRC | V.NAT_DST)
    if proto in (6, 17):
        p = l3_off + l4_off
        if mask & V.NAT_SPORT:
            e["sport"] = arena[p:p + 2]
        if mask & V.NAT_DPORT:
            e["dport"] = arena[p + 2:p + 4]
        m |= mask & (V.NAT_SPORT | V.NAT_DPORT)
    e["mask"] = m
    return e


def hsum_entry(rec) -> np.void:
    """The 48-B pre-image entry (NAT_DTYPE, mask PRE_HSUM) that carries a frame's ingress header
    sum (HSUM_DTYPE record, from Context.verify_frames_hsum) to the egress flush: the record in
    its first 8 bytes (GpuCsumBatch.defer, java/io/vproxy/vpcsum/PreImage.java:writeTo)."""
    raw = np.zeros(48, np.uint8)
    raw[:8] = np.frombuffer(np.asarray(rec, V.HSUM_DTYPE).tobytes(), np.uint8)
    raw[36] = V.PRE_HSUM
    return raw.view(V.NAT_DTYPE)[0]


def hsum_eligible(rx_status: int, rec, l3_rx: int, in_place: bool, l3_now: int, ver: int, proto: int, l3_len: int,
                  l4_off: int, tcp_hlen: int) -> bool:
    """GpuCsumBatch.defer's rule for F_PRE: a frame whose L4 sum is dirty
    takes the header-sum update instead of the full recompute only when
      * the ingress verify proved its stored L4 sum (S_L4_OK, no S_BAD_DESC) and recorded its header
        sum (l2_len != 0);
      * it leaves from the zero-copy branch of XDPIface.sendPacket with its bytes still the received
        frame (`in_place`: pkb.fullbuf is still the RX chunk -- any clearRawPacket on the packet or
        its layers, e.g. TcpPacket.setData / setOptions / the MSS option added by
        SwitchUtils.checkAndUpdateMss, and PacketBuffer.replacePacket null it, AbstractPacket.java:
        27-36, PacketBuffer.java:199-253) and its L3 header where it was received (`l3_now` ==
        `l3_rx`: a decapsulated inner frame or a moved header never matches);
      * its version, protocol, segment length and L4 header length (the TCP data offset the packet
        object now reports) are the record's.
    Then every byte outside the header words the record sums is the received byte, so the update is
    exact whatever the in-place setters wrote into those words (addresses, ports, sequence and
    acknowledgement numbers, flags, an option's data)."""
    if (rx_status & (V.S_L4_OK | V.S_BAD_DESC)) != V.S_L4_OK or int(rec["l2_len"]) == 0:
        return False
    if not in_place or l3_now != l3_rx:
        return False
    if int(rec["l3_ver"]) != ver or int(rec["l4_proto"]) != proto or int(rec["l4_len"]) != l3_len - l4_off:
        return False
    return proto == 17 and int(rec["hlen"]) == 8 or proto == 6 and int(rec["hlen"]) == tcp_hlen


def pre_eligible(rx_status: int) -> bool:
    """Whether a NAT'd frame's L4 sum may be updated from its pre-image at egress: ingress verify
    proved the stored L4 sum correct (S_L4_OK; a UDP stored 0 never carries it).  Otherwise the
    frame takes the full recompute, as Java's getRawPacket(0) does (AbstractPacket.java:58-65)."""
    return (rx_status & V.S_BAD_DESC) == 0 and (rx_status & V.S_L4_OK) != 0


class RxPacket:
    """A received frame as the vswitch holds it between XDPIface.readable and sendPacket: its
    PacketBuffer with the fields the integration adds (csumStatus, csumHsum, csumL3: the verify
    status, the ingress header sum and the L3 header's umem offset) and the byte
    effects of the packet objects' setters on the umem frame.

    The in-place setters (the `raw != null` branch of TcpPacket.setSrcPort / setDstPort /
    setSeqNum / setAckNum / setFlags, TcpPacket.java:31-100; TcpOption.setData of a same-length
    option, :561-569; UdpPacket.setSrcPort / setDstPort, UdpPacket.java:188-209; Ipv4Packet.setSrc /
    setDst / setTtl, Ipv4Packet.java:401-458; Ipv6Packet.setSrc / setDst) write the frame's bytes
    and mark sums dirty.  Every other change rebuilds the packet (clearRawPacket, which clears the
    PacketBuffer's buffers up the parent chain, AbstractPacket.java:27-36, PacketBuffer.java:
    199-208): the frame then leaves through XDPIface.sendPacket's copying branch from another chunk
    (:139-168) -- :meth:`rebuild` -- and PacketBuffer.replacePacket (TcpReset, TcpStack, the ICMP
    answers) also resets the integration's fields -- :meth:`replace`."""

    def __init__(self, arena: np.ndarray, frame_off: int, rx_status: int, hsum_rec):
        self.arena = arena
        self.frame_off = frame_off
        self.csum_status = int(rx_status)
        self.csum_hsum = np.asarray(hsum_rec, V.HSUM_DTYPE).copy()
        l2 = int(self.csum_hsum["l2_len"])
        self.csum_l3 = frame_off + l2 if l2 else -1
        self.in_place = True      # pkb.fullbuf is still the RX chunk (the zero-copy send branch)
        self.ip_dirty = self.l4_dirty = False
        d = egress_descriptor(arena[frame_off:frame_off + 512], frame_off, 0)
        self.l3 = int(d["l3_off"])
        self.ver, self.proto = int(d["l3_ver"]), int(d["l4_proto"])
        self.l4 = self.l3 + int(d["l4_off"])

    # -- in-place setters ------------------------------------------------------------------
    def _pseudo_dirty(self):
        self.ip_dirty = self.ip_dirty or self.ver == 4
        self.l4_dirty = self.l4_dirty or self.proto in (6, 17)

    def set_src(self, addr: bytes):
        a, n = (self.l3 + 12, 4) if self.ver == 4 else (self.l3 + 8, 16)
        self.arena[a:a + n] = np.frombuffer(addr[:n], np.uint8)
        self._pseudo_dirty()

    def set_dst(self, addr: bytes):
        a, n = (self.l3 + 16, 4) if self.ver == 4 else (self.l3 + 24, 16)
        self.arena[a:a + n] = np.frombuffer(addr[:n], np.uint8)
        self._pseudo_dirty()

    def _l4_write(self, off: int, data: bytes):
        self.arena[self.l4 + off:self.l4 + off + len(data)] = np.frombuffer(data, np.uint8)
        self.l4_dirty = True

    def set_ports(self, sport: int, dport: int):
        self._l4_write(0, sport.to_bytes(2, "big") + dport.to_bytes(2, "big"))

    def set_seq(self, v: int):
        self._l4_write(4, (v & 0xFFFFFFFF).to_bytes(4, "big"))

    def set_ack(self, v: int):
        self._l4_write(8, (v & 0xFFFFFFFF).to_bytes(4, "big"))

    def set_tcp_flags(self, flags: int):
        """TcpPacket.setFlags in place (TcpPacket.java:90-96): the low 6 bits of the word at 12."""
        w = (int(self.arena[self.l4 + 12]) << 8 | int(self.arena[self.l4 + 13])) & 0xFFC0 | (flags & 0x3F)
        self._l4_write(12, w.to_bytes(2, "big"))

    def set_option_data(self, opt_off: int, data: bytes):
        """TcpOption.setData of an option of the same length: its data bytes at option + 2."""
        self._l4_write(opt_off + 2, data)

    def set_ttl(self, ttl: int):
        if self.ver == 4:
            self.arena[self.l3 + 8] = ttl
            self.ip_dirty = True
        else:
            self.arena[self.l3 + 7] = ttl   # Ipv6Packet.setHopLimit: no sum covers it

    # -- rebuilds --------------------------------------------------------------------------
    def rebuild(self, new_off: int, frame: bytes):
        """The packet was rebuilt (clearRawPacket): sendPacket copies its new bytes to another
        chunk; every sum of the new bytes is Java's to compute."""
        self.arena[new_off:new_off + len(frame)] = np.frombuffer(frame, np.uint8)
        self.__init_moved(new_off)

    def replace(self, new_off: int, frame: bytes):
        """PacketBuffer.replacePacket / clearAndSetPacket: a new packet in the same PacketBuffer
        (TcpReset.java:82 and the other callers); clearPackets resets csumStatus / csumHsum / csumL3."""
        self.csum_status, self.csum_l3 = -1, -1
        self.csum_hsum = np.zeros((), V.HSUM_DTYPE)
        self.rebuild(new_off, frame)

    def __init_moved(self, new_off: int):
        self.frame_off = new_off
        self.in_place = False
        d = egress_descriptor(self.arena[new_off:new_off + 512], new_off, 0)
        self.l3 = int(d["l3_off"])
        self.ver, self.proto = int(d["l3_ver"]), int(d["l4_proto"])
        self.l4 = self.l3 + int(d["l4_off"])
        self.ip_dirty = self.ver == 4
        self.l4_dirty = self.proto in L4_WITH_CSUM

    def tcp_hlen(self) -> int:
        """The TCP header length now in the frame (data offset nibble of byte 12 * 4; GpuCsumBatch
        reads the umem byte: a partially parsed TcpPacket has no getDataOffset(), :186-199)."""
        return (int(self.arena[self.l4 + 12]) >> 4) * 4 if self.proto == 6 else 0


class EgressBatch:
    """Deferred egress checksums over one host frame arena (e.g. an AF_XDP umem).

    ``defer`` is O(1) host work (fills a 16-B descriptor); ``complete_tx`` submits the batch and
    waits: one GPU launch per flush, results written in place (MODE_WRITE).  With
    ``register=True`` the arena is page-locked once and the kernel works on it zero-copy; with
    ``service_idle_us`` > 0 as well, flushes go to the low-latency service grid
    (vpcsum_ctx_set_service) instead of a kernel launch each."""

    def __init__(self, arena: np.ndarray, capacity: int = 4096, device: int = 0, register: bool = True,
                 service_idle_us: int = 0, small_flush: int = 0):
        self.arena = arena
        self.capacity = capacity
        # flushes of fewer frames are handed back to the caller's native path (GpuCsumBatch.flush,
        # SMALL_FLUSH: the GPU breaks even at ~5 frames per flush)
        self.small_flush = small_flush
        self.handed_back: list[np.ndarray] = []
        self.ctx = V.Context(device, max_arena=max(arena.nbytes, 1 << 16), max_pkts=capacity)
        if register:
            self.ctx.register(arena)
            if service_idle_us:
                # flushes go to the persistent service grid instead of a launch each
                self.ctx.set_service(service_idle_us)
        self.desc = np.zeros(capacity, V.DESC_DTYPE)
        self.pre = np.zeros(capacity, V.NAT_DTYPE)   # pre-images of NAT'd frames (F_PRE), by slot
        self.out = np.zeros(capacity, np.uint32)
        self.status = np.zeros(capacity, np.uint8)
        self.n = 0
        # GpuCsumBatch.stats(): tx_csum_skip is what IfaceStatistics.txCsumSkip counts with
        # INTEGRATION.md §3's diff (every frame whose sums Java left to someone else: the GPU or the
        # native path, XDPIface.java:117-120, 161-164); the rest say who took them.  Invariant:
        # deferred == gpu_handled + small_flush_handed_back + bad_desc_handed_back + pending.
        # pre_deferred: frames whose L4 sum is updated from a pre-image (a subset of deferred).
        self.stats = {"tx_pkts": 0, "tx_csum_skip": 0, "deferred": 0, "gpu_handled": 0, "tx_csum_gpu": 0,
                      "small_flush_handed_back": 0, "bad_desc_handed_back": 0, "handed_back": 0, "rejected": 0,
                      "flushes": 0, "pre_deferred": 0, "pre_full": 0}

    def _take(self, flags: int) -> bool:
        self.stats["tx_pkts"] += 1
        if flags == 0:
            return False
        self.stats["tx_csum_skip"] += 1
        return True

    def defer(self, l3_off: int, l3_len: int, l4_off: int, ver: int, proto: int, flags: int,
              pre=None, rx_status: int | None = None) -> bool:
        """Record a frame whose sums are dirty.  Returns False (nothing to do) when flags == 0.

        A NAT'd frame passes the `pre` image recorded before its setters ran
        (:func:`record_pre_image`) and its ingress verify status: when that proved the stored L4
        sum (:func:`pre_eligible`) the frame's L4 sum is updated from the pre-image (F_PRE: only its
        header is read at the flush), otherwise it is recomputed in full (`pre_full`)."""
        if not self._take(flags):
            return False
        if self.n == self.capacity:
            self.complete_tx()
        if pre is not None and flags & V.F_L4:
            if rx_status is not None and pre_eligible(rx_status):
                flags |= V.F_PRE
                self.pre[self.n] = pre
                self.stats["pre_deferred"] += 1
            else:
                self.stats["pre_full"] += 1
        self.desc[self.n] = (l3_off, l3_len, l4_off, ver, proto, flags, 0)
        self.n += 1
        self.stats["deferred"] += 1
        return True

    def defer_rx(self, pkt: RxPacket) -> bool:
        """GpuCsumBatch.defer for a received packet the vswitch is sending (XDPIface.sendPacket):
        its dirty sums from the setters that ran, the descriptor from the IP header fields, and
        F_PRE with the frame's ingress header sum when :func:`hsum_eligible` holds -- otherwise a
        frame that carries a record is summed in full (`pre_full`)."""
        flags = checksum_flags_for(pkt.ver == 4, pkt.ip_dirty, pkt.proto, pkt.l4_dirty)
        if not self._take(flags):
            return False
        d = egress_descriptor(self.arena[pkt.frame_off:pkt.frame_off + 512], pkt.frame_off, flags)
        if d is None:
            return False
        if self.n == self.capacity:
            self.complete_tx()
        if flags & V.F_L4 and int(pkt.csum_hsum["l2_len"]):
            if hsum_eligible(pkt.csum_status, pkt.csum_hsum, pkt.csum_l3, pkt.in_place, int(d["l3_off"]),
                             int(d["l3_ver"]), int(d["l4_proto"]), int(d["l3_len"]), int(d["l4_off"]), pkt.tcp_hlen()):
                d["flags"] |= V.F_PRE
                self.pre[self.n] = hsum_entry(pkt.csum_hsum)
                self.stats["pre_deferred"] += 1
            else:
                self.stats["pre_full"] += 1
        self.desc[self.n] = d
        self.n += 1
        self.stats["deferred"] += 1
        return True

    def defer_frame(self, frame_off: int, flags: int) -> bool:
        """GpuCsumBatch.defer for a frame at `frame_off` of the arena: the descriptor comes from
        the IP header fields (:func:`egress_descriptor`), never from the buffer length."""
        if not self._take(flags):
            return False
        d = egress_descriptor(self.arena[frame_off:frame_off + 64], frame_off, flags)
        if d is None:   # not IP: the chunk keeps its native flags
            return False
        if self.n == self.capacity:
            self.complete_tx()
        self.desc[self.n] = d
        self.n += 1
        self.stats["deferred"] += 1
        return True

    def complete_tx(self) -> int:
        """Iface.completeTx: flush every deferred checksum into the frames.  Returns the frames
        the GPU wrote.  A descriptor the kernel rejects (S_BAD_DESC: nothing written) is handed
        back with the small flushes (`handed_back`), as GpuCsumBatch.flush restores the chunk's
        native VP_CSUM_* flags: the frame is never sent with a stale sum."""
        if self.n == 0:
            return 0
        n = self.n
        if n < self.small_flush:
            self.handed_back.append(self.desc[:n].copy())
            self.stats["handed_back"] += n
            self.stats["small_flush_handed_back"] += n
            self.n = 0
            return 0
        if np.any(self.desc["flags"][:n] & V.F_PRE):
            t = self.ctx.submit_pre(self.arena, self.desc[:n], self.pre[:n], self.out[:n], self.status[:n], V.MODE_WRITE)
        else:
            t = self.ctx.submit(self.arena, self.desc[:n], self.out[:n], self.status[:n], V.MODE_WRITE)
        self.ctx.wait(t)
        bad = (self.status[:n] & V.S_BAD_DESC) != 0
        nbad = int(np.count_nonzero(bad))
        if nbad:
            self.handed_back.append(self.desc[:n][bad].copy())
            self.stats["handed_back"] += nbad
            self.stats["rejected"] += nbad
            self.stats["bad_desc_handed_back"] += nbad
        self.stats["tx_csum_gpu"] += n - nbad
        self.stats["gpu_handled"] += n - nbad
        self.stats["flushes"] += 1
        self.n = 0
        return n - nbad

    def close(self):
        self.ctx.close()


class FrameEgressBatch:
    """The egress seam without host-side descriptors (vpcsum_ctx_egress_frames, the Java form is
    VPCsum.egressFrames): ``defer`` records only what XDPIface.sendPacket already has -- the frame's
    umem offset and length (chunk.getAddr() + pkb.pktOff, pkb.pktBuf.length(): padding included)
    and its F_* flags -- and ``complete_tx`` has the GPU parse the frames with the vswitch's rules and
    write their sums in place, in one submission.  A frame the GPU refuses (not parsable as IP, or
    flags it cannot honour) is handed back untouched (``handed_back``).  With ``service_idle_us`` > 0
    flushes of up to 512 frames go to the low-latency service grid, which parses and sums each frame
    in one pass (no kernel launch)."""

    def __init__(self, arena: np.ndarray, capacity: int = 4096, device: int = 0, service_idle_us: int = 0):
        self.arena = arena
        self.capacity = capacity
        self.ctx = V.Context(device, max_arena=max(arena.nbytes, 1 << 16), max_pkts=capacity)
        self.ctx.register(arena)
        if service_idle_us:
            self.ctx.set_service(service_idle_us)
        self.off = np.zeros(capacity, np.uint64)
        self.len = np.zeros(capacity, np.uint32)
        self.flags = np.zeros(capacity, np.uint8)
        self.n = 0
        self.handed_back: list[tuple[int, int, int]] = []
        self.stats = {"tx_csum_skip": 0, "deferred": 0, "gpu_handled": 0, "bad_desc_handed_back": 0, "flushes": 0}

    def defer(self, frame_off: int, frame_len: int, flags: int) -> bool:
        if flags == 0:
            return False
        self.stats["tx_csum_skip"] += 1
        if self.n == self.capacity:
            self.complete_tx()
        self.off[self.n], self.len[self.n], self.flags[self.n] = frame_off, frame_len, flags
        self.n += 1
        self.stats["deferred"] += 1
        return True

    def complete_tx(self) -> int:
        n = self.n
        if n == 0:
            return 0
        _, st = self.ctx.egress_frames(self.arena, self.off[:n], self.len[:n], self.flags[:n])
        bad = np.nonzero(st & V.S_BAD_DESC)[0]
        self.handed_back += [(int(self.off[i]), int(self.len[i]), int(self.flags[i])) for i in bad]
        self.stats["gpu_handled"] += n - len(bad)
        self.stats["bad_desc_handed_back"] += len(bad)
        self.stats["flushes"] += 1
        self.n = 0
        return n - len(bad)

    def close(self):
        self.ctx.close()


CSUM_RECALC_NONE, CSUM_RECALC_ALL = "none", "all"     # CSumRecalcType.java:3-6


class RecalcDecision:
    """What DevInput does with each frame of a verified RX batch (see :func:`recalc_policy`)."""

    def __init__(self, ip_dirty: np.ndarray, l4_dirty: np.ndarray, drop: np.ndarray, stats: dict):
        self.ip_dirty, self.l4_dirty, self.drop, self.stats = ip_dirty, l4_dirty, drop, stats

    def egress_flags(self) -> np.ndarray:
        """F_IP / F_L4 per frame: the sums the egress batch must recompute for it (0: none)."""
        return np.where(self.ip_dirty, V.F_IP, 0).astype(np.uint8) | np.where(self.l4_dirty, V.F_L4, 0).astype(np.uint8)


def recalc_policy(status: np.ndarray, desc: np.ndarray, csum_recalc: str = CSUM_RECALC_ALL,
                  drop_bad: bool = False) -> RecalcDecision:
    """DevInput.handle's csum-recalc step (core/.../vswitch/node/DevInput.java:37-49) driven by the
    GPU's ingress verify of the batch (status from MODE_VERIFY over the parse descriptors `desc`).

    * ``none``: the stored sums are kept and nothing is marked dirty -- the reference's behaviour.
    * ``all``: the reference clears the L4 checksum of every IP packet and the IPv4 header
      checksum too (clearChecksum -> checksumSkipped, AbstractPacket.java:43-53), so egress
      recomputes every sum.  A sum that verified is recomputed to the value it already holds, so
      only the frames that fail need the dirty mark for the egress bytes to be identical: IPv4
      header dirty iff S_IP_OK is missing, L4 dirty iff S_L4_OK is missing -- which includes a UDP
      stored 0 (no checksum, S_UDP_NOCSUM), that Java's recompute replaces with a real sum.
      A frame the parser refused (S_BAD_DESC) is PacketBytes to Java (EthernetPacket.java:60-64):
      untouched.  Later rewrites (NAT, TTL) still dirty their sums through the setters.
    * ``drop_bad`` (a new capability, off by default; meant for NIC-facing interfaces, not for
      veth / tap peers whose host stack leaves CHECKSUM_PARTIAL sums): frames whose stored sums
      fail are dropped instead of repaired.  A UDP stored 0 is legal (RFC 768) and kept.

    The counts in ``stats`` are what an interface would add to its statistics
    (IfaceStatistics: rx csum errors / repaired / dropped)."""
    n = len(status)
    parsed = (status & V.S_BAD_DESC) == 0
    has_ip = parsed & ((desc["flags"] & V.F_IP) != 0)
    has_l4 = parsed & ((desc["flags"] & V.F_L4) != 0)
    ip_bad = has_ip & ((status & V.S_IP_OK) == 0)
    l4_bad = has_l4 & ((status & V.S_L4_OK) == 0)
    nocsum = has_l4 & ((status & V.S_UDP_NOCSUM) != 0)
    bad = ip_bad | (l4_bad & ~nocsum)
    none = np.zeros(n, bool)
    if csum_recalc not in (CSUM_RECALC_NONE, CSUM_RECALC_ALL):
        raise ValueError(f"csum-recalc {csum_recalc!r}: none | all (CSumRecalcType)")
    drop = bad if drop_bad else none
    if csum_recalc == CSUM_RECALC_ALL:
        ip_dirty, l4_dirty = ip_bad & ~drop, l4_bad & ~drop
    else:
        ip_dirty, l4_dirty = none, none.copy()
    stats = {"rx_frames": int(n), "rx_not_ip": int(np.count_nonzero(~parsed)),
             "rx_csum_bad": int(np.count_nonzero(bad)), "rx_udp_nocsum": int(np.count_nonzero(nocsum)),
             "rx_dropped": int(np.count_nonzero(drop)),
             "rx_marked_dirty": int(np.count_nonzero(ip_dirty | l4_dirty))}
    return RecalcDecision(ip_dirty, l4_dirty, drop, stats)


def verify_frames(ctx: "V.Context", arena: np.ndarray, desc: np.ndarray):
    """Ingress verify: (out, status) with S_IP_OK / S_L4_OK / S_UDP_NOCSUM per frame."""
    return ctx.run(arena, desc, V.MODE_VERIFY)


def descriptors_for_frames(arena_t, frame_off: np.ndarray, frame_len: np.ndarray,
                           flags: int = V.F_IP | V.F_L4, stream=None):
    """Parse Ethernet frames on the GPU into descriptors (vpcsum_parse_ether_async)."""
    import torch
    n = len(frame_off)
    d = torch.zeros(n * 16, dtype=torch.uint8, device=arena_t.device)
    st = torch.zeros(n, dtype=torch.uint8, device=arena_t.device)
    fo = torch.from_numpy(np.ascontiguousarray(frame_off, dtype=np.uint64)).to(arena_t.device)
    fl = torch.from_numpy(np.ascontiguousarray(frame_len, dtype=np.uint32)).to(arena_t.device)
    V.parse_ether(arena_t, fo, fl, n, d, st, flags, stream=stream)
    return d, st
