"""Host-side mirror of the vswitch seam that drives the GPU checksum (tests / tooling / Python
callers).  Same contract as java/io/vproxy/vpcsum/GpuCsumBatch.java:

* :func:`checksum_flags_for` -- SwitchUtils.checksumFlagsFor (core/.../vswitch/util/
  SwitchUtils.java:297-316): IP dirty -> F_IP (VP_CSUM_IP), upper layer dirty -> F_L4 (VP_CSUM_UP).
* :class:`EgressBatch` -- defer dirty frames at Iface.sendPacket, compute every deferred sum at
  Iface.completeTx in one GPU launch, written into the frames (XDPIface.java:100-178, 227-243).
* :func:`descriptors_for_frames` -- build descriptors for received Ethernet frames on the GPU
  (EthernetPacket/Ipv4Packet/Ipv6Packet.from rules) for ingress verify.

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
        self.out = np.zeros(capacity, np.uint32)
        self.status = np.zeros(capacity, np.uint8)
        self.n = 0
        self.stats = {"tx_pkts": 0, "tx_csum_gpu": 0, "flushes": 0}

    def defer(self, l3_off: int, l3_len: int, l4_off: int, ver: int, proto: int, flags: int) -> bool:
        """Record a frame whose sums are dirty.  Returns False (nothing to do) when flags == 0."""
        self.stats["tx_pkts"] += 1
        if flags == 0:
            return False
        if self.n == self.capacity:
            self.complete_tx()
        self.desc[self.n] = (l3_off, l3_len, l4_off, ver, proto, flags, 0)
        self.n += 1
        return True

    def complete_tx(self) -> int:
        """Iface.completeTx: flush every deferred checksum into the frames."""
        if self.n == 0:
            return 0
        n = self.n
        if n < self.small_flush:
            self.handed_back.append(self.desc[:n].copy())
            self.stats["handed_back"] = self.stats.get("handed_back", 0) + n
            self.n = 0
            return 0
        t = self.ctx.submit(self.arena, self.desc[:n], self.out[:n], self.status[:n], V.MODE_WRITE)
        self.ctx.wait(t)
        bad = int(np.count_nonzero(self.status[:n] & V.S_BAD_DESC))
        if bad:
            raise V.VpcsumError(f"{bad} descriptors rejected by the checksum kernel")
        self.stats["tx_csum_gpu"] += n
        self.stats["flushes"] += 1
        self.n = 0
        return n

    def close(self):
        self.ctx.close()


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
