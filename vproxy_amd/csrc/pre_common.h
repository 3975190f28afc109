// pre_common.h -- device code shared by nat.hip (the NAT kernels, k_pre) and kernels.hip (the
// service grid's pre-image frames): the decoded rewrite / pre-image entry, the NAT descriptor
// rules, and one packet's sums from its pre-image (RFC 1624 eqn. 3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "vpcsum.h"
#include "device_common.h"

namespace vpcsum {

// One packet's rewrite, decoded from either entry format.  Address bytes stay in load order
// (byte i of the address = byte i & 3 of word i >> 2).
struct NatRw {
    uint32_t src[4], dst[4];
    uint32_t ports;   // bytes 0..1 source port, 2..3 destination port (network order)
    int mask, ttl;
};

__device__ __forceinline__ NatRw nat_rw4(const uint4 q) {
    NatRw r;
    r.src[0] = q.x; r.dst[0] = q.y;
    r.src[1] = r.src[2] = r.src[3] = r.dst[1] = r.dst[2] = r.dst[3] = 0;
    r.ports = q.z;
    r.mask = (int)(q.w & 0xff);
    r.ttl = (int)((q.w >> 8) & 0xff);   // rsv[0]: the VPCSUM_NAT_SET_TTL value
    return r;
}
__device__ __forceinline__ NatRw nat_rw6(const uint4 a, const uint4 b, const uint4 c) {
    NatRw r;
    r.src[0] = a.x; r.src[1] = a.y; r.src[2] = a.z; r.src[3] = a.w;
    r.dst[0] = b.x; r.dst[1] = b.y; r.dst[2] = b.z; r.dst[3] = b.w;
    r.ports = c.x;
    r.mask = (int)(c.y & 0xff);
    r.ttl = (int)((c.y >> 8) & 0xff);
    return r;
}
// big-endian 16-bit word k (bytes 2k, 2k+1) of an address / of the port pair
__device__ __forceinline__ uint32_t rw_word(const uint32_t* a, int k) {
    const uint32_t w = a[k >> 1] >> ((k & 1) * 16);
    return ((w & 0xff) << 8) | ((w >> 8) & 0xff);
}

// Descriptor checks shared by both kernels; fmt 0 and 2 entries carry IPv4 addresses only.
__device__ __forceinline__ bool nat_desc_ok(uint64_t off, int len, int l4o, int ver, uint64_t arena_len, int fmt) {
    if (off > arena_len || (uint64_t)len > arena_len - off) return false;
    if (ver == 4) return len >= 20 && l4o >= 20 && l4o <= len && !(l4o & 3);
    if (ver == 6) return fmt == 1 && len >= 40 && l4o >= 40 && l4o <= len;
    return false;
}
__device__ __forceinline__ bool nat_l4sum(int ver, int proto, int len, int l4o) {
    const int fld = l4_field(proto);
    return fld >= 0 && !(ver == 4 && proto == 58) && len - l4o >= fld + 2;
}

// The F_PRE descriptor rules: F_L4 and / or F_IP, nothing else but F_PRE (no F_L4P / F_RAW), F_IP on
// IPv4 only, nat_desc_ok's bounds and header rules (fmt 0, 16-B entries: IPv4 only), and with F_L4
// an L4 checksum field inside the segment.
__device__ __forceinline__ bool pre_desc_ok(const uint4 dv, uint64_t arena_len, int fmt) {
    const uint64_t off = (uint64_t)dv.x | ((uint64_t)dv.y << 32);
    const int len = dv.z & 0xffff, l4o = dv.z >> 16;
    const int ver = dv.w & 0xff, proto = (dv.w >> 8) & 0xff, fl = (dv.w >> 16) & 0xff;
    if ((fl & ~(VPCSUM_F_IP | VPCSUM_F_L4 | VPCSUM_F_PRE)) || !(fl & (VPCSUM_F_IP | VPCSUM_F_L4))) return false;
    if ((fl & VPCSUM_F_IP) && ver != 4) return false;
    return nat_desc_ok(off, len, l4o, ver, arena_len, fmt) && (!(fl & VPCSUM_F_L4) || nat_l4sum(ver, proto, len, l4o));
}

struct PreSums {
    uint32_t ipc, l4c;
    bool udp_full;   // UDP stored 0: the caller sums the segment (udp_full_sum)
};

// One packet's sums from its L3 header at l3 (its LDS window, or the frame on the byte path) and
// its pre-image r.
// hc_in >= 0: the stored L4 sum as it was before this flush (the service grid's host-captured copy,
// which keeps a re-run batch exact); otherwise it is read from the frame.
__device__ __forceinline__ PreSums pre_sums(const uint8_t* l3, int ver, int proto, int l4o, bool do_ip, bool do_l4,
                                            const NatRw& r, int hc_in = -1) {
    PreSums o = {0u, 0u, false};
    if (do_ip) {   // Ipv4Packet.__updateChecksum: the header, its own field as 0 (Ipv4Packet.java:209-217)
        uint32_t s = 0;
        for (int k = 0; k < l4o; k += 2)
            if (k != 10) s += ld16(l3 + k);
        o.ipc = 0xffff - fold32(s);
    }
    if (!do_l4) return o;
    // the L4 sum's words a rewrite changes: the pseudo-header addresses of TCP / UDP and ICMPv6 (an
    // ICMPv4 message has no pseudo header, inside IPv6 too) and the TCP / UDP ports (nat_setters)
    const bool ports = proto == 6 || proto == 17;
    const bool addr = ports || (ver == 6 && proto == 58);
    uint32_t diff = 0;
    // (constant trip counts: a runtime word index into the entry's registers would put it in scratch)
    if (addr && ver == 4) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (r.mask & VPCSUM_NAT_SRC) diff += (~rw_word(r.src, k) & 0xffff) + ld16(l3 + 12 + 2 * k);
            if (r.mask & VPCSUM_NAT_DST) diff += (~rw_word(r.dst, k) & 0xffff) + ld16(l3 + 16 + 2 * k);
        }
    } else if (addr) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (r.mask & VPCSUM_NAT_SRC) diff += (~rw_word(r.src, k) & 0xffff) + ld16(l3 + 8 + 2 * k);
            if (r.mask & VPCSUM_NAT_DST) diff += (~rw_word(r.dst, k) & 0xffff) + ld16(l3 + 24 + 2 * k);
        }
    }
    if (ports) {
        if (r.mask & VPCSUM_NAT_SPORT) diff += (~rw_word(&r.ports, 0) & 0xffff) + ld16(l3 + l4o);
        if (r.mask & VPCSUM_NAT_DPORT) diff += (~rw_word(&r.ports, 1) & 0xffff) + ld16(l3 + l4o + 2);
    }
    const uint32_t hc = hc_in >= 0 ? (uint32_t)hc_in : ld16(l3 + l4o + l4_field(proto));
    if (proto == 17 && hc == 0) {   // "no checksum": Java's recompute writes a real one (UdpPacket.java:136-164)
        o.udp_full = true;
        return o;
    }
    uint32_t c = ~fold32((~hc & 0xffff) + fold32(diff)) & 0xffff;
    if (proto == 17 && c == 0) c = 0xffff;
    o.l4c = c;
    return o;
}

}  // namespace vpcsum
