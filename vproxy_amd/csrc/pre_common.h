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
    uint32_t hs0, hs1;   // the entry's first 8 bytes: a vpcsum_hsum_t with VPCSUM_PRE_HSUM
};

__device__ __forceinline__ NatRw nat_rw4(const uint4 q) {
    NatRw r;
    r.src[0] = q.x; r.dst[0] = q.y;
    r.src[1] = r.src[2] = r.src[3] = r.dst[1] = r.dst[2] = r.dst[3] = 0;
    r.ports = q.z;
    r.mask = (int)(q.w & 0xff);
    r.ttl = (int)((q.w >> 8) & 0xff);   // rsv[0]: the VPCSUM_NAT_SET_TTL value
    r.hs0 = q.x;
    r.hs1 = q.y;
    return r;
}
__device__ __forceinline__ NatRw nat_rw6(const uint4 a, const uint4 b, const uint4 c) {
    NatRw r;
    r.src[0] = a.x; r.src[1] = a.y; r.src[2] = a.z; r.src[3] = a.w;
    r.dst[0] = b.x; r.dst[1] = b.y; r.dst[2] = b.z; r.dst[3] = b.w;
    r.ports = c.x;
    r.mask = (int)(c.y & 0xff);
    r.ttl = (int)((c.y >> 8) & 0xff);
    r.hs0 = a.x;
    r.hs1 = a.y;
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
    bool bad;        // a VPCSUM_PRE_HSUM record that does not describe this packet: nothing written
};

// The ingress header sum's words (vpcsum.h vpcsum_hsum_t) of a TCP / UDP packet at l3: the
// pseudo-header addresses (Utils.buildPseudoIPv4Header / IPv6Header, Utils.java:758-776: IPv4
// L3+12..19, IPv6 L3+8..39) and the L4 header's 16-bit words [0, hlen) except the checksum field
// `fld` -- every word of the L4 sum an in-place setter of the vswitch can change.  Folded end-around:
// 0 only when every word is 0 (the per-step fold of Utils.calculateChecksumIntermediate,
// Utils.java:783-797, gives the same value).
__device__ __forceinline__ uint32_t hdr_words_sum(const uint8_t* l3, int ver, int l4o, int hlen, int fld) {
    uint32_t s = 0;
    if (ver == 4) {
#pragma unroll
        for (int k = 0; k < 8; k += 2) s += ld16(l3 + 12 + k);
    } else {
#pragma unroll
        for (int k = 0; k < 32; k += 2) s += ld16(l3 + 8 + k);
    }
    for (int k = 0; k < hlen; k += 2)
        if (k != fld) s += ld16(l3 + l4o + k);
    return fold32(s);
}

// A parsed packet's vpcsum_hsum_t as two dwords (bytes 0..3, 4..7), from its L3 bytes at l3:
// {sum, l4_len} and {hlen, proto, ver, l2_len}; zeros (no record) unless it is TCP with a data
// offset of 20..seg bytes or UDP with its 8-B header in the segment.
__device__ __forceinline__ uint2 hsum_record(const uint8_t* l3, int ver, int proto, int len, int l4o, int l2) {
    const int seg = len - l4o;
    int hlen;
    if (proto == 6) {
        if (seg < 20) return make_uint2(0u, 0u);
        hlen = (l3[l4o + 12] >> 4) * 4;
        if (hlen < 20 || hlen > seg) return make_uint2(0u, 0u);
    } else if (proto == 17) {
        if (seg < 8) return make_uint2(0u, 0u);
        hlen = 8;
    } else {
        return make_uint2(0u, 0u);
    }
    const uint32_t s = hdr_words_sum(l3, ver, l4o, hlen, l4_field(proto));
    return make_uint2(s | ((uint32_t)seg << 16),
                      (uint32_t)hlen | ((uint32_t)proto << 8) | ((uint32_t)ver << 16) | ((uint32_t)l2 << 24));
}

// The L4 header length a VPCSUM_PRE_HSUM entry asks for (0: not such an entry); the window a
// pre-image kernel loads must reach l4o + this.
__device__ __forceinline__ int pre_hsum_hlen(const NatRw& r) {
    return (r.mask & VPCSUM_PRE_HSUM) ? (int)(r.hs1 & 0xff) : 0;
}

// RFC 1624's sum(~m + m') over the words a NAT entry records: the pseudo-header addresses of TCP /
// UDP and ICMPv6 (an ICMPv4 message has no pseudo header, inside IPv6 too) and the TCP / UDP ports
// (nat_setters); m from the entry, m' from the frame.
__device__ __forceinline__ uint32_t nat_words_diff(const uint8_t* l3, int ver, int proto, int l4o, const NatRw& r) {
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
    return diff;
}

// One packet's sums from its L3 header at l3 (its LDS window, or the frame on the byte path) and
// its pre-image r.
// hc_in >= 0: the stored L4 sum as it was before this flush (the service grid's host-captured copy,
// which keeps a re-run batch exact); otherwise it is read from the frame.
__device__ __forceinline__ PreSums pre_sums(const uint8_t* l3, int ver, int proto, int len, int l4o, bool do_ip,
                                            bool do_l4, const NatRw& r, int hc_in = -1) {
    PreSums o = {0u, 0u, false, false};
    if (do_ip) {   // Ipv4Packet.__updateChecksum: the header, its own field as 0 (Ipv4Packet.java:209-217)
        uint32_t s = 0;
        for (int k = 0; k < l4o; k += 2)
            if (k != 10) s += ld16(l3 + k);
        o.ipc = 0xffff - fold32(s);
    }
    if (!do_l4) return o;
    uint32_t diff = 0;
    if (r.mask & VPCSUM_PRE_HSUM) {
        // the header as one word: ~m = the recorded header sum's complement, m' = the same words
        // now.  Only for the packet the record describes: same version and protocol, same segment
        // length (the pseudo header's length word and the payload's place), same header length
        // (a TCP option list rebuilt in place would move the payload)
        const int hlen = (int)(r.hs1 & 0xff);
        const int cur = proto == 6 ? (l3[l4o + 12] >> 4) * 4 : 8;
        if ((r.hs1 >> 24) == 0 || (int)((r.hs1 >> 16) & 0xff) != ver || (int)((r.hs1 >> 8) & 0xff) != proto ||
            (int)(r.hs0 >> 16) != len - l4o || hlen != cur || hlen > len - l4o || !(proto == 6 || proto == 17)) {
            o.bad = true;
            return o;
        }
        diff = (~r.hs0 & 0xffff) + hdr_words_sum(l3, ver, l4o, hlen, l4_field(proto));
    } else {
        diff = nat_words_diff(l3, ver, proto, l4o, r);
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
