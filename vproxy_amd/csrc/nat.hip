// nat.hip -- K5 of libvpcsum (gfx950): NAT / TTL rewrites with the checksum update, in place.
//
// Java writes the new bytes through the setters and marks the sums dirty, and the next
// getRawPacket(0) recomputes the dirty sums in full:
//   SwitchUtils.applyNat                   core/.../vswitch/util/SwitchUtils.java:522-542
//   Ipv4Packet.setSrc / setDst / setTtl    base/.../vpacket/Ipv4Packet.java:401-407, 433-458
//     pseudoHeaderChanges (TCP / UDP)      Ipv4Packet.java:236-240
//   Ipv6Packet.setSrc / setDst             Ipv6Packet.java:374-396 (setHopLimit :354-359 marks
//     pseudoHeaderChanges (ICMP, TCP, UDP) nothing dirty: no sum covers the hop limit)
//                                          Ipv6Packet.java:238-242
//   TcpPacket / UdpPacket.setSrcPort / setDstPort  TcpPacket.java:31-51, UdpPacket.java:188-209
// RFC 1624 eqn. 3, HC' = ~(~HC + ~m + m'), is bit-identical to that full recompute whenever the
// incoming checksum is correct; UDP with stored 0 is recomputed in full.
// VPCSUM_NAT_STRICT_JAVA rewrites only and hands the dirty flags to the checksum kernel, which
// recomputes in full: identical to Java for any input.
//
// Three rewrite-entry formats: vpcsum_nat4_t (16 B, IPv4 only: BASELINE config C5's 72 B/packet),
// vpcsum_nat_t (48 B, IPv4 and IPv6), and vpcsum_nat4_rec_t (FMT 2: the descriptor and the IPv4
// entry in one 32-B record, so a packet's rewrite comes from one read stream instead of two).  One lane per packet for the rewrite; the default wide
// kernel (k_natq) moves the header windows in and out by quads of lanes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include "vpcsum.h"
#include "internal.h"
#include "device_common.h"
#include "pre_common.h"

namespace vpcsum {

// What a packet's rewrite did: RFC 1624 differences (sums of ~m + m'), Java's dirty flags, and the
// byte range [lo, hi) (relative to the L3 start) that changed.
struct NatAcc {
    uint32_t ip_diff, l4_diff;
    bool ip_dirty, l4_dirty, l4_touch;
    int lo, hi;
};

// Overwrites the big-endian word at w[q] with mn; returns its RFC 1624 difference ~m + m'.  (The
// callers add it to the sums it changes by value: a pointer into NatAcc put the struct in scratch
// memory, 124 scratch accesses per packet set in k_natq)
__device__ __forceinline__ uint32_t nat_word(uint8_t* w, int q, uint32_t mn) {
    const uint32_t m = ((uint32_t)w[q] << 8) | w[q + 1];
    w[q] = (uint8_t)(mn >> 8);
    w[q + 1] = (uint8_t)mn;
    return (~m & 0xffff) + mn;
}
__device__ __forceinline__ void grow(NatAcc& a, int lo, int hi) {
    a.lo = min(a.lo, lo);
    a.hi = max(a.hi, hi);
}

// The setters on the packet whose L3 header is w[0..len) (w: an LDS window or the frame itself).
// l4sum: the L4 checksum field exists (the segment holds it).
__device__ __forceinline__ NatAcc nat_setters(uint8_t* w, int ver, int proto, int len, int l4o, bool l4sum,
                                             const NatRw& r) {
    NatAcc a = {0u, 0u, false, false, false, 1 << 20, 0};
    // which L4 sums the pseudo-header addresses dirty: TCP / UDP under IPv4, also ICMP / ICMPv6
    // under IPv6; an ICMPv4 message has no pseudo header, so its sum does not change
    const bool addr_dirty = l4sum && (proto == 6 || proto == 17 || (ver == 6 && (proto == 58 || proto == 1)));
    const bool addr_sum = addr_dirty && proto != 1;
    const uint32_t l4m = addr_sum ? 0xffffffffu : 0u;   // address differences into the L4 sum too
    if (ver == 4) {
        if (r.mask & VPCSUM_NAT_SRC) {
            for (int k = 0; k < 2; ++k) {
                const uint32_t dd = nat_word(w, 12 + 2 * k, rw_word(r.src, k));
                a.ip_diff += dd;
                a.l4_diff += dd & l4m;
            }
            a.ip_dirty = true; a.l4_dirty |= addr_dirty; a.l4_touch |= addr_sum;
            grow(a, 12, 16);
        }
        if (r.mask & VPCSUM_NAT_DST) {
            for (int k = 0; k < 2; ++k) {
                const uint32_t dd = nat_word(w, 16 + 2 * k, rw_word(r.dst, k));
                a.ip_diff += dd;
                a.l4_diff += dd & l4m;
            }
            a.ip_dirty = true; a.l4_dirty |= addr_dirty; a.l4_touch |= addr_sum;
            grow(a, 16, 20);
        }
        if (r.mask & VPCSUM_NAT_SET_TTL) {   // setTtl(ttl)
            a.ip_diff += nat_word(w, 8, ((uint32_t)r.ttl << 8) | w[9]);
            a.ip_dirty = true;
            grow(a, 8, 9);
        }
        if (r.mask & VPCSUM_NAT_DEC_TTL) {   // IPInputRoute: setTtl(ttl - 1)
            a.ip_diff += nat_word(w, 8, ((uint32_t)((w[8] - 1) & 0xff) << 8) | w[9]);
            a.ip_dirty = true;
            grow(a, 8, 9);
        }
    } else {
        if (r.mask & VPCSUM_NAT_SRC) {
            for (int k = 0; k < 8; ++k) a.l4_diff += nat_word(w, 8 + 2 * k, rw_word(r.src, k)) & l4m;
            a.l4_dirty |= addr_dirty; a.l4_touch |= addr_sum;
            grow(a, 8, 24);
        }
        if (r.mask & VPCSUM_NAT_DST) {
            for (int k = 0; k < 8; ++k) a.l4_diff += nat_word(w, 24 + 2 * k, rw_word(r.dst, k)) & l4m;
            a.l4_dirty |= addr_dirty; a.l4_touch |= addr_sum;
            grow(a, 24, 40);
        }
        if (r.mask & VPCSUM_NAT_SET_TTL) { w[7] = (uint8_t)r.ttl; grow(a, 7, 8); }          // setHopLimit
        if (r.mask & VPCSUM_NAT_DEC_TTL) { w[7] = (uint8_t)(w[7] - 1); grow(a, 7, 8); }
    }
    if (l4sum && (proto == 6 || proto == 17)) {
        if (r.mask & VPCSUM_NAT_SPORT) {
            a.l4_diff += nat_word(w, l4o, rw_word(&r.ports, 0));
            a.l4_dirty = a.l4_touch = true;
            grow(a, l4o, l4o + 2);
        }
        if (r.mask & VPCSUM_NAT_DPORT) {
            a.l4_diff += nat_word(w, l4o + 2, rw_word(&r.ports, 1));
            a.l4_dirty = a.l4_touch = true;
            grow(a, l4o + 2, l4o + 4);
        }
    }
    return a;
}

// IPInputRoute.java:81-88: a packet whose TTL / hop limit is <= 1 is dropped (and answered with
// ICMP time exceeded), never decremented: DEC_TTL refuses it -- nothing written -- rather than
// storing 0 or 255.  The value checked is the one DEC_TTL would decrement (after SET_TTL).
__device__ __forceinline__ bool nat_ttl_expired(const uint8_t* l3, int ver, const NatRw& r) {
    if (!(r.mask & VPCSUM_NAT_DEC_TTL)) return false;
    const int t = (r.mask & VPCSUM_NAT_SET_TTL) ? r.ttl : (int)l3[ver == 4 ? 8 : 7];
    return t <= 1;
}
constexpr uint32_t kNatExpired = VPCSUM_S_BAD_DESC | VPCSUM_S_TTL_EXPIRED;

// RFC 1624 eqn. 3 on the fields of w.  Returns true when the L4 sum is a UDP "no checksum" (stored
// 0): Java recomputes it in full (UdpPacket.java:136-164), done by nat_udp_full once the rewritten
// header is in memory.
__device__ __forceinline__ bool nat_rfc1624(uint8_t* w, int proto, int l4o, int fld, NatAcc& a) {
    if (a.ip_dirty) {
        const uint32_t hc = ((uint32_t)w[10] << 8) | w[11];
        const uint32_t c = ~fold32((~hc & 0xffff) + fold32(a.ip_diff)) & 0xffff;
        w[10] = (uint8_t)(c >> 8); w[11] = (uint8_t)c;
        grow(a, 10, 12);
    }
    if (a.l4_touch) {
        const int f = l4o + fld;
        const uint32_t hc = ((uint32_t)w[f] << 8) | w[f + 1];
        if (proto == 17 && hc == 0) return true;
        uint32_t c = ~fold32((~hc & 0xffff) + fold32(a.l4_diff)) & 0xffff;
        if (proto == 17 && c == 0) c = 0xffff;
        w[f] = (uint8_t)(c >> 8); w[f + 1] = (uint8_t)c;
        grow(a, f, f + 2);
    }
    return false;
}

// Folded LE-absolute sum of bytes [lo, hi) (absolute addresses) minus a 2-byte field, one lane.
__device__ uint32_t lane_sum_range(const uint8_t* lo_p, const uint8_t* hi_p, const uint8_t* fld_p) {
    const uintptr_t lo = (uintptr_t)lo_p, hi = (uintptr_t)hi_p, fa = (uintptr_t)fld_p;
    const uintptr_t a = lo & ~(uintptr_t)3;
    uint64_t acc = 0;
    for (uintptr_t d = a; d < hi; d += 4) {
        const uint32_t v = *(const __attribute__((address_space(1))) uint32_t*)d;
        const int rd = (int)(d - a);
        uint32_t m = bmask(rd, (int)(lo - a), (int)(hi - a));
        if (fld_p) m &= ~bmask(rd, (int)(fa - a), (int)(fa - a) + 2);
        acc += v & m;
    }
    return fold64(acc);
}

// Full UDP sum from memory (the stored-0 case): pseudo header (IPv4 12..20 / IPv6 8..40, proto 17,
// the L4 length as 16 / 32 bits) + the segment with the field excluded.
__device__ uint32_t udp_full_sum(const uint8_t* l3, int ver, int len, int l4o) {
    const uint8_t* l4p = l3 + l4o;
    const uint32_t seg = orient(lane_sum_range(l4p, l3 + len, l4p + 6), (int)((uintptr_t)l4p & 1));
    const uint32_t ps = orient(lane_sum_range(l3 + (ver == 4 ? 12 : 8), l3 + (ver == 4 ? 20 : 40), nullptr),
                               (int)((uintptr_t)l3 & 1));
    const uint32_t l4len = (uint32_t)(len - l4o);
    uint32_t c = 0xffff - fold32(seg + ps + 17u + (l4len & 0xffff) + (l4len >> 16));
    if (c == 0) c = 0xffff;
    return c;
}
__device__ void nat_udp_full(uint8_t* l3, int ver, int len, int l4o) { st16(l3 + l4o + 6, udp_full_sum(l3, ver, len, l4o)); }

// Packet p's descriptor and rewrite.  FMT 2 (vpcsum_nat4_rec_t): desc and rw both point at the
// records, the descriptor is the record's first 16 B and the IPv4 entry its second.
template <int FMT>
__device__ __forceinline__ uint4 nat_load_desc(const uint4* desc, uint32_t p) {
    return FMT == 2 ? desc[2 * (size_t)p] : desc[p];
}
template <int FMT>
__device__ __forceinline__ NatRw nat_load_rw(const void* rw, uint32_t p) {
    if (FMT == 0) return nat_rw4(((const uint4*)rw)[p]);
    if (FMT == 2) return nat_rw4(((const uint4*)rw)[2 * (size_t)p + 1]);
    const uint4* q = (const uint4*)rw + 3 * (size_t)p;
    return nat_rw6(q[0], q[1], q[2]);
}

// One packet with byte accesses straight on the frame (IPv4 options / IPv6 extension headers
// beyond the wide window, arenas the buffer path cannot address, or nat_mode bit 8).  Returns the
// packet's result byte: its status (S_DONE / S_BAD_DESC) or, in strict mode, Java's dirty flags
// for the checksum kernel (kFlagRejected for a rejected descriptor).
template <int FMT>
__device__ uint32_t nat_scalar(uint8_t* __restrict__ arena, uint64_t arena_len, const uint4 dv, const NatRw& r,
                               bool strict) {
    const uint64_t off = (uint64_t)dv.x | ((uint64_t)dv.y << 32);
    const int len = dv.z & 0xffff, l4o = dv.z >> 16;
    const int ver = dv.w & 0xff, proto = (dv.w >> 8) & 0xff;
    if (!nat_desc_ok(off, len, l4o, ver, arena_len, FMT)) return strict ? kFlagRejected : VPCSUM_S_BAD_DESC;
    uint8_t* l3 = arena + off;
    if (nat_ttl_expired(l3, ver, r)) return strict ? kFlagRejected : kNatExpired;
    const bool l4sum = nat_l4sum(ver, proto, len, l4o);
    NatAcc a = nat_setters(l3, ver, proto, len, l4o, l4sum, r);
    if (strict) return (a.ip_dirty ? VPCSUM_F_IP : 0) | (a.l4_dirty ? VPCSUM_F_L4 : 0);
    if (nat_rfc1624(l3, proto, l4o, l4_field(proto), a)) nat_udp_full(l3, ver, len, l4o);
    return VPCSUM_S_DONE;
}

// The result bytes of 64 consecutive packets (one per lane; every lane of the wave calls this):
// lanes 4k gather the bytes of lanes 4k..4k+3 and store one dword, so the wave writes 64 B in one
// request instead of byte stores the memory path splits per dword (measured: 15 B of writes per
// packet for the 1-B status alone).  p = this lane's packet, 4-aligned for lane 4k.
__device__ __forceinline__ void store_bytes_packed(uint8_t* __restrict__ dst, uint32_t p, uint32_t n, uint32_t v) {
    v &= 0xff;
    const uint32_t b1 = (uint32_t)__shfl_down((int)v, 1, 64), b2 = (uint32_t)__shfl_down((int)v, 2, 64),
                   b3 = (uint32_t)__shfl_down((int)v, 3, 64);
    if ((threadIdx.x & 3) == 0 && p < n) {
        const uint32_t packed = v | ((b1 & 0xff) << 8) | ((b2 & 0xff) << 16) | (b3 << 24);
        if (p + 4 <= n && !((uintptr_t)(dst + p) & 3)) {
            *(__attribute__((address_space(1))) uint32_t*)(dst + p) = packed;
        } else {   // shifts, not an indexed array: no scratch
            for (uint32_t k = 0; k < 4 && p + k < n; ++k) dst[p + k] = (uint8_t)(packed >> (8 * k));
        }
    }
}

template <int FMT>
__global__ __launch_bounds__(256) void k_nat(uint8_t* __restrict__ arena, uint64_t arena_len,
                                            const uint4* __restrict__ desc, const void* __restrict__ rw, uint32_t n,
                                            uint8_t* __restrict__ status, uint8_t* __restrict__ flags_out, int strict) {
    uint8_t* res = strict ? flags_out : status;
    // grid-stride in whole waves, so every lane reaches the packed result store together
    for (uint32_t p0 = blockIdx.x * blockDim.x; p0 < n; p0 += gridDim.x * blockDim.x) {
        const uint32_t p = p0 + threadIdx.x;
        uint32_t v = 0;
        if (p < n) v = nat_scalar<FMT>(arena, arena_len, nat_load_desc<FMT>(desc, p), nat_load_rw<FMT>(rw, p), strict != 0);
        if (res) store_bytes_packed(res, p, n, v);
    }
}

// Wide form: the window [align16(L3), align16(L3) + 96) holding every byte a rewrite touches --
// the header, the ports and the L4 checksum field of IPv4 with options or IPv6 without extension
// headers -- is read with up to six 16-B global loads (only the chunks the packet needs), staged
// in this lane's LDS slot, rewritten there with byte-addressed LDS ops (the window's offset
// differs per packet), and the changed range is stored back as ONE run of dwordx4 / x2 / dword
// stores (bytewise only where it would pass the packet end: the next bytes may be another
// packet's).  W packets per lane and iteration keep W windows in flight.
constexpr int kNatChunks = 6;                   // window: 96 B

// Store back bytes [lo, hi) of the packet (relative to L3; the window holds it at w + r0, base is
// the window's 16-B aligned global address) as one run of dwords, widest first, bytewise only
// where a dword would pass the packet end (the next bytes may be another packet's).
__device__ __forceinline__ void nat_store_range(uint8_t* base, const uint32_t* slot, const uint8_t* w, int r0,
                                                int len, int lo, int hi) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef unsigned int v2u __attribute__((ext_vector_type(2)));
    typedef __attribute__((address_space(1))) uint32_t g32;
    if (hi <= lo) return;
    const int lim = r0 + len;
    int j = (r0 + lo) >> 2;
    const int je = (r0 + hi + 3) >> 2;
    const int jfull = lim >> 2;   // dwords below this lie inside the packet
    while (j < je) {
        uint8_t* dst = base + 4 * j;
        if (!(j & 3) && j + 4 <= je && j + 4 <= jfull) {
            const v4u q = {slot[j], slot[j + 1], slot[j + 2], slot[j + 3]};
            *(__attribute__((address_space(1))) v4u*)dst = q;
            j += 4;
        } else if (!(j & 1) && j + 2 <= je && j + 2 <= jfull) {
            const v2u q = {slot[j], slot[j + 1]};
            *(__attribute__((address_space(1))) v2u*)dst = q;
            j += 2;
        } else if (j + 1 <= jfull) {
            *(g32*)dst = slot[j];
            j += 1;
        } else {
            for (int q = 4 * j; q < lim; ++q) base[q] = w[q];
            j += 1;
        }
    }
}

// PROBE: the same loads, LDS staging and stores with no rewrite -- the changed range is set to
// what a rewrite of both addresses and ports produces ([10, L4 checksum end) for IPv4, [8, ..) for
// IPv6) and the window is stored back unchanged.  It prices NAT's access pattern (the "pattern
// ceiling" of BASELINE config C5): a rewrite cannot run faster than its own memory operations.
// CH: window chunks (16 B each).  6 hold any header the wide path takes (IPv4 with options, IPv6
// without extension headers, any alignment); 4 hold IPv4 + TCP / UDP without options at any L3
// alignment (an umem frame puts L3 at chunk offset 14: 14 + 38 <= 64), and need 16 fewer VGPRs
// at W = 2.  A packet whose header does not fit takes the byte-access path.
template <int FMT, bool STRICT, int W, bool PROBE = false, int CH = kNatChunks>
__global__ __launch_bounds__(256) void k_natw(uint8_t* __restrict__ arena, uint64_t arena_len,
                                             const uint4* __restrict__ desc, const void* __restrict__ rw, uint32_t n,
                                             uint8_t* __restrict__ status, uint8_t* __restrict__ flags_out) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) const v4u gv4u;
    constexpr int kSlotDw = 4 * CH + 1;   // LDS slot per lane: an odd dword stride (no bank conflicts)
    __shared__ uint32_t s_win[256 * kSlotDw];
    uint32_t* slot = &s_win[threadIdx.x * kSlotDw];
    uint8_t* w = (uint8_t*)slot;
    const uint32_t T = gridDim.x * blockDim.x;
    for (uint32_t p0 = blockIdx.x * blockDim.x + threadIdx.x; p0 < n; p0 += W * T) {
        uint4 dv[W];
        NatRw rr[W];
        int wend[W];
        uint4 v[W][CH];
#pragma unroll
        for (int i = 0; i < W; ++i) {
            const uint32_t p = p0 + i * T;
            dv[i] = p < n ? nat_load_desc<FMT>(desc, p) : make_uint4(0, 0, 0, 0);
            rr[i] = nat_load_rw<FMT>(rw, p < n ? p : 0);
        }
#pragma unroll
        for (int i = 0; i < W; ++i) {
            const uint32_t p = p0 + i * T;
            const uint64_t off = (uint64_t)dv[i].x | ((uint64_t)dv[i].y << 32);
            const int len = dv[i].z & 0xffff, l4o = dv[i].z >> 16;
            const int ver = dv[i].w & 0xff, proto = (dv[i].w >> 8) & 0xff;
            const bool ok = p < n && nat_desc_ok(off, len, l4o, ver, arena_len, FMT);
            // the window starts at the 16-B aligned address below the L3 header (absolute: any
            // arena alignment, any arena size -- 64-bit global loads)
            const uintptr_t la = ok ? (uintptr_t)(arena + off) : 0;
            const int r0 = (int)(la & 15);
            int need = ver == 4 ? 20 : 40;
            if (nat_l4sum(ver, proto, len, l4o)) need = max(need, l4o + l4_field(proto) + 2);
            wend[i] = ok && r0 + need <= 16 * CH ? r0 + need : 0;   // 0: the byte-access path
            const uintptr_t base = la - (uintptr_t)r0;
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                // only the chunks the packet needs: all lie in its 16-B blocks, which never cross
                // a page, so none reads past the arena's last page
                v4u x = {0u, 0u, 0u, 0u};
                if ((k << 4) < wend[i]) x = *(gv4u*)(base + 16 * k);
                v[i][k] = make_uint4(x.x, x.y, x.z, x.w);
            }
        }
        uint32_t res[W];
#pragma unroll
        for (int i = 0; i < W; ++i) {
            const uint32_t p = p0 + i * T;
            res[i] = 0;
            if (p >= n) continue;
            if (!wend[i]) {
                if (!PROBE) res[i] = nat_scalar<FMT>(arena, arena_len, dv[i], rr[i], STRICT);
                continue;
            }
            const uint64_t off = (uint64_t)dv[i].x | ((uint64_t)dv[i].y << 32);
            const int len = dv[i].z & 0xffff, l4o = dv[i].z >> 16;
            const int ver = dv[i].w & 0xff, proto = (dv[i].w >> 8) & 0xff;
            const uintptr_t la = (uintptr_t)(arena + off);
            const int r0 = (int)(la & 15);
            uint8_t* base = (uint8_t*)(la - (uintptr_t)r0);
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                if ((k << 4) < wend[i]) {
                    slot[4 * k] = v[i][k].x; slot[4 * k + 1] = v[i][k].y;
                    slot[4 * k + 2] = v[i][k].z; slot[4 * k + 3] = v[i][k].w;
                }
            }
            uint8_t* l3w = w + r0;
            if (PROBE) {
                int hi = ver == 4 ? 20 : 40;
                if (nat_l4sum(ver, proto, len, l4o)) hi = max(hi, l4o + l4_field(proto) + 2);
                nat_store_range(base, slot, w, r0, len, ver == 4 ? 10 : 8, hi);
                res[i] = VPCSUM_S_DONE;
                continue;
            }
            if (nat_ttl_expired(l3w, ver, rr[i])) {
                res[i] = STRICT ? kFlagRejected : kNatExpired;
                continue;
            }
            NatAcc a = nat_setters(l3w, ver, proto, len, l4o, nat_l4sum(ver, proto, len, l4o), rr[i]);
            const bool udp_zero = !STRICT && nat_rfc1624(l3w, proto, l4o, l4_field(proto), a);
            nat_store_range(base, slot, w, r0, len, a.lo, a.hi);
            if (STRICT) {
                res[i] = (a.ip_dirty ? VPCSUM_F_IP : 0) | (a.l4_dirty ? VPCSUM_F_L4 : 0);
                continue;
            }
            if (udp_zero) nat_udp_full(arena + off, ver, len, l4o);
            res[i] = VPCSUM_S_DONE;
        }
        uint8_t* dst = STRICT ? flags_out : status;
        if (dst) {
#pragma unroll
            for (int i = 0; i < W; ++i) store_bytes_packed(dst, p0 + i * T, n, res[i]);
        }
    }
}

// Store bytes [s, e) of window chunk c (window coordinates; bytes before r0 and at or past lim are
// not the packet's and are left alone) from the packet's LDS slot to base + 16c: the whole chunk
// as one dwordx4 when it lies inside the packet (its unchanged bytes rewritten with their own
// values), else dwordx2 / dword pieces, bytes only at the packet end.
__device__ __forceinline__ void natq_store_chunk(uint8_t* base, const uint32_t* slot, int c, int s, int e, int lim,
                                                 int r0) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef unsigned int v2u __attribute__((ext_vector_type(2)));
    typedef __attribute__((address_space(1))) uint32_t g32;
    const int cs = max(s, 16 * c), ce = min(e, 16 * c + 16);
    if (ce <= cs) return;
    int j = cs >> 2;
    const int je = (ce + 3) >> 2;
    const int jfull = lim >> 2;   // dwords below this lie inside the packet
    if (16 * c >= r0 && 16 * c + 16 <= lim) {
        const uint32_t* q = slot + 4 * c;
        *(__attribute__((address_space(1))) v4u*)(base + 16 * c) = v4u{q[0], q[1], q[2], q[3]};
        return;
    }
    while (j < je) {
        uint8_t* dst = base + 4 * j;
        if (!(j & 1) && j + 2 <= je && j + 2 <= jfull) {
            *(__attribute__((address_space(1))) v2u*)dst = v2u{slot[j], slot[j + 1]};
            j += 2;
        } else if (j + 1 <= jfull) {
            *(g32*)dst = slot[j];
            j += 1;
        } else {
            const uint8_t* wb = (const uint8_t*)slot;
            for (int q = 4 * j; q < lim; ++q) base[q] = wb[q];
            j += 1;
        }
    }
}

// Quad form of k_natw: the same per-lane rewrite on an LDS window, but the wave's header windows
// are loaded and stored back by quads -- lane L moves chunk L & 3 of packet 16u + (L >> 2) in
// instruction u -- so one vector-memory instruction touches 16 frames' lines instead of 64.  The
// NAT access pattern (one 128-B line read and a 32..64-B write per 2-KB frame) measured 20.5 vs
// 24.9 Gframes/s for the two layouts (tools/bwlab.hip nat).  Windows of more than
// 4 chunks (IPv4 options, IPv6: CH = 6) take a second quad round when any packet of the wave needs
// it.  The loop is wave-uniform: every lane takes part in the quad moves.
template <int FMT, bool STRICT, int W, bool PROBE = false, int CH = kNatChunks, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_natq(uint8_t* __restrict__ arena, uint64_t arena_len,
                                             const uint4* __restrict__ desc, const void* __restrict__ rw, uint32_t n,
                                             uint8_t* __restrict__ status, uint8_t* __restrict__ flags_out) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) const v4u gv4u;
    constexpr int kSlotDw = 4 * CH + 1;   // LDS slot per packet: an odd dword stride
    constexpr int NR = (CH + 3) / 4;       // quad rounds per window
    __shared__ uint32_t s_win[256 * kSlotDw];
    const int lane = threadIdx.x & 63;
    uint32_t* wsl = &s_win[(threadIdx.x & ~63u) * kSlotDw];   // this wave's 64 slots
    uint32_t* slot = wsl + lane * kSlotDw;
    uint8_t* w = (uint8_t*)slot;
    const uint32_t T = gridDim.x * blockDim.x;
    const int ql = lane & 3;
    for (uint32_t p0w = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); p0w < n; p0w += W * T) {
        const uint32_t p0 = p0w + (uint32_t)lane;
        uint4 dv[W];
        NatRw rr[W];
        uint32_t blo[W], bhi[W];   // window base (16-B aligned absolute address)
        int wend[W];               // bytes of the window this packet needs; 0: none (byte path / idle)
#pragma unroll
        for (int i = 0; i < W; ++i) {
            const uint32_t p = p0 + i * T;
            dv[i] = p < n ? nat_load_desc<FMT>(desc, p) : make_uint4(0, 0, 0, 0);
            rr[i] = nat_load_rw<FMT>(rw, p < n ? p : 0);
        }
        v4u v[W][4];   // quad round 0 (chunks 0..3); a second round, when a window needs it, is rare
        bool r2[W];
#pragma unroll
        for (int i = 0; i < W; ++i) {
            const uint32_t p = p0 + i * T;
            const uint64_t off = (uint64_t)dv[i].x | ((uint64_t)dv[i].y << 32);
            const int len = dv[i].z & 0xffff, l4o = dv[i].z >> 16;
            const int ver = dv[i].w & 0xff, proto = (dv[i].w >> 8) & 0xff;
            const bool ok = p < n && nat_desc_ok(off, len, l4o, ver, arena_len, FMT);
            const uintptr_t la = ok ? (uintptr_t)(arena + off) : 0;
            const int r0 = (int)(la & 15);
            int need = ver == 4 ? 20 : 40;
            if (nat_l4sum(ver, proto, len, l4o)) need = max(need, l4o + l4_field(proto) + 2);
            wend[i] = ok && r0 + need <= 16 * CH ? r0 + need : 0;
            const uint64_t base = (uint64_t)(la - (uintptr_t)r0);
            blo[i] = (uint32_t)base;
            bhi[i] = (uint32_t)(base >> 32);
            r2[i] = NR > 1 && __ballot(wend[i] > 64) != 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = 16 * u + (lane >> 2);
                const uint32_t ql_lo = (uint32_t)__shfl((int)blo[i], q, 64);
                const uint32_t ql_hi = (uint32_t)__shfl((int)bhi[i], q, 64);
                const int qe = __shfl(wend[i], q, 64);
                v4u x = {0u, 0u, 0u, 0u};
                // only the chunks the packet needs, inside its 16-B blocks (never past a page)
                if ((ql << 4) < qe) x = *(gv4u*)((((uint64_t)ql_hi << 32) | ql_lo) + 16u * (uint32_t)ql);
                v[i][u] = x;
            }
        }
        uint32_t res[W];
#pragma unroll
        for (int i = 0; i < W; ++i) {
            const uint32_t p = p0 + i * T;
            // stage the quads' chunks in the owners' slots
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                uint32_t* d = wsl + (16 * u + (lane >> 2)) * kSlotDw + 4 * ql;
                d[0] = v[i][u].x; d[1] = v[i][u].y; d[2] = v[i][u].z; d[3] = v[i][u].w;
            }
            if (NR > 1 && r2[i]) {   // chunks 4.. of windows past 64 B (IPv4 options, IPv6)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int q = 16 * u + (lane >> 2);
                    const uint32_t ql_lo = (uint32_t)__shfl((int)blo[i], q, 64);
                    const uint32_t ql_hi = (uint32_t)__shfl((int)bhi[i], q, 64);
                    const int qe = __shfl(wend[i], q, 64);
                    const int k = 4 + ql;
                    if (k < CH && (k << 4) < qe) {
                        const v4u x = *(gv4u*)((((uint64_t)ql_hi << 32) | ql_lo) + 16u * (uint32_t)k);
                        uint32_t* d = wsl + q * kSlotDw + 4 * k;
                        d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            res[i] = 0;
            // this lane's store range [s, e) in window coordinates and the packet end lim
            int s = 0, e = 0, lim = 0;
            bool udp_zero = false;
            const uint64_t off = (uint64_t)dv[i].x | ((uint64_t)dv[i].y << 32);
            const int len = dv[i].z & 0xffff, l4o = dv[i].z >> 16;
            const int ver = dv[i].w & 0xff, proto = (dv[i].w >> 8) & 0xff;
            if (p < n) {
                if (!wend[i]) {
                    if (!PROBE) res[i] = nat_scalar<FMT>(arena, arena_len, dv[i], rr[i], STRICT);
                } else {
                    const int r0 = (int)((uintptr_t)(arena + off) & 15);
                    uint8_t* l3w = w + r0;
                    lim = r0 + len;
                    if (PROBE) {
                        int hi = ver == 4 ? 20 : 40;
                        if (nat_l4sum(ver, proto, len, l4o)) hi = max(hi, l4o + l4_field(proto) + 2);
                        s = r0 + (ver == 4 ? 10 : 8);
                        e = r0 + hi;
                        res[i] = VPCSUM_S_DONE;
                    } else if (nat_ttl_expired(l3w, ver, rr[i])) {
                        res[i] = STRICT ? kFlagRejected : kNatExpired;
                    } else {
                        NatAcc a = nat_setters(l3w, ver, proto, len, l4o, nat_l4sum(ver, proto, len, l4o), rr[i]);
                        if (!STRICT) udp_zero = nat_rfc1624(l3w, proto, l4o, l4_field(proto), a);
                        if (a.hi > a.lo) { s = r0 + a.lo; e = r0 + a.hi; }
                        res[i] = STRICT ? ((a.ip_dirty ? VPCSUM_F_IP : 0) | (a.l4_dirty ? VPCSUM_F_L4 : 0)) : VPCSUM_S_DONE;
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            // the quads store the changed ranges back
            // window coordinates are below 128: lim is clipped to a byte, r0 takes bits 24..27
            const uint32_t rng = (uint32_t)s | ((uint32_t)e << 8) | ((uint32_t)min(lim, 255) << 16) |
                                 ((uint32_t)(lim > 0 ? (int)((uintptr_t)(arena + off) & 15) : 0) << 24);
#pragma unroll
            for (int r = 0; r < NR; ++r) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int q = 16 * u + (lane >> 2);
                    const uint32_t qr = (uint32_t)__shfl((int)rng, q, 64);
                    const uint32_t ql_lo = (uint32_t)__shfl((int)blo[i], q, 64);
                    const uint32_t ql_hi = (uint32_t)__shfl((int)bhi[i], q, 64);
                    const int k = 4 * r + ql;
                    const int qs = (int)(qr & 0xff), qe = (int)((qr >> 8) & 0xff), qlim = (int)((qr >> 16) & 0xff);
                    if (k < CH && qe > qs)
                        natq_store_chunk((uint8_t*)(((uint64_t)ql_hi << 32) | ql_lo), wsl + q * kSlotDw, k, qs, qe, qlim,
                                         (int)(qr >> 24));
                }
            }
            if (!STRICT && !PROBE && __ballot(udp_zero)) {
                // the quads' stores of the rewritten header before the owner reads it back
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                if (udp_zero) nat_udp_full(arena + off, ver, len, l4o);
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");   // the slots are rewritten for the next packet set
        }
        uint8_t* dst = STRICT ? flags_out : status;
        if (dst) {
#pragma unroll
            for (int i = 0; i < W; ++i) store_bytes_packed(dst, p0 + i * T, n, res[i]);
        }
    }
}

// ------------------------------------------------------------------------------------------
// K6: egress sums of NAT'd packets from their pre-images (vpcsum_pre_async, VPCSUM_F_PRE).
//
// In the reference the rewrite is Java's: SwitchUtils.applyNat (SwitchUtils.java:531-542) calls
// the setters, which write the new addresses / ports into the frame (raw.pktBuf.set, e.g.
// Ipv4Packet.setSrc :433-445, TcpPacket.setSrcPort :31-40) and mark the sums dirty; the packet
// then routes on the fields those setters cached (IPOutputRoute.java:52-53), and getRawPacket(0)
// at egress recomputes every dirty sum over the whole segment (AbstractPacket.java:15-22, 58-65).
// The vswitch keeps its setters and records, just before them, the old values (the pre-image);
// at the egress flush the L4 sum is RFC 1624 eqn. 3 from the stored field, HC' = ~(~HC +
// sum(~m + m')), m the recorded words, m' the words now in the frame -- nat_rfc1624's arithmetic
// with the old words taken from the pre-image instead of the frame.  Bit-identical to the full
// recompute when HC was correct (ingress verify's S_L4_OK, the caller's condition for F_PRE); a
// UDP stored 0 is summed in full.  The IPv4 header sum is recomputed in full: its bytes are in
// the window anyway.  Memory pattern: k_natq's quad-loaded header windows, minus the rewrite --
// only the two sum fields are stored, 4 B per packet, by the owner lane.
// ------------------------------------------------------------------------------------------

// Status bytes of the F_PRE lanes only (a mixed batch's other bytes are the checksum kernel's): a
// quad of four such lanes stores one dword (as store_bytes_packed), the others byte by byte.
__device__ __forceinline__ void store_bytes_masked(uint8_t* __restrict__ dst, uint32_t p, uint32_t n, uint32_t v, bool act) {
    v &= 0xff;
    const uint64_t am = __ballot(act);
    const uint32_t b1 = (uint32_t)__shfl_down((int)v, 1, 64), b2 = (uint32_t)__shfl_down((int)v, 2, 64),
                   b3 = (uint32_t)__shfl_down((int)v, 3, 64);
    const int lane = threadIdx.x & 63;
    if (((am >> (lane & ~3)) & 0xfull) == 0xfull) {
        if ((lane & 3) == 0) {
            const uint32_t packed = v | ((b1 & 0xff) << 8) | ((b2 & 0xff) << 16) | (b3 << 24);
            if (p + 4 <= n && !((uintptr_t)(dst + p) & 3)) {
                *(__attribute__((address_space(1))) uint32_t*)(dst + p) = packed;
            } else {
                for (uint32_t k = 0; k < 4 && p + k < n; ++k) dst[p + k] = (uint8_t)(packed >> (8 * k));
            }
        }
    } else if (act) {
        dst[p] = (uint8_t)v;
    }
}

// FMT: entry format (0: vpcsum_pre4_t, 1: vpcsum_pre_t); W packets per lane and iteration; CH
// window chunks (k_natq's); PROBE: the same loads and stores with no arithmetic -- the stored sums
// are written back unchanged (tooling: the pattern ceiling of the pre-image flush).  byte_path: every
// packet takes byte accesses on the frame (tests).
template <int FMT, int W, int CH = kNatChunks, bool PROBE = false>
__global__ __launch_bounds__(256) void k_pre(uint8_t* __restrict__ arena, uint64_t arena_len,
                                            const uint4* __restrict__ desc, const void* __restrict__ pre, uint32_t n,
                                            uint32_t* __restrict__ out, uint8_t* __restrict__ status, int write,
                                            int byte_path, int nt_store) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) const v4u gv4u;
    constexpr int kSlotDw = 4 * CH + 1;   // LDS slot per packet: an odd dword stride
    constexpr int NR = (CH + 3) / 4;       // quad rounds per window
    __shared__ uint32_t s_win[256 * kSlotDw];
    const int lane = threadIdx.x & 63;
    uint32_t* wsl = &s_win[(threadIdx.x & ~63u) * kSlotDw];   // this wave's 64 slots
    const uint8_t* w = (const uint8_t*)(wsl + lane * kSlotDw);
    const uint32_t T = gridDim.x * blockDim.x;
    const int ql = lane & 3;
    for (uint32_t p0w = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); p0w < n; p0w += W * T) {
        const uint32_t p0 = p0w + (uint32_t)lane;
        uint4 dv[W];
        NatRw rr[W];
        bool act[W], ok[W];
        uint32_t blo[W], bhi[W];   // window base (16-B aligned absolute address)
        int wend[W];               // bytes of the window this packet needs; 0: none (byte path / idle)
#pragma unroll
        for (int i = 0; i < W; ++i) {
            const uint32_t p = p0 + i * T;
            dv[i] = p < n ? desc[p] : make_uint4(0, 0, 0, 0);
            rr[i] = nat_load_rw<FMT>(pre, p < n ? p : 0);   // issued with the descriptor: independent of it
        }
        v4u v[W][4];
        bool r2[W];
#pragma unroll
        for (int i = 0; i < W; ++i) {
            const uint32_t p = p0 + i * T;
            const uint64_t off = (uint64_t)dv[i].x | ((uint64_t)dv[i].y << 32);
            const int len = dv[i].z & 0xffff, l4o = dv[i].z >> 16;
            const int ver = dv[i].w & 0xff, proto = (dv[i].w >> 8) & 0xff;
            act[i] = p < n && (((dv[i].w >> 16) & 0xff) & VPCSUM_F_PRE) != 0;
            ok[i] = act[i] && pre_desc_ok(dv[i], arena_len, FMT);
            const uintptr_t la = ok[i] ? (uintptr_t)(arena + off) : 0;
            const int r0 = (int)(la & 15);
            const bool l4 = ((dv[i].w >> 16) & VPCSUM_F_L4) != 0;
            // the header through the L4 checksum field, or through the L4 header an ingress header
            // sum covers (VPCSUM_PRE_HSUM: TCP options included)
            const int need = max(ver == 4 ? 20 : 40,
                                 l4 ? min(len, l4o + max(l4_field(proto) + 2, pre_hsum_hlen(rr[i]))) : l4o);
            wend[i] = ok[i] && !byte_path && r0 + need <= 16 * CH ? r0 + need : 0;
            const uint64_t base = (uint64_t)(la - (uintptr_t)r0);
            blo[i] = (uint32_t)base;
            bhi[i] = (uint32_t)(base >> 32);
            r2[i] = NR > 1 && __ballot(wend[i] > 64) != 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = 16 * u + (lane >> 2);
                const uint32_t ql_lo = (uint32_t)__shfl((int)blo[i], q, 64);
                const uint32_t ql_hi = (uint32_t)__shfl((int)bhi[i], q, 64);
                const int qe = __shfl(wend[i], q, 64);
                v4u x = {0u, 0u, 0u, 0u};
                // only the chunks the packet needs, inside its 16-B blocks (never past a page)
                if ((ql << 4) < qe) x = *(gv4u*)((((uint64_t)ql_hi << 32) | ql_lo) + 16u * (uint32_t)ql);
                v[i][u] = x;
            }
        }
        uint32_t res_out[W], res_st[W];
#pragma unroll
        for (int i = 0; i < W; ++i) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {   // stage the quads' chunks in the owners' slots
                uint32_t* d = wsl + (16 * u + (lane >> 2)) * kSlotDw + 4 * ql;
                d[0] = v[i][u].x; d[1] = v[i][u].y; d[2] = v[i][u].z; d[3] = v[i][u].w;
            }
            if (NR > 1 && r2[i]) {   // chunks 4.. of windows past 64 B (IPv4 options, IPv6)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int q = 16 * u + (lane >> 2);
                    const uint32_t ql_lo = (uint32_t)__shfl((int)blo[i], q, 64);
                    const uint32_t ql_hi = (uint32_t)__shfl((int)bhi[i], q, 64);
                    const int qe = __shfl(wend[i], q, 64);
                    const int k = 4 + ql;
                    if (k < CH && (k << 4) < qe) {
                        const v4u x = *(gv4u*)((((uint64_t)ql_hi << 32) | ql_lo) + 16u * (uint32_t)k);
                        uint32_t* d = wsl + q * kSlotDw + 4 * k;
                        d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            res_out[i] = 0;
            res_st[i] = VPCSUM_S_BAD_DESC;
            if (ok[i]) {
                const uint64_t off = (uint64_t)dv[i].x | ((uint64_t)dv[i].y << 32);
                const int len = dv[i].z & 0xffff, l4o = dv[i].z >> 16;
                const int ver = dv[i].w & 0xff, proto = (dv[i].w >> 8) & 0xff;
                const bool do_ip = ((dv[i].w >> 16) & VPCSUM_F_IP) != 0;
                const bool do_l4 = ((dv[i].w >> 16) & VPCSUM_F_L4) != 0;
                const int fld = l4_field(proto);
                uint8_t* l3 = arena + off;
                const int r0 = (int)((uintptr_t)l3 & 15);
                PreSums s = {0u, 0u, false, false};
                if (PROBE) {
                    if (do_ip) s.ipc = ld16(w + r0 + 10);
                    if (do_l4) s.l4c = ld16(w + r0 + l4o + fld);
                } else {
                    s = wend[i] ? pre_sums(w + r0, ver, proto, len, l4o, do_ip, do_l4, rr[i])
                                : pre_sums(l3, ver, proto, len, l4o, do_ip, do_l4, rr[i]);
                    if (s.udp_full) s.l4c = udp_full_sum(l3, ver, len, l4o);
                }
                // s.bad: a header-sum record of another packet -- refused (S_BAD_DESC), nothing written
                if (!s.bad) {
                    if (write) {
                        // plain stores: the two fields usually share a line, which L2 writes back once
                        // (non-temporal ones reach DRAM apart: C5 12.6 vs 18.4 Gpps)
                        if (nt_store) {
                            if (do_ip) st_be16_nt(l3 + 10, s.ipc);
                            if (do_l4) st_be16_nt(l3 + l4o + fld, s.l4c);
                        } else {
                            if (do_ip) st_be16(l3 + 10, s.ipc);
                            if (do_l4) st_be16(l3 + l4o + fld, s.l4c);
                        }
                    }
                    res_out[i] = (s.ipc & 0xffff) | ((s.l4c & 0xffff) << 16);
                    res_st[i] = VPCSUM_S_DONE;
                }
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");   // the slots are rewritten for the next packet set
        }
#pragma unroll
        for (int i = 0; i < W; ++i) {
            const uint32_t p = p0 + i * T;
            if (out && act[i]) out[p] = res_out[i];
            if (status) store_bytes_masked(status, p, n, res_st[i], act[i]);
        }
    }
}

static uint32_t nat_grid(uint32_t n, int wl2, uint32_t wgs_per_cu);
static uint32_t nat_wgs_per_cu(uint32_t nat_mode);

hipError_t launch_pre(uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* desc, const void* pre, int fmt, uint32_t n,
                      uint32_t* out, uint8_t* status, uint32_t mode, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const int write = (mode & VPCSUM_MODE_WRITE) ? 1 : 0;
    const int byte_path = (mode & 0x100u) ? 1 : 0;
    // packets per lane: one by default (C5 +0.9% over two, profiles/r05d_presweep.json), bits 12..13 = 2: two
    const int w1 = ((mode >> 12) & 3u) != 2;
    const bool ch4 = ((mode >> 16) & 3u) == 2 && fmt == 0;       // 4-chunk windows (16-B entries only)
    const bool probe = (mode & 0x800000u) != 0 && fmt == 0;
    const int nt_store = (mode & 0x1000000u) ? 1 : 0;   // bit 24: non-temporal field stores (A/B)
    const uint32_t g = nat_grid(n, w1 ? 0 : 1, nat_wgs_per_cu(mode));
    const uint4* d = (const uint4*)desc;
#define VPC_PRE(F, W, C, P)                                                                                             \
    hipLaunchKernelGGL((k_pre<F, W, C, P>), dim3(g), dim3(256), 0, stream, arena, arena_len, d, pre, n, out, status, write, \
                       byte_path, nt_store)
    if (probe) {
        if (ch4) VPC_PRE(0, 2, 4, true); else VPC_PRE(0, 2, kNatChunks, true);
    } else if (fmt == 0) {
        if (ch4) { if (w1) VPC_PRE(0, 1, 4, false); else VPC_PRE(0, 2, 4, false); }
        else { if (w1) VPC_PRE(0, 1, kNatChunks, false); else VPC_PRE(0, 2, kNatChunks, false); }
    } else {
        if (w1) VPC_PRE(1, 1, kNatChunks, false); else VPC_PRE(1, 2, kNatChunks, false);
    }
#undef VPC_PRE
    return hipGetLastError();
}

// Strict mode's status after the recompute kernel: that kernel reports a refused packet as
// S_BAD_DESC only, so the TTL-expired ones get their S_TTL_EXPIRED bit here, from the same test on
// the same bytes: a refused packet was left untouched.  Only refused packets are looked at (a TTL
// of 2 decremented to 1 passed); the recompute kernel refuses exactly the packets the rewrite
// refused, since its descriptor rules equal nat_desc_ok for the flags the rewrite hands it.
template <int FMT>
__global__ __launch_bounds__(256) void k_nat_ttl_status(const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                       const uint4* __restrict__ desc, const void* __restrict__ rw,
                                                       uint32_t n, uint8_t* __restrict__ status) {
    // status[p] is read before it is written, by this lane only
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
        const NatRw r = nat_load_rw<FMT>(rw, p);
        if (!(r.mask & VPCSUM_NAT_DEC_TTL) || status[p] != VPCSUM_S_BAD_DESC) continue;
        const uint4 dv = nat_load_desc<FMT>(desc, p);
        const uint64_t off = (uint64_t)dv.x | ((uint64_t)dv.y << 32);
        const int len = dv.z & 0xffff, l4o = dv.z >> 16, ver = dv.w & 0xff;
        if (nat_desc_ok(off, len, l4o, ver, arena_len, FMT) && nat_ttl_expired(arena + off, ver, r))
            status[p] = (uint8_t)kNatExpired;
    }
}

hipError_t launch_nat_ttl_status(const uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* desc, const void* rw,
                                 int fmt, uint32_t n, uint8_t* status, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    int dev = 0;
    (void)hipGetDevice(&dev);
    uint32_t g = (n + 255) / 256;
    const uint32_t cap = (uint32_t)num_cus(dev) * 8;
    if (g > cap) g = cap;
    if (fmt == 0)
        hipLaunchKernelGGL(k_nat_ttl_status<0>, dim3(g), dim3(256), 0, stream, arena, arena_len, (const uint4*)desc, rw, n, status);
    else
        hipLaunchKernelGGL(k_nat_ttl_status<1>, dim3(g), dim3(256), 0, stream, arena, arena_len, (const uint4*)desc, rw, n, status);
    return hipGetLastError();
}

constexpr int kNatWideLog2 = 1;   // packets per lane and iteration of k_natw: 2

// Grid of the wide kernel: enough workgroups that one iteration of W packets per lane covers the
// batch, capped at `wgs_per_cu` per CU (grid-stride beyond that).
static uint32_t nat_grid(uint32_t n, int wl2, uint32_t wgs_per_cu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    uint32_t g = (n + (256u << wl2) - 1) / (256u << wl2);
    const uint32_t cap = (uint32_t)num_cus(dev) * wgs_per_cu;
    return g > cap ? cap : g;
}

// Internal tuning bits of nat_mode (not part of the stable ABI): bit 8 byte-access kernel; bits
// 12..14 log2(packets per lane) + 1 of the wide kernel (k_natw takes 1, 2 or 4 packets per lane;
// k_natq only 1 or 2, so a request for 4 runs k_natq at 2); bits 16..17 window chunks (1: 6,
// 2: 4); bits 18..22 workgroups per CU (0: 24); bit 23 the lane layout (k_natw) instead of quads
// (k_natq); bits 24..25 k_natq's forced occupancy (1: 6, 2: 8 waves per SIMD -- tuning shapes that
// may spill to scratch, tests/test_kernel_resources.py exempts them; 0 and 3: the default).
static int nat_chunks_sel(uint32_t nat_mode, int fmt) {
    const uint32_t c = (nat_mode >> 16) & 3u;
    if (c == 1) return 6;
    if (c == 2 && fmt != 1) return 4;
    return kNatChunks;
}
// Default: 24 workgroups per CU (4 resident at 101 VGPRs, so the grid-stride loop starts in six
// dispatch rounds): +2.6% over 8 on 10M C5 packets, 12 and 16 in between (profiles/r03e_nat_grid/)
static uint32_t nat_wgs_per_cu(uint32_t nat_mode) {
    const uint32_t w = (nat_mode >> 18) & 31u;
    return w ? w : 24u;
}

hipError_t launch_nat_probe(uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* desc, const void* rw, int fmt,
                            uint32_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    // tooling: the tuning bits of nat_mode, to price the same shapes launch_nat can take
    static const uint32_t tune = [] {
        const char* e = getenv("VPCSUM_NAT_PROBE_TUNE");
        return e ? (uint32_t)strtoul(e, nullptr, 0) : 0u;
    }();
    const uint32_t g = nat_grid(n, kNatWideLog2, nat_wgs_per_cu(tune));
    const uint4* d = (const uint4*)desc;
    constexpr int W = 1 << kNatWideLog2;
    if (!(tune & 0x800000u)) {   // the quad layout (k_natq), as launch_nat's default
        if (fmt == 2)
            hipLaunchKernelGGL((k_natq<2, false, W, true>), dim3(g), dim3(256), 0, stream, arena, arena_len, d, rw, n,
                               (uint8_t*)nullptr, (uint8_t*)nullptr);
        else if (fmt == 0 && nat_chunks_sel(tune, 0) == 4)
            hipLaunchKernelGGL((k_natq<0, false, W, true, 4>), dim3(g), dim3(256), 0, stream, arena, arena_len, d, rw, n,
                               (uint8_t*)nullptr, (uint8_t*)nullptr);
        else if (fmt == 0)
            hipLaunchKernelGGL((k_natq<0, false, W, true>), dim3(g), dim3(256), 0, stream, arena, arena_len, d, rw, n,
                               (uint8_t*)nullptr, (uint8_t*)nullptr);
        else
            hipLaunchKernelGGL((k_natq<1, false, W, true>), dim3(g), dim3(256), 0, stream, arena, arena_len, d, rw, n,
                               (uint8_t*)nullptr, (uint8_t*)nullptr);
    } else if (fmt == 0 && nat_chunks_sel(tune, 0) == 4)
        hipLaunchKernelGGL((k_natw<0, false, W, true, 4>), dim3(g), dim3(256), 0, stream, arena, arena_len, d, rw, n,
                           (uint8_t*)nullptr, (uint8_t*)nullptr);
    else if (fmt == 0)
        hipLaunchKernelGGL((k_natw<0, false, W, true>), dim3(g), dim3(256), 0, stream, arena, arena_len, d, rw, n,
                           (uint8_t*)nullptr, (uint8_t*)nullptr);
    else
        hipLaunchKernelGGL((k_natw<1, false, W, true>), dim3(g), dim3(256), 0, stream, arena, arena_len, d, rw, n,
                           (uint8_t*)nullptr, (uint8_t*)nullptr);
    return hipGetLastError();
}

hipError_t launch_nat(uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* desc, const void* rw, int fmt,
                      uint32_t n, uint8_t* status, uint8_t* flags_out, uint32_t nat_mode, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const bool strict = (nat_mode & VPCSUM_NAT_STRICT_JAVA) != 0;
    const int wsel = (int)((nat_mode >> 12) & 7u);
    const int wl2 = wsel ? (wsel - 1 > 2 ? 2 : wsel - 1) : kNatWideLog2;
    const uint32_t g = nat_grid(n, wl2, nat_wgs_per_cu(nat_mode));
    const int ch = nat_chunks_sel(nat_mode, fmt);
    const bool wide = !(nat_mode & 0x100u);
    const bool quad = (nat_mode & 0x800000u) == 0;
    const uint4* d = (const uint4*)desc;
    if (wide && quad) {
#define VPC_NATQ(F, S, W, C)                                                                                           \
    do {                                                                                                               \
        const uint32_t wpe = (nat_mode >> 24) & 3u;                                                                    \
        if (wpe == 1)                                                                                                  \
            hipLaunchKernelGGL((k_natq<F, S, W, false, C, 6>), dim3(g), dim3(256), 0, stream, arena, arena_len, d, rw, n, status, flags_out); \
        else if (wpe == 2)                                                                                             \
            hipLaunchKernelGGL((k_natq<F, S, W, false, C, 8>), dim3(g), dim3(256), 0, stream, arena, arena_len, d, rw, n, status, flags_out); \
        else                                                                                                           \
            hipLaunchKernelGGL((k_natq<F, S, W, false, C>), dim3(g), dim3(256), 0, stream, arena, arena_len, d, rw, n, status, flags_out); \
    } while (0)
#define VPC_NATQ_W(F, S, C) do { if (wl2 == 0) VPC_NATQ(F, S, 1, C); else VPC_NATQ(F, S, 2, C); } while (0)
        if (fmt == 2) {   // records: RFC 1624 only (the strict recompute takes plain descriptors)
            if (ch == 4) VPC_NATQ_W(2, false, 4); else VPC_NATQ_W(2, false, kNatChunks);
        } else if (fmt == 0 && ch == 4) {
            if (strict) VPC_NATQ_W(0, true, 4); else VPC_NATQ_W(0, false, 4);
        } else if (fmt == 0) {
            if (strict) VPC_NATQ_W(0, true, kNatChunks); else VPC_NATQ_W(0, false, kNatChunks);
        } else {
            if (strict) VPC_NATQ_W(1, true, kNatChunks); else VPC_NATQ_W(1, false, kNatChunks);
        }
#undef VPC_NATQ_W
#undef VPC_NATQ
    } else if (wide) {
#define VPC_NAT(F, S, W, C) hipLaunchKernelGGL((k_natw<F, S, W, false, C>), dim3(g), dim3(256), 0, stream, arena, arena_len, d, rw, n, status, flags_out)
#define VPC_NAT_W(F, S) do { if (wl2 == 0) VPC_NAT(F, S, 1, kNatChunks); else if (wl2 == 1) VPC_NAT(F, S, 2, kNatChunks); else VPC_NAT(F, S, 4, kNatChunks); } while (0)
        if (fmt == 2) {
            VPC_NAT_W(2, false);
        } else if (fmt == 0 && !strict && ch == 4) {
            if (wl2 == 2) VPC_NAT(0, false, 4, 4); else VPC_NAT(0, false, 2, 4);
        } else if (fmt == 0) {
            if (strict) VPC_NAT_W(0, true); else VPC_NAT_W(0, false);
        } else {
            if (strict) VPC_NAT_W(1, true); else VPC_NAT_W(1, false);
        }
#undef VPC_NAT_W
#undef VPC_NAT
    } else if (fmt == 2) {
        hipLaunchKernelGGL(k_nat<2>, dim3(g), dim3(256), 0, stream, arena, arena_len, d, rw, n, status, flags_out, 0);
    } else if (fmt == 0) {
        hipLaunchKernelGGL(k_nat<0>, dim3(g), dim3(256), 0, stream, arena, arena_len, d, rw, n, status, flags_out, strict ? 1 : 0);
    } else {
        hipLaunchKernelGGL(k_nat<1>, dim3(g), dim3(256), 0, stream, arena, arena_len, d, rw, n, status, flags_out, strict ? 1 : 0);
    }
    return hipGetLastError();
}


}  // namespace vpcsum
