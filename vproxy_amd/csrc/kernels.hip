// kernels.hip -- gfx950 (MI355X, CDNA4) kernels of libvpcsum.
//
// The hot path restates, batched, the Java checksum code of vproxy's vswitch:
//   Utils.calculateChecksumIntermediate / DoFinal     base/src/main/java/io/vproxy/base/util/Utils.java:778-801
//   Utils.buildPseudoIPv4Header / IPv6Header          Utils.java:758-776
//   Ipv4Packet.__updateChecksum                       base/src/main/java/io/vproxy/vpacket/Ipv4Packet.java:209-217
//   TcpPacket.updateChecksumWithIPv4/IPv6             vpacket/TcpPacket.java:475-485, 508-518
//   UdpPacket.updateChecksumWithIPv4/IPv6 (0->ffff)   vpacket/UdpPacket.java:136-164
//   IcmpPacket.__updateChecksum / WithIPv6            vpacket/IcmpPacket.java:64-74, 124-135
//
// Arithmetic: the Java loop folds the end-around carry after every big-endian 16-bit word.
// Here each lane sums little-endian 32-bit words of 16-byte aligned chunks into 64 bits,
// the team (lanes of one packet) reduces with wave shuffles, and the sum is folded once and
// byte-swapped when the range starts at an even address.  That is bit-exact with the Java
// per-step fold, including the 0x0000/0xffff representation (both give 0 only for an
// all-zero input; tests/test_oracle_golden.py::test_deferred_fold_equivalence).
//
// No MFMA: this is a bandwidth-bound integer reduction (~0.4 integer ops per byte).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "vpcsum.h"
#include "internal.h"
#include "device_common.h"
#include "pre_common.h"

namespace vpcsum {

// ------------------------------------------------------------------------------------------
// small helpers
// ------------------------------------------------------------------------------------------

// Default lanes per packet (large tier of K2) and 16-B loads in flight per lane.  The payload
// loop costs the same per byte for any TEAM; 8 x 6 covers a 1500-B packet in two trips.
constexpr int kDefaultTeam = 8;
constexpr int kDefaultUnroll = 6;
// Small tier of the default kernel (K2): packets of at most kSmallTeam * kSmallUnroll 16-B chunks
// (64 B incl. alignment) are streamed by 2-lane teams, 32 packets per iteration.
constexpr int kSmallTeam = 2;
constexpr int kSmallUnroll = 2;
// Large-tier slot rotation of the default kernel: wave w starts its unit at slot (9 w) mod the
// tier size.  Units are 64 packets, a power-of-two stride apart (128 KB at a 2-KB frame stride);
// without it, all waves read the same offset within their units at the same moment, and the
// HBM channel/bank mapping aliases those addresses: C2 -4%.
constexpr int kDefaultRot = -9;
constexpr int kEsUnits = 8;   // K2 (DS): units whose out / status words a wave stages in LDS

// Sum over the TEAM lanes of a team (aligned lane groups; every lane gets the total).  Teams of
// up to 16 lanes reduce with DPP lane swizzles inside a row (xor 1, xor 2 by quad_perm, then
// the half-row and row mirrors), one VALU op per step instead of an LDS-crossbar bpermute.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_add(uint32_t v) {
    return v + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int TEAM>
__device__ __forceinline__ uint32_t team_sum(uint32_t v) {
    if (TEAM <= 16) {
        if (TEAM >= 2) v = dpp_add<0xB1>(v);    // quad_perm [1,0,3,2]
        if (TEAM >= 4) v = dpp_add<0x4E>(v);    // quad_perm [2,3,0,1]
        if (TEAM >= 8) v = dpp_add<0x141>(v);   // row_half_mirror
        if (TEAM >= 16) v = dpp_add<0x140>(v);  // row_mirror
        return v;
    }
#pragma unroll
    for (int m = TEAM / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, TEAM);
    return v;
}

// ------------------------------------------------------------------------------------------
// k_csum: team-per-packet compute / verify kernel, the fallback for arenas the buffer path
// (K2, below) cannot address (> 4 GiB or not 16-B aligned), and the variant ids 2..11 of
// launch_csum.  One team of TEAM lanes per packet; each lane owns the 16-byte chunks
// k = tl, tl+TEAM, ... of [align16(L3), L3+need).  U chunks per lane are
// loaded (global_load_dwordx4) before any is consumed so every lane keeps U*16 bytes in
// flight; chunks fully inside the L4 payload take the 8-instruction fast path, the few
// header / tail chunks take the byte-masked path.
// ------------------------------------------------------------------------------------------
struct PktPlan {
    int r0;        // L3 start relative to the 16-B aligned base
    int nch;       // chunks to read
    int fast_lo;   // first byte (rel) of the all-L4 region (16-B aligned)
    int fast_hi;   // end (rel) of the all-L4 region (16-B aligned)
    int l4lo, l4hi, fa;     // L4 range (rel) and L4 checksum field (rel), fa < -8 if none
    int iplo, iphi;         // IPv4 header range (rel); empty if no IP sum
    int pslo, pshi;         // pseudo-header address bytes (rel); empty if none
};

// One packet streamed by a team of TEAM lanes (tl = this lane's index in the team): the body of
// k1_run.
template <int TEAM, int U, bool VERIFY, bool NT, bool PRED = false>
__device__ __forceinline__ void k1_packet(const uint8_t* __restrict__ arena, uint64_t arena_len, const uint4 dv,
                                          const int fov, const bool has_override, const uint32_t p,
                                          uint32_t* __restrict__ out, uint8_t* __restrict__ status,
                                          uint8_t* __restrict__ arena_w, const int tl) {
    const uint64_t off = (uint64_t)dv.x | ((uint64_t)dv.y << 32);
    const int len = dv.z & 0xffff;
    const int l4o = dv.z >> 16;
    const int ver = dv.w & 0xff;
    const int proto = (dv.w >> 8) & 0xff;
    int fl = (dv.w >> 16) & 0xff;
    if (has_override) fl = fov;
    fl = csum_flags(fl);

    // ---- validate (never read or write outside the arena) ----
    bool bad = off > arena_len || (uint64_t)len > arena_len - off || (fl & kFlagRejected);
    const bool raw = (fl & VPCSUM_F_RAW) != 0;
    bool do_ip = false, do_l4 = false, psonly = false;
    int fld = -1;
    if (!bad && !raw) {
        if (ver == 4) bad = len < 20 || l4o < 20 || l4o > len || (l4o & 3);
        else if (ver == 6) bad = len < 40 || l4o < 40 || l4o > len;
        else bad = true;
        if (!bad && (fl & (VPCSUM_F_L4 | VPCSUM_F_L4P))) {
            psonly = (fl & VPCSUM_F_L4P) != 0;
            fld = l4_field(proto);
            if (fld < 0 || (ver == 4 && proto == 58) || len - l4o < fld + 2) bad = true;
            else if (psonly && ((fl & VPCSUM_F_L4) || proto == 1)) bad = true;
            else do_l4 = true;
        }
        if (!bad && (fl & VPCSUM_F_IP)) {
            if (ver != 4) bad = true;
            else do_ip = true;
        }
    }
    if (bad) {
        if (tl == 0) {
            if (out) out[p] = 0;
            if (status) status[p] = VPCSUM_S_BAD_DESC;
        }
        return;
    }

    const uint8_t* l3 = arena + off;
    const uint4* base = (const uint4*)((uintptr_t)l3 & ~(uintptr_t)15);
    PktPlan pl;
    pl.r0 = (int)((uintptr_t)l3 & 15);
    // pseudo-only (F_L4P): the IP header holds the pseudo addresses, the segment is not read
    const int need = psonly ? l4o + fld + 2 : (raw || do_l4) ? len : (do_ip ? l4o : 0);
    pl.nch = need ? (pl.r0 + need + 15) >> 4 : 0;   // no sums (flags 0, F_PRE): nothing to read
    if (raw) {
        pl.l4lo = pl.r0; pl.l4hi = pl.r0 + len; pl.fa = -64;
        pl.fast_lo = (pl.r0 + 15) & ~15;
    } else if (psonly) {
        pl.l4lo = 0; pl.l4hi = 0; pl.fa = pl.r0 + l4o + fld;
        pl.fast_lo = 1 << 30;
    } else if (do_l4) {
        pl.l4lo = pl.r0 + l4o; pl.l4hi = pl.r0 + len; pl.fa = pl.r0 + l4o + fld;
        pl.fast_lo = (pl.fa + 2 + 15) & ~15;
    } else {
        pl.l4lo = 0; pl.l4hi = 0; pl.fa = -64;
        pl.fast_lo = 1 << 30;
    }
    pl.fast_hi = (pl.r0 + need) & ~15;
    if (do_ip) { pl.iplo = pl.r0; pl.iphi = pl.r0 + l4o; } else { pl.iplo = 0; pl.iphi = 0; }
    if (do_l4 && proto != 1) {
        pl.pslo = pl.r0 + (ver == 4 ? 12 : 8);
        pl.pshi = pl.r0 + (ver == 4 ? 20 : 40);
    } else { pl.pslo = 0; pl.pshi = 0; }

    uint64_t acc_l4 = 0, acc_ip = 0, acc_ps = 0;
    uint32_t st_ip = 0, st_l4 = 0;   // stored fields (verify), as masked LE bytes

    for (int r0 = 0; r0 * TEAM < pl.nch; r0 += U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            // unconditional load (index clamped to the last chunk, a cache hit) keeps the
            // U loads branch-free and in flight together; out-of-range chunks are skipped below
            if (PRED) {
                const int k = (r0 + u) * TEAM + tl;
                v[u] = k < pl.nch ? ld_stream<NT>(base + k) : make_uint4(0, 0, 0, 0);
            } else {
                const int k = min((r0 + u) * TEAM + tl, pl.nch - 1);
                v[u] = ld_stream<NT>(base + k);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = (r0 + u) * TEAM + tl;
            if (k >= pl.nch) continue;
            const int c = k << 4;
            if (c >= pl.fast_lo && c + 16 <= pl.fast_hi) {
                // payload chunk: every byte belongs to the L4 sum
                acc_l4 += (uint64_t)v[u].x + v[u].y;
                acc_l4 += (uint64_t)v[u].z + v[u].w;
            } else if (c >= pl.fast_lo) {
                // tail chunk: past the header and the checksum field, only the end is cut
                const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int j = 0; j < 4; ++j) acc_l4 += w[j] & tailmask(c + 4 * j, pl.l4hi);
            } else {
                // header chunk: IPv4 header / pseudo addresses / L4 header / fields
                const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int d = c + 4 * j;
                    const uint32_t mf = bmask(d, pl.fa, pl.fa + 2);
                    acc_l4 += w[j] & bmask(d, pl.l4lo, pl.l4hi) & ~mf;
                    const uint32_t mif = bmask(d, pl.r0 + 10, pl.r0 + 12);
                    acc_ip += w[j] & bmask(d, pl.iplo, pl.iphi) & ~mif;
                    acc_ps += w[j] & bmask(d, pl.pslo, pl.pshi);
                    if (VERIFY) {
                        st_l4 += w[j] & mf;
                        st_ip += (w[j] & mif) & (do_ip ? 0xffffffffu : 0u);
                    }
                }
            }
        }
    }

    uint32_t s_l4 = team_sum<TEAM>(fold64(acc_l4));
    uint32_t s_ip = team_sum<TEAM>(fold64(acc_ip));
    uint32_t s_ps = team_sum<TEAM>(fold64(acc_ps));
    uint32_t s_stl4 = 0, s_stip = 0;
    if (VERIFY) {
        s_stl4 = team_sum<TEAM>(fold32(st_l4));
        s_stip = team_sum<TEAM>(fold32(st_ip));
    }

    if (tl == 0) {
        uint32_t ipc = 0, l4c = 0;
        uint8_t st = VPCSUM_S_DONE;
        if (raw) {
            ipc = 0xffff - orient(fold32(s_l4), pl.r0);
        } else {
            if (do_ip) {
                ipc = 0xffff - orient(fold32(s_ip), pl.r0);
            }
            if (do_l4) {
                uint32_t tot = orient(fold32(s_l4), pl.r0 + l4o);
                if (proto != 1) {
                    const uint32_t l4len = (uint32_t)(len - l4o);
                    const int pproto = proto;   // Consts.IP_PROTOCOL_* of the L4 class
                    tot += orient(fold32(s_ps), pl.r0) + (uint32_t)pproto + (l4len & 0xffff) + (l4len >> 16);
                }
                if (psonly) {
                    l4c = fold32(tot);   // CHECKSUM_PARTIAL: uncomplemented
                } else {
                    l4c = 0xffff - fold32(tot);
                    if (proto == 17 && l4c == 0) l4c = 0xffff;
                }
            }
            if (VERIFY) {
                if (do_ip && orient(fold32(s_stip), pl.r0) == ipc) st |= VPCSUM_S_IP_OK;
                if (do_l4) {
                    const uint32_t stored = orient(fold32(s_stl4), pl.fa);
                    if (stored == l4c) st |= VPCSUM_S_L4_OK;
                    if (!psonly && proto == 17 && stored == 0) st |= VPCSUM_S_UDP_NOCSUM;
                }
            }
            if (arena_w) {
                uint8_t* w = arena_w + off;
                if (do_ip) { w[10] = (uint8_t)(ipc >> 8); w[11] = (uint8_t)ipc; }
                if (do_l4) { w[l4o + fld] = (uint8_t)(l4c >> 8); w[l4o + fld + 1] = (uint8_t)l4c; }
            }
        }
        if (out) out[p] = (ipc & 0xffff) | ((l4c & 0xffff) << 16);
        if (status) status[p] = st;
    }
}

// A pre-image frame (VPCSUM_F_PRE) on the service grid, one wave per frame: k_pre's arithmetic
// (nat.hip, pre_common.h:pre_sums) for the small zero-copy flushes of NAT'd frames.  The header
// window (chunk k on lane k, predicated: only the chunks the frame needs cross PCIe) and the
// pre-image (its 16-B pieces on lanes 32..34) come in one round trip and are staged in LDS; lane 0
// rebuilds the IPv4 header sum, applies RFC 1624 eqn. 3 to the L4 sum and stores the two fields.
// A UDP frame whose stored sum is 0 is summed in full by the whole wave (k1_packet without F_PRE),
// where k_pre takes byte reads: the same value as Java's recompute.  The stored L4 sum comes from
// the entry's spare bytes (vpcsum_pre4_t rsv[1..2], vpcsum_pre_t rsv[0..1]), where the host copied
// it when it posted the batch: the frame's own field is what this flush overwrites, so a batch that
// a leaving grid re-runs (api.cpp:svc_wait) must not read it back.
constexpr int kSvcPreChunks = 24;   // 384 B: any IPv4 header, IPv6 with one extension header
__device__ __forceinline__ uint4 shfl_u4(const uint4 v, int src) {
    return make_uint4((uint32_t)__shfl((int)v.x, src, 64), (uint32_t)__shfl((int)v.y, src, 64),
                      (uint32_t)__shfl((int)v.z, src, 64), (uint32_t)__shfl((int)v.w, src, 64));
}

template <bool PRED>
__device__ __forceinline__ void svc_pre_packet(const uint8_t* __restrict__ arena, uint64_t arena_len, const uint4 dv,
                                               const void* __restrict__ pre, int fmt, const uint32_t p,
                                               uint32_t* __restrict__ out, uint8_t* __restrict__ status,
                                               uint8_t* __restrict__ arena_w, const int tl) {
    __shared__ uint4 s_pw[4][kSvcPreChunks];   // a window per wave of the 256-thread workgroup
    if (!pre_desc_ok(dv, arena_len, fmt)) {
        if (tl == 0) {
            if (out) out[p] = 0;
            if (status) status[p] = VPCSUM_S_BAD_DESC;
        }
        return;
    }
    const int wv = (threadIdx.x >> 6) & 3;
    const uint64_t off = (uint64_t)dv.x | ((uint64_t)dv.y << 32);
    const int l4o = dv.z >> 16;
    const int ver = dv.w & 0xff, proto = (dv.w >> 8) & 0xff, fl = (dv.w >> 16) & 0xff;
    const bool do_ip = (fl & VPCSUM_F_IP) != 0, do_l4 = (fl & VPCSUM_F_L4) != 0;
    const int fld = l4_field(proto);
    const uint8_t* l3 = arena + off;
    const int r0 = (int)((uintptr_t)l3 & 15);
    // the header through the L4 checksum field, or -- for a VPCSUM_PRE_HSUM entry, which is read in
    // the same round trip -- through a TCP header of up to 60 B (options included), within the packet
    const int len = dv.z & 0xffff;
    const int need = max(ver == 4 ? 20 : 40, do_l4 ? max(l4o + fld + 2, min(len, l4o + 60)) : l4o);
    const int nch = (r0 + need + 15) >> 4;
    const bool win = nch <= kSvcPreChunks;
    const int npc = fmt ? 3 : 1;   // 16-B pieces of an entry
    uint4 v = make_uint4(0, 0, 0, 0);
    if (win && tl < nch) v = ((const uint4*)(l3 - r0))[tl];
    else if (tl >= 32 && tl < 32 + npc) v = ((const uint4*)pre)[(size_t)p * npc + (tl - 32)];
    if (tl < kSvcPreChunks) s_pw[wv][tl] = v;
    const uint4 e0 = shfl_u4(v, 32), e1 = shfl_u4(v, 33), e2 = shfl_u4(v, 34);
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    PreSums s = {0u, 0u, false, false};
    if (tl == 0) {
        const NatRw r = fmt ? nat_rw6(e0, e1, e2) : nat_rw4(e0);
        const uint32_t sp = fmt ? e2.y : e0.w;   // the captured sum, big endian, in its top 16 bits
        const int hc = (int)(((sp >> 8) & 0xff00u) | (sp >> 24));
        s = win ? pre_sums((const uint8_t*)&s_pw[wv][0] + r0, ver, proto, len, l4o, do_ip, do_l4, r, hc)
                : pre_sums(l3, ver, proto, len, l4o, do_ip, do_l4, r, hc);   // a window past 384 B: byte reads
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");   // s_pw is the next frame's
    if (__shfl((int)s.bad, 0, 64)) {   // a header-sum record of another packet: refused, nothing written
        if (tl == 0) {
            if (out) out[p] = 0;
            if (status) status[p] = VPCSUM_S_BAD_DESC;
        }
        return;
    }
    if (__shfl((int)s.udp_full, 0, 64)) {   // UDP stored 0: Java's recompute over the segment
        k1_packet<64, 4, false, true, PRED>(arena, arena_len, dv, fl & ~VPCSUM_F_PRE, true, p, out, status, arena_w, tl);
        return;
    }
    if (tl == 0) {
        if (arena_w) {
            uint8_t* w = arena_w + off;
            if (do_ip) { w[10] = (uint8_t)(s.ipc >> 8); w[11] = (uint8_t)s.ipc; }
            if (do_l4) { w[l4o + fld] = (uint8_t)(s.l4c >> 8); w[l4o + fld + 1] = (uint8_t)s.l4c; }
        }
        if (out) out[p] = (s.ipc & 0xffff) | ((s.l4c & 0xffff) << 16);
        if (status) status[p] = VPCSUM_S_DONE;
    }
}

__device__ __forceinline__ uint8_t parse_frame(const uint8_t* f, uint64_t o, uint32_t L, bool ok, uint8_t w, bool egress,
                                               vpcsum_desc_t& d);
__device__ __forceinline__ void frame_tuple(const uint8_t* b, const vpcsum_desc_t& d, uint32_t st, uint32_t t[10]);

// A raw frame on the service grid, one wave per frame: an egress frame (vpcsum_ctx_egress_frames)
// or, VERIFY, a received one (vpcsum_ctx_verify_frames).  Its first 384 B (every byte parse_frame
// reads) come in one PCIe round trip and are staged in LDS; lane 0 parses them with the vswitch's
// rules (k_parse_ether's parse_frame: egress, the frame's own flags, all honoured; ingress, those of
// F_IP / F_L4 the frame allows) and the wave sums or verifies the packet it found (k1_packet),
// where the launched path runs a parse kernel and a checksum kernel.  rec: the frame's 16-B record
// {u64 offset; u32 length; u8 flags; ...}.
constexpr int kSvcFrameChunks = 25;   // 384 B at any offset within a 16-B chunk
// PARSE (vpcsum_ctx_parse_frames): no sums; lane 0 writes the frame's descriptor to aux[p] and its
// flow tuple to the tuple array after kSvcBatchMax descriptors (frame_tuple, from the staged bytes).
template <bool VERIFY, bool PRED, bool PARSE = false>
__device__ __forceinline__ void svc_frame_packet(const uint8_t* __restrict__ arena, uint64_t arena_len, const uint4 rec,
                                                 const uint32_t p, uint32_t* __restrict__ out,
                                                 uint8_t* __restrict__ status, uint8_t* __restrict__ arena_w,
                                                 const int tl, void* __restrict__ aux = nullptr) {
    __shared__ uint4 s_fw[4][kSvcFrameChunks];
    const int wv = (threadIdx.x >> 6) & 3;
    const uint64_t o = (uint64_t)rec.x | ((uint64_t)rec.y << 32);
    const uint32_t L = rec.z;
    const bool inb = o <= arena_len && (uint64_t)L <= arena_len - o;
    const uint8_t* f = arena + o;
    const int r0 = (int)((uintptr_t)f & 15);
    const int nch = inb ? (r0 + (int)min(L, 384u) + 15) >> 4 : 0;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (tl < nch) v = ((const uint4*)(f - r0))[tl];
    if (tl < kSvcFrameChunks) s_fw[wv][tl] = v;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    uint4 dd = make_uint4(0, 0, 0, 0);
    uint32_t st = VPCSUM_S_BAD_DESC;
    if (tl == 0) {
        vpcsum_desc_t d;
        const uint8_t* fb = (const uint8_t*)&s_fw[wv][0] + r0;
        st = parse_frame(fb, o, L, inb, (uint8_t)(rec.w & 0xffu), !VERIFY && !PARSE, d);
        dd = make_uint4((uint32_t)d.l3_off, (uint32_t)(d.l3_off >> 32), (uint32_t)d.l3_len | ((uint32_t)d.l4_off << 16),
                        (uint32_t)d.l3_ver | ((uint32_t)d.l4_proto << 8) | ((uint32_t)d.flags << 16));
        if constexpr (VERIFY) {
            // the ingress header sum (vpcsum_hsum_t) into the aux buffer, from the staged header
            if (aux) {
                const int l2 = st == 0 ? (int)(d.l3_off - o) : 0;
                ((uint2*)aux)[p] = st == 0 ? hsum_record(fb + l2, d.l3_ver, d.l4_proto, d.l3_len, d.l4_off, l2)
                                           : make_uint2(0u, 0u);
            }
        }
        if constexpr (PARSE) {
            // the descriptor, the status byte and the tuple straight to the host's buffers
            uint32_t t[10];
            frame_tuple(fb + (st == 0 ? (int)(d.l3_off - o) : 0), d, st, t);
            ((uint4*)aux)[p] = dd;
            uint32_t* tp = (uint32_t*)((uint8_t*)aux + (size_t)kSvcBatchMax * sizeof(vpcsum_desc_t)) + (size_t)p * 10;
            for (int k = 0; k < 10; ++k) tp[k] = t[k];
            if (status) status[p] = (uint8_t)st;
        }
    }
    if constexpr (PARSE) return;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");   // s_fw is the next frame's
    dd = shfl_u4(dd, 0);
    if (__shfl((int)st, 0, 64) != 0) {   // refused: nothing written, handed back by the caller
        if (tl == 0) {
            if (out) out[p] = 0;
            if (status) status[p] = VPCSUM_S_BAD_DESC;
        }
        return;
    }
    k1_packet<64, 4, VERIFY, true, PRED>(arena, arena_len, dd, 0, false, p, out, status, arena_w, tl);
}

// Body for workgroup `blk` of a grid of `gdim` workgroups (k_csum: the launch grid;
// k_csum_service: the persistent service grid, once per batch).
// PRED: chunks past the packet end are not loaded (exec-masked) instead of re-loading the last
// chunk.  On device memory the clamped re-load is a cache hit and keeps the loads branch-free;
// on uncached host memory (zero-copy frames) every such load is another PCIe read.
// SVC (the service grid, TEAM 64): 1 = F_PRE descriptors take svc_pre_packet with the pre-images
// at `pre` (fmt 0: vpcsum_pre4_t, 1: vpcsum_pre_t; without `pre` they are no-ops, as everywhere
// else); 2 = `desc` holds raw frame records (svc_frame_packet); 3 = the same, parse only (descriptors
// and tuples into the aux buffer at `pre`).
template <int TEAM, int U, bool VERIFY, bool NT, bool PRED = false, int SVC = 0>
__device__ __forceinline__ void k1_run(const uint8_t* __restrict__ arena, uint64_t arena_len,
                                       const uint4* __restrict__ desc, uint32_t n,
                                       uint32_t* __restrict__ out, uint8_t* __restrict__ status,
                                       const uint8_t* __restrict__ flags_override,
                                       uint8_t* __restrict__ arena_w, uint32_t blk, uint32_t gdim,
                                       const void* __restrict__ pre = nullptr, int pre_fmt = 0) {
    static_assert(SVC == 0 || TEAM == 64, "the service grid's frames take a whole wave");
    const int tl = threadIdx.x & (TEAM - 1);
    const uint32_t team = (blk * 256u + threadIdx.x) / TEAM;
    const uint32_t nteams = gdim * (256u / TEAM);

    uint4 dnext = make_uint4(0, 0, 0, 0);
    int fnext = 0;
    if (team < n) {
        dnext = desc[team];
        if (flags_override) fnext = flags_override[team];
    }

    for (uint32_t p = team; p < n; p += nteams) {
        const uint4 dv = dnext;
        const int fov = fnext;
        if (p + nteams < n) {   // prefetch the next descriptor while this packet streams
            dnext = desc[p + nteams];
            if (flags_override) fnext = flags_override[p + nteams];
        }
        if constexpr (SVC == 2) {
            // RX verify: `pre` names the aux buffer for the frames' header sums (kSvcHsum), else NULL
            svc_frame_packet<VERIFY, PRED>(arena, arena_len, dv, p, out, status, arena_w, tl, const_cast<void*>(pre));
        } else if constexpr (SVC == 3) {
            svc_frame_packet<false, PRED, true>(arena, arena_len, dv, p, out, status, arena_w, tl, const_cast<void*>(pre));
        } else {
            if constexpr (SVC == 1) {
                if (pre && (((dv.w >> 16) & 0xffu) & VPCSUM_F_PRE)) {
                    svc_pre_packet<PRED>(arena, arena_len, dv, pre, pre_fmt, p, out, status, arena_w, tl);
                    continue;
                }
            }
            k1_packet<TEAM, U, VERIFY, NT, PRED>(arena, arena_len, dv, fov, flags_override != nullptr, p, out, status,
                                                 arena_w, tl);
        }
    }
}

__device__ __forceinline__ void hdr_dword(uint32_t w, int d, const PktPlan& pl, bool do_ip, uint64_t& acc_l4,
                                          uint64_t& acc_ip, uint64_t& acc_ps, uint32_t& st_l4, uint32_t& st_ip,
                                          bool verify) {
    const uint32_t mf = bmask(d, pl.fa, pl.fa + 2);
    acc_l4 += w & bmask(d, pl.l4lo, pl.l4hi) & ~mf;
    const uint32_t mif = bmask(d, pl.r0 + 10, pl.r0 + 12);
    acc_ip += w & bmask(d, pl.iplo, pl.iphi) & ~mif;
    acc_ps += w & bmask(d, pl.pslo, pl.pshi);
    if (verify) {
        st_l4 += w & mf;
        st_ip += (w & mif) & (do_ip ? 0xffffffffu : 0u);
    }
}

// [lo, hi) as a 32-bit halfword mask (bits clipped to 0..31)
__device__ __forceinline__ uint32_t hw_range(int lo, int hi) {
    const uint32_t mh = hi >= 32 ? 0xffffffffu : (hi <= 0 ? 0u : ((1u << hi) - 1u));
    const uint32_t ml = lo >= 32 ? 0xffffffffu : (lo <= 0 ? 0u : ((1u << lo) - 1u));
    return mh & ~ml;
}
__device__ __forceinline__ uint32_t hw_bit(int b) { return (b >= 0 && b < 32) ? (1u << b) : 0u; }
// 2 halfword-select bits -> dword byte mask: bit0 -> 0x0000ffff, bit1 -> 0xffff0000
__device__ __forceinline__ uint32_t hmask(uint32_t b) { return ((b & 1u) | ((b & 2u) << 15)) * 0xffffu; }

template <int TEAM, int U, bool VERIFY, bool NT, bool PRED = false>
__global__ __launch_bounds__(256) void k_csum(const uint8_t* __restrict__ arena, uint64_t arena_len,
                                              const uint4* __restrict__ desc, uint32_t n,
                                              uint32_t* __restrict__ out, uint8_t* __restrict__ status,
                                              const uint8_t* __restrict__ flags_override,
                                              uint8_t* __restrict__ arena_w) {
    k1_run<TEAM, U, VERIFY, NT, PRED>(arena, arena_len, desc, n, out, status, flags_override, arena_w, blockIdx.x, gridDim.x);
}

template <int TEAM, int U, bool PRED = false>
static hipError_t launch_team(const uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* desc, uint32_t n,
                              uint32_t* out, uint8_t* status, const uint8_t* flags_override, bool verify, bool nt,
                              uint8_t* arena_w, int grid, hipStream_t stream) {
    const uint32_t per_block = 256 / TEAM;
    uint32_t need = (n + per_block - 1) / per_block;
    uint32_t g = grid > 0 ? (uint32_t)grid : need;
    if (g > need) g = need;
    if (g == 0) g = 1;
#define VPC_LAUNCH(V, N)                                                                                         \
    hipLaunchKernelGGL((k_csum<TEAM, U, V, N, PRED>), dim3(g), dim3(256), 0, stream, arena, arena_len,                   \
                       (const uint4*)desc, n, out, status, flags_override, arena_w)
    if (verify) {
        if (nt) VPC_LAUNCH(true, true); else VPC_LAUNCH(true, false);
    } else {
        if (nt) VPC_LAUNCH(false, true); else VPC_LAUNCH(false, false);
    }
#undef VPC_LAUNCH
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Buffer addressing (K2).  The packet bytes come in through buffer_load_dwordx4 on ONE
// wave-uniform descriptor spanning the arena: a chunk past the packet end gets an offset outside
// the descriptor's range and the hardware returns zeros without touching memory.  So all U loads
// of a lane are issued unconditionally (no branch, nothing for the compiler to sink), address
// math is one 32-bit add per load, and the per-chunk classification is a single range test.
// Needs a 16-B aligned arena < 4 GiB (device_common.h); launch_d falls back to k_csum otherwise.
// ------------------------------------------------------------------------------------------

// ------------------------------------------------------------------------------------------
// K2: owner-lane plans, size-sorted teams.  A wave takes 64 consecutive packets per
// super-iteration.  Lane L decodes descriptor P0+L once (validation, chunk plan, header
// bitmaps), ranks its packet by cost class with ballots and publishes the plan to LDS slot
// `rank`.  Then TEAM iterations: team t of iteration `it` streams the packet of slot
// it*PPI+t and leaves its partial sums in that slot.  Last, lane L reads its slot back and
// finalizes its own packet; out/status are written coalesced.  Decode and finalize are
// issued once per 64 packets instead of TEAM times (k_csum repeats them in every team lane),
// and the sort puts packets of similar length in the same iteration, so a ragged batch
// (C3) no longer pays the longest of PPI random packets per iteration.
// ------------------------------------------------------------------------------------------
// Workgroup barrier for LDS exchange between waves: waits for LDS operations only (the fences
// name the local address space), not for the wave's outstanding global loads and stores.
__device__ __forceinline__ void wg_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ void wave_sync_lds() {
    // LDS instructions of one wave execute in program order, so lanes exchanging data through
    // LDS only need the compiler not to move accesses across this point (no memory fence: a
    // fence makes the compiler wait for every outstanding store, vmcnt(0), once per unit)
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// acc + both 16-bit halves of w, one v_sad_u16 (|w.hi - 0| + |w.lo - 0| + acc).  A sum of
// halfwords folds to the same one's-complement value as the sum of the dwords they form (equal
// mod 0xffff, zero only for zero data) and needs no carry chain: one VALU op per dword instead
// of a 64-bit add's two, and one accumulator register instead of two.
__device__ __forceinline__ uint32_t hsum(uint32_t acc, uint32_t w) { return __builtin_amdgcn_sad_u16(w, 0u, acc); }

// Halfword h (0..7) of a 16-B chunk held as four dwords, little-endian.
__device__ __forceinline__ uint32_t pick_half(const uint32_t (&w)[4], uint32_t h) {
    const uint32_t lo = (h & 2u) ? w[1] : w[0], hi = (h & 2u) ? w[3] : w[2];
    const uint32_t d = (h & 4u) ? hi : lo;
    return (h & 1u) ? d >> 16 : d & 0xffffu;
}

// Fast-class trips of one team over its packet's chunks [0, nch): U loads per lane issued
// back to back, then consumed (payload fast path, masked tail, header bitmaps).  Verify: the
// stored checksum fields are one halfword each (the fast class has L3 and L4 at even offsets),
// held by one lane of the team in its first trip; that lane writes it to the slot's q3.w (st_slot:
// L4 field, IP field), instead of every lane summing the fields through all trips for a team
// reduction (two accumulators live across the trip loop: with them the verify build held 95
// VGPRs, 5 waves per SIMD).
template <int TEAM, int U, bool VERIFY, bool NT>
__device__ __forceinline__ void fast_trips(const __amdgpu_buffer_rsrc_t rsrc, uint32_t boff, int nch, int klo,
                                           uint32_t kfast, int l4hi, const uint4 bm, int tl, uint32_t& acc_l4,
                                           uint32_t& acc_ip, uint16_t* st_slot) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    for (int rr = 0; rr * TEAM < nch; rr += U) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = (rr + u) * TEAM + tl;
            const uint32_t bo = k < nch ? boff + ((uint32_t)k << 4) : kOutOfRange;
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, bo, 0, NT ? 2 : 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = (rr + u) * TEAM + tl;
            if ((uint32_t)(k - klo) < kfast) {
                acc_l4 = hsum(hsum(hsum(hsum(acc_l4, v[u].x), v[u].y), v[u].z), v[u].w);
            } else if (k >= klo) {
                const int c = k << 4;
                const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int j = 0; j < 4; ++j) acc_l4 = hsum(acc_l4, w[j] & tailmask(c + 4 * j, l4hi));
            } else if (u * TEAM < 4) {   // header chunks: k < klo <= 4
                const int hb0 = k << 3;
                const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int hb = hb0 + 2 * j;
                    acc_ip = hsum(acc_ip, w[j] & hmask((bm.x >> hb) & 3));
                    acc_l4 = hsum(acc_l4, w[j] & hmask((bm.y >> hb) & 3));
                }
                if (VERIFY) {
                    // each field bitmap holds one bit, the field's halfword in the first 64 B
                    // (chunk = bit >> 3): the lane of that chunk picks the halfword directly
                    const uint32_t fz = (uint32_t)__builtin_ctz(bm.z | 0x80000000u);
                    const uint32_t fw = (uint32_t)__builtin_ctz(bm.w | 0x80000000u);
                    if (bm.z && (int)(fz >> 3) == k) st_slot[1] = (uint16_t)pick_half(w, fz & 7u);
                    if (bm.w && (int)(fw >> 3) == k) st_slot[0] = (uint16_t)pick_half(w, fw & 7u);
                }
            }
            asm volatile("" ::"v"(v[u].x), "v"(v[u].y), "v"(v[u].z), "v"(v[u].w));
        }
    }
}

// One team of TEAM lanes streams the packet of slot sidx (act: the team has one) and leaves its
// {l4, ip, pseudo, stored} sums in the slot's q0.
template <int TEAM, int U, bool VERIFY, bool NT>
__device__ __forceinline__ void tier_team(const __amdgpu_buffer_rsrc_t rsrc, uint4 (*slots)[4], int tl, int sidx,
                                          bool act) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    uint4* sl = slots[act ? sidx : 0];
    uint4 a = sl[0];
    if (!act) a = make_uint4(0, 0, 0, 0);
    const uint32_t boff = a.x;
    const int nch = (int)(a.y & 0xffff);
    const int klo = (int)((a.y >> 16) & 0x3fff);
    const uint32_t kfast = a.z;
    const int l4hi = (int)a.w;
    uint64_t acc_l4 = 0, acc_ip = 0, acc_ps = 0;
    uint32_t st_ip = 0, st_l4 = 0;
    uint32_t h_l4 = 0, h_ip = 0;   // fast class: halfword sums
    if (a.y >> 31) {
        const uint4 bm = sl[1];
        fast_trips<TEAM, U, VERIFY, NT>(rsrc, boff, nch, klo, kfast, l4hi, bm, tl, h_l4, h_ip, (uint16_t*)&sl[3].w);
    } else if (nch > 0) {
        const uint4 q2 = sl[2], q3 = sl[3];
        PktPlan pl;
        pl.r0 = (int)q2.x; pl.l4lo = (int)q2.y; pl.fa = (int)q2.z; pl.iphi = (int)q2.w;
        pl.iplo = (int)q3.x; pl.pslo = (int)q3.y; pl.pshi = (int)q3.z;
        pl.l4hi = l4hi; pl.nch = nch;
        const bool dip = (a.y >> 30) & 1;
        for (int r = 0; r * TEAM < nch; ++r) {
            const int k = r * TEAM + tl;
            const uint32_t bo = k < nch ? boff + ((uint32_t)k << 4) : kOutOfRange;
            const v4u vv = __builtin_amdgcn_raw_buffer_load_b128(rsrc, bo, 0, NT ? 2 : 0);
            const int c = k << 4;
            const uint32_t w[4] = {vv.x, vv.y, vv.z, vv.w};
            if ((uint32_t)(k - klo) < kfast) {
                acc_l4 += (uint64_t)w[0] + w[1];
                acc_l4 += (uint64_t)w[2] + w[3];
            } else if (k >= klo) {
#pragma unroll
                for (int j = 0; j < 4; ++j) acc_l4 += w[j] & tailmask(c + 4 * j, l4hi);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    hdr_dword(w[j], c + 4 * j, pl, dip, acc_l4, acc_ip, acc_ps, st_l4, st_ip, VERIFY);
            }
            asm volatile("" ::"v"(vv.x), "v"(vv.y), "v"(vv.z), "v"(vv.w));
        }
    }
    const uint32_t s_l4 = fold32(team_sum<TEAM>(fold64(acc_l4 + h_l4)));
    const uint32_t s_ip = fold32(team_sum<TEAM>(fold64(acc_ip + h_ip)));
    const uint32_t s_ps = fold32(team_sum<TEAM>(fold64(acc_ps)));
    if (VERIFY && !(a.y >> 31) && nch > 0) {   // the slow class's stored fields: team sums, to q3.w too
        const uint32_t s_st = fold32(team_sum<TEAM>(fold32(st_l4))) | (fold32(team_sum<TEAM>(fold32(st_ip))) << 16);
        if (act && tl == 0) sl[3].w = s_st;
    }
    if (act && tl == 0) sl[0] = make_uint4(s_l4, s_ip, s_ps, 0u);
}

// Phase B of K2 for one tier: slots [s_begin, s_end) streamed by teams of TEAM lanes, 64/TEAM
// packets per iteration.  WT: a last iteration that fills at most half of its teams (the tail of
// the tier's costliest class, in a size-sorted unit) runs with teams of 2 x TEAM lanes, so its
// packets need half the trips.
// it0 / istep: the iterations this wave takes (workgroup-sorted units: every fourth, from the
// wave index).
template <int TEAM, int U, bool VERIFY, bool NT, bool SLOTROT = false, bool WT = false>
__device__ __forceinline__ void stream_tier(const __amdgpu_buffer_rsrc_t rsrc, uint4 (*slots)[4], int lane,
                                            int s_begin, int s_end, uint32_t rot = 0, int it0 = 0, int istep = 1) {
    constexpr int PPI = 64 / TEAM;
    const int tl = lane & (TEAM - 1);
    const int tid = lane / TEAM;
    // rot: this wave starts at iteration rot (mod the count), so that waves whose units are a
    // power-of-two stride apart do not read the same offsets within their units at once
    const int range = s_end - s_begin;
    int nit = (range + PPI - 1) / PPI;
    const int r0 = nit > 0 ? (int)(rot % (uint32_t)(SLOTROT ? range : nit)) : 0;
    const int rem = range % PPI;
    const bool wide = WT && TEAM <= 16 && rot == 0 && rem > 0 && 2 * rem <= PPI;
    if (wide) --nit;
#pragma unroll 1
    for (int it = it0; it < nit; it += istep) {
        int sidx;
        bool act;
        if (SLOTROT) {   // rotation by slots: the wave's first packet is slot r0
            const int q = it * PPI + tid;
            act = q < range;
            sidx = s_begin + (q + r0 < range ? q + r0 : q + r0 - range);
        } else {
            sidx = s_begin + (it + r0 < nit ? it + r0 : it + r0 - nit) * PPI + tid;
            act = sidx < s_end;
        }
        tier_team<TEAM, U, VERIFY, NT>(rsrc, slots, tl, sidx, act);
    }
    if (WT && TEAM <= 16 && wide && it0 == 0) {
        constexpr int T2 = TEAM <= 16 ? 2 * TEAM : TEAM;
        const int sidx = s_begin + nit * PPI + lane / T2;
        tier_team<T2, U, VERIFY, NT>(rsrc, slots, lane & (T2 - 1), sidx, sidx < s_end);
    }
}

// Window chunk c -> LDS slot: rotated by the 256-B row index within its row, so that lanes
// reading the chunks of packets 64 B apart (ds_read_b128, 16-lane groups) hit distinct slots,
// and 8 consecutive lanes writing consecutive chunks (ds_write_b128) still do.
__device__ __forceinline__ uint32_t win_slot(uint32_t c) { return (c & ~15u) | ((c + (c >> 4)) & 15u); }

// The descriptor rules of K2's phase A that depend on the descriptor's fields alone (bounds,
// liveness, raw ranges and rejected flags are checked by the caller): IP version and lengths,
// the L4 checksum field inside the segment, flag combinations.  Wave-uniform arguments give
// scalar code (window units check lane 0's descriptor once for the whole unit).
struct DescRules {
    bool bad, do_ip, do_l4, psonly;
    int fld;
};
__device__ __forceinline__ DescRules desc_rules(int len, int l4o, int ver, int proto, int fl) {
    DescRules r;
    r.do_ip = r.do_l4 = r.psonly = false;
    r.fld = -1;
    bool bad;
    if (ver == 4) bad = len < 20 || l4o < 20 || l4o > len || (l4o & 3);
    else if (ver == 6) bad = len < 40 || l4o < 40 || l4o > len;
    else bad = true;
    if (!bad && (fl & (VPCSUM_F_L4 | VPCSUM_F_L4P))) {
        r.psonly = (fl & VPCSUM_F_L4P) != 0;
        r.fld = l4_field(proto);
        if (r.fld < 0 || (ver == 4 && proto == 58) || len - l4o < r.fld + 2) bad = true;
        else if (r.psonly && ((fl & VPCSUM_F_L4) || proto == 1)) bad = true;
        else r.do_l4 = true;
    }
    if (!bad && (fl & VPCSUM_F_IP)) {
        if (ver != 4) bad = true;
        else r.do_ip = true;
    }
    r.bad = bad;
    return r;
}

// Sums of a window unit's packet in K2's slot format {l4, ip, 0, stored ip << 16} (the caller adds
// the stored L4 field, read from LDS) from x = the packet's chunks (20 dwords from its chunk-aligned start).  L3 starts at dword Q
// + sh bytes (sh 0 or 2: even offsets only), so a[k] = alignbyte(x[Q+k+1], x[Q+k], sh) is L3
// dword k, little-endian, and with IPv4 of 20 B or IPv6 of 40 B every field is at a fixed
// dword: IP checksum a[2] high half, pseudo addresses a[3..4] / a[2..9], the L4 checksum at
// l4o + fld.  Bytes past the packet (a neighbour's) are masked off at dword nd - 1 and beyond.
// An even start gives the sums the same byte orientation as K2's chunk-aligned ones.
template <int Q, bool VERIFY>
__device__ __forceinline__ uint4 win_sums(const uint32_t (&x)[20], int sh, int ver, int proto, int len, int fl) {
    uint32_t a[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) a[k] = __builtin_amdgcn_alignbyte(x[Q + k + 1], x[Q + k], (uint32_t)sh);
    const bool do_ip = (fl & VPCSUM_F_IP) != 0;
    const bool psonly = (fl & VPCSUM_F_L4P) != 0;
    const bool do_l4 = (fl & (VPCSUM_F_L4 | VPCSUM_F_L4P)) != 0;
    const int l4d = ver == 4 ? 5 : 10;
    const int nd = (len + 3) >> 2;
    const uint32_t tail = (len & 3) ? (0xffffffffu >> (8 * (4 - (len & 3)))) : 0xffffffffu;
    uint32_t ip = 0, l4 = 0;   // halfword sums (hsum)
    uint32_t st_ip = 0;
    if (do_ip) {   // IPv4 only (checked with the descriptor)
        ip = hsum(hsum(hsum(hsum(hsum(0u, a[0]), a[1]), a[2] & 0xffffu), a[3]), a[4]);
        st_ip = a[2] >> 16;
    }
    if (do_l4) {
        const int fo = 4 * l4d + l4_field(proto);   // L4 checksum field, bytes from L3
        const int fd = fo >> 2;
        const uint32_t fkeep = (fo & 2) ? 0x0000ffffu : 0xffff0000u;
        if (proto != 1) {
            if (ver == 4) l4 = hsum(hsum(0u, a[3]), a[4]);
            else {
#pragma unroll
                for (int k = 2; k < 10; ++k) l4 = hsum(l4, a[k]);
            }
        }
#pragma unroll
        for (int k = 5; k < 16; ++k) {
            if (k >= l4d && k < nd) {
                uint32_t w = a[k];
                if (k == nd - 1) w &= tail;
                if (k == fd) w &= fkeep;   // the stored field itself: read from LDS by the caller
                if (!psonly) l4 = hsum(l4, w);
            }
        }
    }
    return make_uint4(fold32(l4), fold32(ip), 0u, VERIFY ? (st_ip << 16) : 0u);
}

// One packet's result word and status byte, stored where the unit's owner lanes store them.  The
// index goes through an opaque copy: hoisted, `out + lane` would be a 64-bit per-lane address kept
// live (or spilled) across the whole unit loop for a store issued once per unit.
template <bool NT>
__device__ __forceinline__ void store_result(uint32_t* out, uint8_t* status, uint32_t idx, uint32_t res_out,
                                             uint32_t res_st) {
    asm volatile("" : "+v"(idx));
    if (NT) {
        if (out) __builtin_nontemporal_store(res_out, (__attribute__((address_space(1))) uint32_t*)(out + idx));
        if (status) __builtin_nontemporal_store((uint8_t)res_st, (__attribute__((address_space(1))) uint8_t*)(status + idx));
    } else {
        if (out) out[idx] = res_out;
        if (status) status[idx] = (uint8_t)res_st;
    }
}

// Arenas past 4 GiB (WIN).  K2 addresses frames with 32-bit buffer offsets on one buffer resource,
// so over a larger arena a unit takes the 2-GiB window its first packet starts in: the resource is
// rebuilt per unit for that window (base arena + w x kWinBytes, covering the window plus the 64 KiB
// the largest packet starting in it can reach), and the unit's packets that start elsewhere are
// done afterwards one at a time by the whole wave through the team kernel's 64-bit loads
// (k1_packet, 64 lanes).  Address-sorted batches (an umem's descriptors in frame order) leave such
// packets only in the units that straddle a window line; any order is correct.
constexpr uint64_t kWinBytes = 1ull << 31;
constexpr uint64_t kWinSpan = kWinBytes + 65536;

// K2 body for workgroup `blk` of a grid of `gdim` workgroups (k_csum_d: the launch grid;
// k_csum_service: the persistent service grid, once per batch).
// ROT: large-tier rotation of the wave's slot order, by multiplier |ROT| of the wave index;
// ROT > 0 rotates whole iterations (64 / TEAM packets), ROT < 0 single slots.
// WGS: workgroup-sorted units on mixed batches (below).
template <int TEAM, int U, int TS, int US, bool VERIFY, bool NT, int IL, int ROT = 0, bool SF = false, bool WT = false, bool DS = false, bool WIN = false, bool WGS = false>
__device__ __forceinline__ void k2_run(const uint8_t* __restrict__ arena, uint64_t arena_len,
                                       const uint4* __restrict__ desc, uint32_t n,
                                       uint32_t* __restrict__ out, uint8_t* __restrict__ status,
                                       const uint8_t* __restrict__ flags_override,
                                       uint8_t* __restrict__ arena_w, uint32_t low_grid, uint32_t blk, uint32_t gdim) {
    // slot: q0 {boff, nch | klo<<16 | do_ip<<30 | fast<<31, kfast, l4hi}, q1 bitmaps,
    // q2/q3 the byte-range plan of the slow class; q0 is overwritten with the team's sums.
    __shared__ uint4 s_slot[4][64][4];
    const __amdgpu_buffer_rsrc_t rsrc_all =
        __builtin_amdgcn_make_buffer_rsrc((void*)arena, 0, WIN ? 0 : (int)buf_records(arena_len), 0x00020000);
    const uint64_t arena_len_all = arena_len;
    uint8_t* const arena_w_all = arena_w;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: an SGPR
    // packet of this lane = P0 + lo.  IL = 0: a wave owns 64 consecutive packets.  IL = 1: the 4
    // waves of a workgroup interleave in groups of 8 over 256 consecutive packets, so the teams
    // of the whole workgroup read one contiguous 64-KB window per iteration (one DRAM stream
    // per workgroup instead of four).
    const uint32_t lo = IL == 1 ? (uint32_t)((lane >> 3) * 32 + wid * 8 + (lane & 7)) : (uint32_t)lane;
    // Concurrency by packet size (low_grid > 0).  Large uniform packets stream fastest with few
    // packets in flight (2 workgroups per CU), small and mixed ones need the full grid to hide
    // per-iteration latency.  Every wave reads the same 64 descriptors,
    // spread evenly over the batch, so all waves take the same decision: when every sampled
    // packet is >= 1 KiB the batch runs on the first low_grid workgroups only and the others
    // leave at once.  The decision affects speed only: the grid-stride loop below covers every
    // unit for either grid.
    // Workgroups below low_grid work in either case and fetch their first descriptors before
    // the sample, so the two loads overlap.
    uint32_t grid = gdim;
    uint32_t P0 = IL == 1 ? blk * 256u : (blk * 4u + (uint32_t)wid) * 64u;   // wave-uniform: SGPRs
    uint4 dnext = make_uint4(0, 0, 0, 0);
    int fnext = 0;
    const bool sample = low_grid != 0 && grid > low_grid;
    const bool early = !sample || blk < low_grid;
    if (early && P0 + lo < n) {
        dnext = desc[P0 + lo];
        if (flags_override) fnext = flags_override[P0 + lo];
    }
    // Workgroup-sorted units (WGS, wg): on a batch the sample found mixed (some packets < 1 KiB,
    // some > 64 B: C3), the 4 waves of a workgroup rank their 256 packets by cost class together
    // and stream the workgroup's slots in one order, each wave every fourth iteration of a tier.
    // A wave's own 64 packets hold a class of C3 in a few iterations, the last one partly empty;
    // across 256 such tails are rarer.  Three workgroup barriers per unit (class counts, slots,
    // sums), no window units (the sample rules out all-small batches, where they apply), and the
    // 4 waves run the same number of units.  DESIGN.md §5 item 31.
    bool wg = false;
    if (sample) {
        const uint4 sd = desc[(uint32_t)(((uint64_t)n * (uint32_t)lane) >> 6)];
        if (__ballot((sd.z & 0xffffu) >= 1024u) == ~0ull) grid = low_grid;
        if (blk >= grid) return;   // whole workgroup, before any LDS use
        // sorted units only where the sample holds more than one cost class (a small packet,
        // one trip, two trips, ... of the large tier): a uniform batch of mid-size packets keeps
        // the per-wave units and their rotation
        if (WGS && !WIN && grid == gdim && n < 0xffff0000u) {
            const uint32_t len = sd.z & 0xffffu;
            const uint32_t cls = len <= 64u ? 0u : 1u + (len + 15u) / (16u * kDefaultTeam * kDefaultUnroll);
            wg = __ballot(cls != (uint32_t)__builtin_amdgcn_readfirstlane(cls)) != 0ull;
        }
        if (!early && P0 + lo < n) {
            dnext = desc[P0 + lo];
            if (flags_override) fnext = flags_override[P0 + lo];
        }
    }
    const uint32_t wstride = grid * 4u * 64u;
    // first descriptor in registers before the loop, so that the loop head holds no wait that
    // the back edge (this unit's stores pending) would have to honour too
    asm volatile("" ::"v"(dnext.x), "v"(dnext.y), "v"(dnext.z), "v"(dnext.w), "v"(fnext));
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    // DS: on a batch the sample found to hold large packets (the low-concurrency grid: few,
    // long-lived waves), the out / status words of up to kEsUnits units wait in LDS and are stored
    // together when the wave's staging is full and when it leaves, instead of cutting into the
    // stream of packet reads once per unit.  Other batches (small and
    // mixed packets: short-lived waves, nothing to batch) and waves of fewer than 4 units (C4's
    // 2 per wave: -0.3%) store each unit's words at once.
    const bool stage = DS && grid < gdim && n / 4u >= wstride;
    __shared__ uint32_t s_eo[4][DS ? kEsUnits : 1][64];
    __shared__ uint8_t s_es[4][DS ? kEsUnits : 1][64];
    uint32_t es_n = 0, es_P0 = P0;
    auto es_flush = [&]() {
        // packet index and LDS lane through opaque copies: the addresses are the same for every
        // flush, and hoisted out of the unit loop they would be kept live (or spilled) across it
        uint32_t ln = lo, la = (uint32_t)lane;
        asm volatile("" : "+v"(ln), "+v"(la));
        for (uint32_t k = 0; k < es_n; ++k) {
            const uint32_t p = es_P0 + k * wstride + ln;
            if (p < n) {
                if (NT) {
                    if (out) __builtin_nontemporal_store(s_eo[wid][k][la], (__attribute__((address_space(1))) uint32_t*)(out + p));
                    if (status) __builtin_nontemporal_store(s_es[wid][k][la], (__attribute__((address_space(1))) uint8_t*)(status + p));
                } else {
                    if (out) out[p] = s_eo[wid][k][la];
                    if (status) status[p] = s_es[wid][k][la];
                }
            }
        }
        es_n = 0;
    };
    uint4 (*const flat)[4] = &s_slot[0][0];   // the workgroup's 256 slots (wave w's at 64 w)
    __shared__ uint32_t s_wcnt[16];           // wg: byte w of word b = packets of class b in wave w's unit
    // wg: the loop runs while the workgroup's first packet is in the batch (all 4 waves alike)
    // The unit loop, instantiated twice in the WGS build: with workgroup-sorted units (WGM) and
    // without, so that the batches the sample does not find mixed run the per-wave code as it is
    // in the builds without WGS (one loop with a runtime mode cost C2 0.9%)
    auto unit_loop = [&](auto wgm_tag) {
    constexpr bool WGM = decltype(wgm_tag)::value;
    for (uint32_t Pn; (WGM ? P0 - (uint32_t)wid * 64u : P0) < n; P0 = Pn) {
        // ---- phase A: this lane's packet ----
        const uint4 dv = dnext;
        const int fov = fnext;
        Pn = P0 + wstride;
        {
            const uint32_t q = Pn + lo;
            if (Pn < n && q < n) {
                dnext = desc[q];
                if (flags_override) fnext = flags_override[q];
            }
        }
        bool live = P0 + lo < n;
        const uint64_t off_abs = (uint64_t)dv.x | ((uint64_t)dv.y << 32);
        // WIN: the unit's window (its first packet's, see kWinBytes); packets starting elsewhere
        // (pend) are done after the unit
        uint64_t pend = 0;
        uint64_t wb = 0;
        if (WIN) {
            const uint32_t wsel = __builtin_amdgcn_readfirstlane((uint32_t)(off_abs >> 31));
            const bool inw = (uint32_t)(off_abs >> 31) == wsel;
            pend = __ballot(live && !inw);
            live = live && inw;
            wb = (uint64_t)wsel * kWinBytes;
        }
        // the window's view of the arena (names shadowed for the pass's body)
        const uint64_t arena_len = WIN ? (wb < arena_len_all ? min(kWinSpan, arena_len_all - wb) : 0) : arena_len_all;
        uint8_t* const arena_w = WIN && arena_w_all ? arena_w_all + wb : arena_w_all;
        const __amdgpu_buffer_rsrc_t rsrc =
            WIN ? __builtin_amdgcn_make_buffer_rsrc((void*)(arena + wb), 0, (int)buf_records(arena_len), 0x00020000) : rsrc_all;
        const uint64_t off = off_abs - wb;
        const int len = dv.z & 0xffff;
        const int l4o = dv.z >> 16;
        const int ver = dv.w & 0xff;
        const int proto = (dv.w >> 8) & 0xff;
        const int fl = csum_flags(flags_override ? fov : (int)((dv.w >> 16) & 0xff));

        const int r0 = (int)(off & 15);
        // this lane's descriptor: set by the window check (one scalar check of lane 0's
        // descriptor for the whole unit) or by the per-lane decode below
        bool bad = true, raw = false, do_ip = false, do_l4 = false, psonly = false;
        int fld = -1;
        int key = 0;
        int n_small = 0, n_cls = 0;   // n_cls: distinct cost classes in the large tier
        bool fastu = false;           // window unit (SF): sums in fsums, no slots
        uint4 fsums = make_uint4(0, 0, 0, 0);
        // Window units (SF): the 64 packets of the unit have one shape (descriptor fields, flags
        // and L3 alignment equal to lane 0's: IPv4 without options or IPv6 without extension
        // headers, L3 <= 64 B at an even offset) and lie in 4 KB from lane 0's first chunk, lane
        // 63 last.  The wave reads that window with coalesced 16-B loads (one round trip, 1 KB
        // per instruction) into its LDS slots, and every lane sums its own packet from L3-aligned
        // dwords, where the header fields sit at fixed dwords: no plan, no sort, no team
        // reduction, no per-dword masks.  The sums have K2's slot format.
        if (SF && !WGM) {
            const uint32_t boff = (uint32_t)off & ~15u;
            const uint32_t base = __builtin_amdgcn_readfirstlane(boff);
            const uint32_t rel = boff - base;
            const uint32_t u_rel63 = __builtin_amdgcn_readlane(rel, 63);
            const uint32_t kd = (dv.w & 0xffffu) | ((uint32_t)fl << 16) | ((uint32_t)r0 << 24);
            const uint32_t u_z = __builtin_amdgcn_readfirstlane(dv.z), u_kd = __builtin_amdgcn_readfirstlane(kd);
            const bool cand = live && off <= arena_len && (uint64_t)len <= arena_len - off &&
                              !(fl & (kFlagRejected | VPCSUM_F_RAW)) && dv.z == u_z && kd == u_kd;
            if (__ballot(cand) == ~0ull) {
                const int u_len = (int)(u_z & 0xffff), u_l4o = (int)(u_z >> 16);
                const int u_ver = (int)(u_kd & 0xff), u_r0 = (int)(u_kd >> 24);
                const DescRules ur = desc_rules(u_len, u_l4o, u_ver, (int)((u_kd >> 8) & 0xff), (int)((u_kd >> 16) & 0xff));
                const int nchw = (u_r0 + u_len + 15) >> 4;                     // chunks per packet
                const uint32_t hiw = u_rel63 + 16u * (uint32_t)nchw;           // bytes of the window
                // contiguous: lane 63 last, all within 4 KB of lane 0's first chunk; otherwise
                // (any frame layout, e.g. 2-KB umem frames) gathered, for packets of <= 4 chunks
                const bool contig = __ballot(rel <= u_rel63) == ~0ull && hiw <= 4096u;
                if (!ur.bad && !(u_r0 & 1) && u_len <= 64 && ((u_ver == 4 && u_l4o == 20) || (u_ver == 6 && u_l4o == 40)) &&
                    (contig || nchw <= 4)) {
                    fastu = true;
                    bad = false;
                    do_ip = ur.do_ip;
                    do_l4 = ur.do_l4;
                    psonly = ur.psonly;
                    fld = ur.fld;
                    v4u* win = (v4u*)&s_slot[wid][0][0];
                    // lane index through an opaque copy: the window addresses below are the same
                    // in every unit, and hoisted out of the unit loop they would stay live across
                    // the large tier's phase B (+20 VGPRs, one wave per SIMD less)
                    uint32_t ln = (uint32_t)lane;
                    asm volatile("" : "+v"(ln));
                    uint32_t c0;   // this lane's first chunk in the LDS window
                    if (contig) {
                        v4u c[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const uint32_t cb = (64u * u + ln) << 4;
                            c[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, cb < hiw ? base + cb : kOutOfRange, 0, NT ? 2 : 0);
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) win[win_slot(64u * u + ln)] = c[u];
                        c0 = rel >> 4;
                    } else {
                        // gathered: flat chunk f = 64u + lane is chunk f % nchw of packet f / nchw,
                        // whose first chunk comes from that packet's lane
                        const uint32_t mul = nchw == 1 ? 65536u : nchw == 2 ? 32768u : nchw == 3 ? 21846u : 16384u;
                        v4u c[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const uint32_t f = 64u * u + ln;
                            const uint32_t pk = (f * mul) >> 16;
                            // lane (pk & 63)'s boff: one ds_bpermute (no lane-base arithmetic, which
                            // __shfl adds and the compiler hoists out of the unit loop)
                            const uint32_t src = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((pk & 63u) << 2), (int)boff);
                            c[u] = __builtin_amdgcn_raw_buffer_load_b128(
                                rsrc, u < nchw ? src + ((f - pk * (uint32_t)nchw) << 4) : kOutOfRange, 0, NT ? 2 : 0);
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u)
                            if (u < nchw) win[win_slot(64u * u + ln)] = c[u];
                        c0 = ln * (uint32_t)nchw;
                    }
                    wave_sync_lds();
                    // this lane's chunks [c0, c0 + 5): 20 dwords from its chunk-aligned start
                    uint32_t x[20];
#pragma unroll
                    for (int k = 0; k < 5; ++k) {
                        v4u v = v4u{0, 0, 0, 0};
                        if (k < nchw) v = win[win_slot(c0 + (uint32_t)k)];
                        x[4 * k] = v.x; x[4 * k + 1] = v.y; x[4 * k + 2] = v.z; x[4 * k + 3] = v.w;
                    }
                    const int u_fl = (int)((u_kd >> 16) & 0xff), u_proto = (int)((u_kd >> 8) & 0xff);
                    // verify: the stored L4 field, one LDS halfword at a wave-uniform offset from the
                    // lane's window (instead of a select per dword of win_sums' unrolled loop)
                    uint32_t st_l4f = 0;
                    if (VERIFY && ur.do_l4) {
                        const uint32_t fb = (uint32_t)u_r0 + (u_ver == 4 ? 20u : 40u) + (uint32_t)ur.fld;
                        st_l4f = *(const uint16_t*)((const uint8_t*)&win[win_slot(c0 + (fb >> 4))] + (fb & 15u));
                    }
                    const int q = u_r0 >> 2;
                    if (q == 0) fsums = win_sums<0, VERIFY>(x, u_r0 & 3, u_ver, u_proto, u_len, u_fl);
                    else if (q == 1) fsums = win_sums<1, VERIFY>(x, u_r0 & 3, u_ver, u_proto, u_len, u_fl);
                    else if (q == 2) fsums = win_sums<2, VERIFY>(x, u_r0 & 3, u_ver, u_proto, u_len, u_fl);
                    else fsums = win_sums<3, VERIFY>(x, u_r0 & 3, u_ver, u_proto, u_len, u_fl);
                    if (VERIFY) fsums.w |= st_l4f;
                    // phase C of a window unit, on the unit's (scalar) descriptor values: the
                    // same arithmetic as finish() below, without its per-lane branches
                    {
                        const int u_l4o2 = u_l4o, u_r02 = u_r0;
                        uint32_t l4c = 0, ipc = 0;
                        if (ur.do_l4) {
                            uint32_t tot = orient(fsums.x, u_r02 + u_l4o2);
                            if (u_proto != 1) {
                                const uint32_t l4len = (uint32_t)(u_len - u_l4o2);
                                tot += orient(fsums.z, u_r02) + (uint32_t)u_proto + (l4len & 0xffff) + (l4len >> 16);
                            }
                            if (ur.psonly) l4c = fold32(tot);
                            else {
                                l4c = 0xffff - fold32(tot);
                                if (u_proto == 17 && l4c == 0) l4c = 0xffff;
                            }
                        }
                        if (ur.do_ip) ipc = 0xffff - orient(fsums.y, u_r02);
                        uint32_t st = VPCSUM_S_DONE;
                        if (VERIFY) {
                            if (ur.do_ip && orient(fsums.w >> 16, u_r02) == ipc) st |= VPCSUM_S_IP_OK;
                            if (ur.do_l4) {
                                const uint32_t stored = orient(fsums.w & 0xffff, u_r02 + u_l4o2 + ur.fld);
                                if (stored == l4c) st |= VPCSUM_S_L4_OK;
                                if (!ur.psonly && u_proto == 17 && stored == 0) st |= VPCSUM_S_UDP_NOCSUM;
                            }
                        }
                        asm volatile("" ::"v"(dnext.x), "v"(dnext.y), "v"(dnext.z), "v"(dnext.w), "v"(fnext));
                        const uint32_t res_out = (ipc & 0xffff) | ((l4c & 0xffff) << 16);
                        if (arena_w) {
                            uint8_t* w = arena_w + off;
                            if (ur.do_ip) st_be16_nt(w + 10, ipc);
                            if (ur.do_l4) st_be16_nt(w + u_l4o2 + ur.fld, l4c);
                        }
                        if (DS && stage) {
                            uint32_t la = (uint32_t)lane;   // opaque: see es_flush
                            asm volatile("" : "+v"(la));
                            s_eo[wid][es_n][la] = res_out;
                            s_es[wid][es_n][la] = (uint8_t)st;
                        } else {
                            store_result<NT>(out, status, P0 + lo, res_out, st);
                        }
                    }
                }
            }
        }
        if (!fastu) {
            bad = !live || off > arena_len || (uint64_t)len > arena_len - off || (fl & kFlagRejected);
            raw = (fl & VPCSUM_F_RAW) != 0;
            if (!bad && !raw) {
                const DescRules r = desc_rules(len, l4o, ver, proto, fl);
                bad = r.bad;
                do_ip = r.do_ip;
                do_l4 = r.do_l4;
                psonly = r.psonly;
                fld = r.fld;
            }
        }
        if (!fastu) {
            PktPlan pl;
            pl.r0 = r0;
            const uint32_t boff = (uint32_t)(off & ~(uint64_t)15);
            // pseudo-only (F_L4P): the IP header holds the pseudo addresses, the segment is not read
            const int need = bad ? 0 : psonly ? l4o + fld + 2 : (raw || do_l4) ? len : (do_ip ? l4o : 0);
            pl.nch = (bad || !need) ? 0 : (r0 + need + 15) >> 4;   // no sums (flags 0, F_PRE): no reads
            if (raw) {
                pl.l4lo = r0; pl.l4hi = r0 + len; pl.fa = -64;
                pl.fast_lo = (r0 + 15) & ~15;
            } else if (psonly) {
                pl.l4lo = 0; pl.l4hi = 0; pl.fa = r0 + l4o + fld;
                pl.fast_lo = 1 << 30;
            } else if (do_l4) {
                pl.l4lo = r0 + l4o; pl.l4hi = r0 + len; pl.fa = r0 + l4o + fld;
                pl.fast_lo = (pl.fa + 2 + 15) & ~15;
            } else {
                pl.l4lo = 0; pl.l4hi = 0; pl.fa = -64;
                pl.fast_lo = 1 << 30;
            }
            pl.fast_hi = (r0 + need) & ~15;
            if (do_ip) { pl.iplo = r0; pl.iphi = r0 + l4o; } else { pl.iplo = 0; pl.iphi = 0; }
            if (do_l4 && proto != 1) {
                pl.pslo = r0 + (ver == 4 ? 12 : 8);
                pl.pshi = r0 + (ver == 4 ? 20 : 40);
            } else { pl.pslo = 0; pl.pshi = 0; }
            const int klo = min(pl.fast_lo >> 4, pl.nch);
            const uint32_t kfast = (uint32_t)max((pl.fast_hi >> 4) - klo, 0);
            const bool hbm = !raw && !(r0 & 1) && !(l4o & 1) && ((((r0 + need) & 1) == 0) || r0 + need >= 64);
            uint32_t B_ip = 0, B_l4 = 0, F_ip = 0, F_l4 = 0;
            if (hbm) {
                const int r0h = r0 >> 1;
                if (do_ip) {
                    F_ip = 1u << (r0h + 5);
                    B_ip = hw_range(r0h, r0h + (l4o >> 1)) & ~F_ip;
                }
                if (do_l4) {
                    F_l4 = hw_bit(pl.fa >> 1);
                    B_l4 = psonly ? 0u : hw_range((r0 + l4o) >> 1, (r0 + need + 1) >> 1) & ~F_l4;
                    if (proto != 1) B_l4 |= (ver == 4) ? hw_range(r0h + 6, r0h + 10) : hw_range(r0h + 4, r0h + 20);
                }
            }
            const bool fastc = hbm && klo <= 4;
            // cost class: bad first (key 0), then the small tier (one trip of TS x US chunks),
            // then trips of the large tier's team loop, the slow class last
            if (!bad) {
                if (TS > 0 && fastc && pl.nch <= TS * US) key = 1;
                else key = fastc ? 2 + min((pl.nch + TEAM * U - 1) / (TEAM * U), 12) : 15;
            }
            uint32_t rank = 0, cnt = 0;
            uint32_t kc = 0, kp = 0;   // wg: lane b holds class b's count and offset in this wave
            for (int b = 0; b < 16 && cnt < 64; ++b) {
                const uint64_t m = __ballot(key == b);
                if (key == b)
                    rank = cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                if (WGS && lane == b) {
                    kc = (uint32_t)__popcll(m);
                    kp = cnt;
                }
                cnt += (uint32_t)__popcll(m);
                if (b >= 2 && m) ++n_cls;
                if (b == 1) n_small = (int)cnt;   // keys 0 and 1 go to the small tier
            }
            uint32_t si = (uint32_t)wid * 64u + rank;   // this packet's slot among the workgroup's 256
            if (WGM) {
                // class b's slots: after all classes < b of the workgroup, then those of waves < wid
                if (lane < 16) ((uint8_t*)&s_wcnt[lane])[wid] = (uint8_t)kc;
                wg_sync_lds();
                const uint32_t cw = lane < 16 ? s_wcnt[lane] : 0u;   // the 4 waves' counts of class `lane`
                const uint32_t tot = __builtin_amdgcn_sad_u8(cw, 0u, 0u);
                const uint32_t before = __builtin_amdgcn_sad_u8(cw & ((1u << (8 * wid)) - 1u), 0u, 0u);
                uint32_t incl = tot;   // prefix over lanes 0..15 (one DPP row)
                incl = dpp_add<0x111>(incl);
                incl = dpp_add<0x112>(incl);
                incl = dpp_add<0x114>(incl);
                incl = dpp_add<0x118>(incl);
                const uint32_t first = incl - tot + before - kp;   // class b's first slot, minus its offset here
                si = (uint32_t)__builtin_amdgcn_ds_bpermute(key << 2, (int)first) + rank;
                n_small = __builtin_amdgcn_readlane((int)(incl - tot), 2);
            }
            key = (int)si;   // from here on: this packet's slot
            {
                uint4* sl = flat[si];
                sl[0] = make_uint4(boff, (uint32_t)pl.nch | ((uint32_t)klo << 16) | ((uint32_t)do_ip << 30) | ((uint32_t)fastc << 31),
                                   kfast, (uint32_t)pl.l4hi);
                sl[1] = make_uint4(B_ip, B_l4, F_ip, F_l4);
                if (!fastc) {
                    sl[2] = make_uint4((uint32_t)r0, (uint32_t)pl.l4lo, (uint32_t)pl.fa, (uint32_t)pl.iphi);
                    sl[3] = make_uint4((uint32_t)pl.iplo, (uint32_t)pl.pslo, (uint32_t)pl.pshi, 0u);
                }
            }
        }
        // ---- phase C: finalize this lane's packet from its sums {l4, ip, pseudo, stored} ----
        auto finish = [&](const uint4 sums) {
            uint32_t res_out = 0, res_st = VPCSUM_S_BAD_DESC;
            {
                if (!bad) {
                    uint32_t ipc = 0, l4c = 0;
                    uint32_t st = VPCSUM_S_DONE;
                    if (raw) {
                        ipc = 0xffff - orient(sums.x, r0);
                    } else {
                        if (do_ip) ipc = 0xffff - orient(sums.y, r0);
                        if (do_l4) {
                            uint32_t tot = orient(sums.x, r0 + l4o);
                            if (proto != 1) {
                                const uint32_t l4len = (uint32_t)(len - l4o);
                                tot += orient(sums.z, r0) + (uint32_t)proto + (l4len & 0xffff) + (l4len >> 16);
                            }
                            if (psonly) {
                                l4c = fold32(tot);   // CHECKSUM_PARTIAL: uncomplemented
                            } else {
                                l4c = 0xffff - fold32(tot);
                                if (proto == 17 && l4c == 0) l4c = 0xffff;
                            }
                        }
                        if (VERIFY) {
                            const uint32_t s_ip = orient(sums.w >> 16, r0);
                            if (do_ip && s_ip == ipc) st |= VPCSUM_S_IP_OK;
                            if (do_l4) {
                                const uint32_t stored = orient(sums.w & 0xffff, r0 + l4o + fld);
                                if (stored == l4c) st |= VPCSUM_S_L4_OK;
                                if (!psonly && proto == 17 && stored == 0) st |= VPCSUM_S_UDP_NOCSUM;
                            }
                        }
                        if (arena_w) {
                            uint8_t* w = arena_w + off;
                            if (do_ip) st_be16_nt(w + 10, ipc);
                            if (do_l4) st_be16_nt(w + l4o + fld, l4c);
                        }
                    }
                    res_out = (ipc & 0xffff) | ((l4c & 0xffff) << 16);
                    res_st = st;
                }
            }
            if (DS && stage) {
                uint32_t la = (uint32_t)lane;   // opaque: see es_flush
                asm volatile("" : "+v"(la));
                s_eo[wid][es_n][la] = res_out;
                s_es[wid][es_n][la] = (uint8_t)res_st;
            } else if (live) {
                store_result<NT>(out, status, P0 + lo, res_out, res_st);
            }
        };

        uint4 sums;
        if (fastu) {
            sums = fsums;   // finished above
        } else {
        // ---- phase B: teams stream the packets in slot order ----
        if (WGM) wg_sync_lds();
        else wave_sync_lds();
        // WGM: the workgroup's 256 slots, each wave taking every fourth iteration of a tier, the
        // large tier's round continuing after the wave that took the small tier's last one (the
        // wave's own 64 slots otherwise)
        uint4 (*const tslots)[4] = WGM ? flat : s_slot[wid];
        const int t_end = WGM ? 256 : 64;
        const int it0 = WGM ? wid : 0, istep = WGM ? 4 : 1;
        if (TS > 0) {
            stream_tier<(TS > 0 ? TS : 1), US, VERIFY, NT>(rsrc, tslots, lane, 0, n_small, 0u, it0, istep);
            const int it0l = WGM ? (it0 + 4 - (((n_small + 64 / (TS > 0 ? TS : 1) - 1) / (64 / (TS > 0 ? TS : 1))) & 3)) & 3 : 0;
            stream_tier<TEAM, U, VERIFY, NT, (ROT < 0), WT>(rsrc, tslots, lane, n_small, t_end,
                                             // rotated only when the tier is one cost class: in a
                                             // sorted mixed tier the wrap would pair unlike sizes
                                             (ROT && n_cls == 1 && !WGM) ? (blk * 4u + (uint32_t)wid) * (uint32_t)(ROT < 0 ? -ROT : ROT) : 0u,
                                             it0l, istep);
        } else {
            stream_tier<TEAM, U, VERIFY, NT>(rsrc, tslots, lane, 0, t_end, 0u, it0, istep);
        }
        if (WGM) wg_sync_lds();
        else wave_sync_lds();
        // The next unit's descriptor (loaded a whole unit ago) is taken into registers here,
        // before this unit's stores: vmcnt counts loads and stores together, so a wait for it
        // after the stores would stall the wave until they complete, once per unit.
        asm volatile("" ::"v"(dnext.x), "v"(dnext.y), "v"(dnext.z), "v"(dnext.w), "v"(fnext));
        sums = flat[key][0];
        if (VERIFY) sums.w = flat[key][3].w;   // stored fields {l4, ip << 16}
        }
        if (!fastu) finish(sums);
        wave_sync_lds();   // slots are rewritten by the next super-iteration
        if (WIN) {
            // the unit's packets outside its window: one at a time, the whole wave as one team,
            // 64-bit loads on the whole arena; results where the unit's own go (staged or stored)
            for (uint64_t m = pend; m != 0; m &= m - 1) {
                const int l = (int)__builtin_ctzll(m);
                const uint4 dl = make_uint4(__builtin_amdgcn_readlane(dv.x, l), __builtin_amdgcn_readlane(dv.y, l),
                                            __builtin_amdgcn_readlane(dv.z, l), __builtin_amdgcn_readlane(dv.w, l));
                const int fl_l = __builtin_amdgcn_readlane(fov, l);
                if (DS && stage)
                    k1_packet<64, 4, VERIFY, false>(arena, arena_len_all, dl, fl_l, flags_override != nullptr, (uint32_t)l,
                                                    &s_eo[wid][es_n][0], &s_es[wid][es_n][0], arena_w_all, lane);
                else
                    k1_packet<64, 4, VERIFY, NT>(arena, arena_len_all, dl, fl_l, flags_override != nullptr, P0 + (uint32_t)l,
                                                 out, status, arena_w_all, lane);
            }
            wave_sync_lds();
        }
        if (DS && stage && ++es_n == kEsUnits) {
            es_flush();
            es_P0 = Pn;
        }
    }
    };
    if (WGS && wg) unit_loop(std::integral_constant<bool, WGS>{});
    else unit_loop(std::false_type{});
    if (DS && stage) es_flush();
}

// Occupancy of a K2 build: WPE > 1 forces that many waves per SIMD (tuning variants).  The default
// shape's verify and staging builds are held to 6 (80 VGPRs), the unstaged compute build's natural
// count: left alone, the compiler gave them 95 and 92 (5 waves) -- the verify build for its stored
// fields, the staging build because its 26 KB of LDS let it budget for fewer resident waves
// (DESIGN.md §5 items 25, 28).  tests/test_kernel_resources.py holds all of them to 80, no scratch.
template <int TEAM, int U, int TS, int US, bool VERIFY, int WPE, int IL, int ROT, bool SF, bool WT, bool DS, bool WIN = false, bool WGS = false>
constexpr int k2_waves_per_eu() {
    return WPE > 1 ? WPE
                   : (TEAM == kDefaultTeam && U == kDefaultUnroll && TS == kSmallTeam && US == kSmallUnroll &&
                      IL == 0 && ROT == kDefaultRot && SF && !WT && (VERIFY || DS || WIN || WGS))
                         ? 6
                         : 1;
}

template <int TEAM, int U, int TS, int US, bool VERIFY, bool NT, int WPE = 1, int IL = 0, int ROT = 0, bool SF = false, bool WT = false, bool DS = false, bool WIN = false, bool WGS = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(k2_waves_per_eu<TEAM, U, TS, US, VERIFY, WPE, IL, ROT, SF, WT, DS, WIN, WGS>()))) void k_csum_d(const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                const uint4* __restrict__ desc, uint32_t n,
                                                uint32_t* __restrict__ out, uint8_t* __restrict__ status,
                                                const uint8_t* __restrict__ flags_override,
                                                uint8_t* __restrict__ arena_w, uint32_t low_grid) {
    k2_run<TEAM, U, TS, US, VERIFY, NT, IL, ROT, SF, WT, DS, WIN, WGS>(arena, arena_len, desc, n, out, status, flags_override,
                                                                       arena_w, low_grid, blockIdx.x, gridDim.x);
}

// ------------------------------------------------------------------------------------------
// Low-latency service: the checksum on a persistent grid of kServiceGrid workgroups that polls
// a host mailbox (internal.h SvcMailbox) instead of being launched per batch, for the small
// flushes of Iface.completeTx (XDPIface.java:227-243) on a registered umem, where a kernel
// launch plus an event wait cost more than the work.  Thread 0 of workgroup 0 alone polls the
// command word at system scope and relays it to the other workgroups through a device-memory
// word (32 pollers of one host line slowed each poll's round trip 2-4x, tools/bar_probe.cpp).
// A batch is processed by the workgroups that own a packet (one packet per wave, grid-stride);
// each of them releases its results at system scope and bumps a device counter, and the one
// that completes the count resets it and publishes `done`.  The grid leaves on kSvcStop or
// after idle_ticks (100 MHz s_memrealtime) without a batch (workgroup 0 relays the stop); the
// host relaunches it on demand and re-runs a batch that a leaving grid left unfinished
// (idempotent: checksum fields are excluded from the sums they hold).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_csum_service(SvcMailbox* mb, uint32_t* __restrict__ ctr, uint32_t seen,
                                                      uint64_t idle_ticks, uint32_t poll) {
    // batch parameters, read over PCIe by thread 0 when the host flags them as changed and kept
    // in LDS across batches: arena, arena_len, arena_w, desc, out, status, opts, pre
    __shared__ uint64_t s_par[8];
    __shared__ uint64_t s_cmd;
    __shared__ uint4 s_idesc[kSvcInlineDesc];   // workgroup 0: the inline descriptors of the batch
    __shared__ uint32_t s_inl;
#ifdef VPCSUM_SVC_STAMPS
    __shared__ uint64_t s_ts;
#endif
    bool have_par = false;
    uint64_t* relay = reinterpret_cast<uint64_t*>(ctr + 2);   // zeroed with the counter at launch
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        uint64_t got = 0;
        if (blockIdx.x == 0) {
            if (threadIdx.x < 64) {
                // the grid's only reader of the host mailbox: lanes 0..3 of wave 0 read its first
                // 64-B line in one request per poll -- the command word and the inline descriptors
                const int lane = threadIdx.x;
                u32x4_t q = {0u, 0u, 0u, 0u};
                const u32x4_t* line = reinterpret_cast<const u32x4_t*>(mb) + (lane & 3);
                for (;;) {
                    if (lane < 4)   // system-coherent, uncached; volatile: re-read every poll
                        asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
                                     : "=v"(q) : "v"(line) : "memory");
                    const uint64_t w = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(q.y) << 32) |
                                       (uint32_t)__builtin_amdgcn_readfirstlane(q.x);
                    if (w & kSvcStop) break;
                    if ((uint32_t)w != seen) { got = w; break; }
                    const uint64_t idle = __builtin_amdgcn_s_memrealtime() - t0;
                    if (idle > idle_ticks) break;
                    // back off after 50 us without a batch: ~1 us more latency, far fewer PCIe reads
                    if (idle > 5000) __builtin_amdgcn_s_sleep(40);
                    else __builtin_amdgcn_s_sleep(1);
                }
                // inline descriptors: lane 1 + k holds descriptor k.  They are used only when every
                // one the batch needs carries this batch's tag; otherwise (a line read that caught
                // the host mid-write) the batch takes them from the descriptor buffer, which the
                // host filled before the command word.
                const uint32_t ni = (uint32_t)(got >> 32) & kSvcMaxPkts;
                const bool need = (got & kSvcInline) && lane >= 1 && lane <= kSvcInlineDesc && (uint32_t)lane <= ni;
                const bool ok = need && (q.w >> 24) == (got & 0xffu);
                const bool all = __ballot(ok) == __ballot(need);
                if (ok) s_idesc[lane - 1] = make_uint4(q.x, q.y, q.z, q.w);
                if (lane == 0) {
                    s_inl = (got & kSvcInline) && all ? 1u : 0u;
                    // to the other workgroups: the command, or a stop when the grid leaves
                    __hip_atomic_store(relay, got ? got : (kSvcStop | seen), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        } else if (threadIdx.x == 0) {
            // the relay in device memory, read with RELAXED loads (poll bit 0, the default): the
            // system-scope acquire after the loop orders the batch's reads.  An acquire load per
            // poll is a cache invalidate per poll; from 31 workgroups polling it slowed launched
            // batches beside an idle grid by 6-17% (profiles/r06f_svc_poll.json; relaxed: +0.2%).
            // A/B tooling (VPCSUM_SVC_POLL): bit 0 clear = acquire loads (round 5), bit 1 back off to
            // s_sleep 40 after 50 us without a batch, bit 2 read the clock every 64th poll only
            for (uint32_t k = 0;; ++k) {
                const uint64_t w = (poll & 1) ? __hip_atomic_load(relay, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                              : __hip_atomic_load(relay, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                if (w & kSvcStop) break;
                if (w && (uint32_t)w != seen) { got = w; break; }
                // workgroup 0 relays a stop before it leaves; this bound only guards the grid
                // against a relay that never comes
                if (!(poll & 4) || (k & 63) == 0) {
                    const uint64_t idle = __builtin_amdgcn_s_memrealtime() - t0;
                    if (idle > 2 * idle_ticks + 100000) break;
                    if ((poll & 2) && idle > 5000) {
                        __builtin_amdgcn_s_sleep(40);
                        continue;
                    }
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        if (threadIdx.x == 0) {
#ifdef VPCSUM_SVC_STAMPS
            const uint64_t ts_seen = __builtin_amdgcn_s_memrealtime();
            if (blockIdx.x == 0) mb->stamp[0] = ts_seen;
            s_ts = ts_seen;
#endif
            // acquire at system scope: the frames, descriptors and parameters the host wrote
            // before the command word are read fresh (no kernel boundary invalidates caches here)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            const uint32_t next = seen + 1 ? seen + 1 : 1;   // the host's sequence skips 0
            if (got && ((got & kSvcParams) || !have_par || (uint32_t)got != next)) {
                // the parameter line in one round trip: three independent 16-B loads
                typedef unsigned int v4u __attribute__((ext_vector_type(4)));
                const v4u* pb = (const v4u*)&mb->arena;
                v4u q[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) q[k] = __builtin_nontemporal_load(pb + k);
                s_par[0] = (uint64_t)q[0].x | ((uint64_t)q[0].y << 32);   // arena
                s_par[1] = (uint64_t)q[0].z | ((uint64_t)q[0].w << 32);   // arena_len
                s_par[2] = (uint64_t)q[1].x | ((uint64_t)q[1].y << 32);   // arena_w
                s_par[3] = (uint64_t)q[1].z | ((uint64_t)q[1].w << 32);   // desc
                s_par[4] = (uint64_t)q[2].x | ((uint64_t)q[2].y << 32);   // out
                s_par[5] = (uint64_t)q[2].z | ((uint64_t)q[2].w << 32);   // status
                const v4u q3 = __builtin_nontemporal_load(pb + 3);   // opts, pre (same line)
                s_par[6] = (uint64_t)q3.x | ((uint64_t)q3.y << 32);
                s_par[7] = (uint64_t)q3.z | ((uint64_t)q3.w << 32);
            }
            s_cmd = got;
#ifdef VPCSUM_SVC_STAMPS
            if (blockIdx.x == 0) mb->stamp[1] = __builtin_amdgcn_s_memrealtime();
#endif
        }
        __syncthreads();
        const uint64_t cmd = s_cmd;
        const uint8_t* arena = (const uint8_t*)s_par[0];
        const uint64_t alen = s_par[1];
        uint8_t* arena_w = (uint8_t*)s_par[2];
        // a batch of up to kSvcInlineDesc frames runs on workgroup 0 alone (below), from the
        // descriptors that came with the command
        const uint4* desc = (blockIdx.x == 0 && s_inl) ? (const uint4*)s_idesc : (const uint4*)s_par[3];
        uint32_t* out = (uint32_t*)s_par[4];
        uint8_t* status = (uint8_t*)s_par[5];
        const bool pred = (s_par[6] & kSvcOptClampLoads) == 0;
        const bool rel_done = (s_par[6] & kSvcOptReleaseDone) != 0;
        const void* s_aux = (const void*)s_par[7];   // the aux buffer: pre-images, or parse results
        const void* pre = (cmd & kSvcPre) ? s_aux : nullptr;
        const void* hsum = (cmd & kSvcHsum) ? s_aux : nullptr;   // RX verify: header sums into the aux buffer
        const int pre_fmt = (cmd & kSvcPreFmt) ? 1 : 0;
        __syncthreads();   // s_cmd / s_par are rewritten next round
        if (cmd == 0) return;
        have_par = true;
        const uint32_t n = (uint32_t)(cmd >> 32) & kSvcMaxPkts;
        // only the workgroups that own a packet take part (packet p goes to wave p mod the grid's
        // waves, workgroup (p / 4) mod grid): a flush of a few frames waits for no relay
        const uint32_t nwg = max(1u, min(gridDim.x, (n + 3u) / 4u));
        if (blockIdx.x < nwg) {
        // one wave per packet: a small flush is a few PCIe round trips deep (descriptor, frame
        // bytes, results) instead of K2's per-unit iterations, which a latency of ~3 us per
        // round trip would serialize
        if (pred) {
            if ((cmd & kSvcVerify) && (cmd & kSvcFrames))
                k1_run<64, 4, true, true, true, 2>(arena, alen, desc, n, out, status, nullptr, arena_w, blockIdx.x, gridDim.x,
                                                   hsum);
            else if (cmd & kSvcVerify)
                k1_run<64, 4, true, true, true>(arena, alen, desc, n, out, status, nullptr, arena_w, blockIdx.x, gridDim.x);
            else if ((cmd & kSvcFrames) && (cmd & kSvcParse))
                k1_run<64, 4, false, true, true, 3>(arena, alen, desc, n, out, status, nullptr, arena_w, blockIdx.x,
                                                    gridDim.x, (const void*)s_aux);
            else if (cmd & kSvcFrames)
                k1_run<64, 4, false, true, true, 2>(arena, alen, desc, n, out, status, nullptr, arena_w, blockIdx.x, gridDim.x);
            else
                k1_run<64, 4, false, true, true, 1>(arena, alen, desc, n, out, status, nullptr, arena_w, blockIdx.x,
                                                    gridDim.x, pre, pre_fmt);
        } else {
            if ((cmd & kSvcVerify) && (cmd & kSvcFrames))
                k1_run<64, 4, true, true, false, 2>(arena, alen, desc, n, out, status, nullptr, arena_w, blockIdx.x, gridDim.x,
                                                    hsum);
            else if (cmd & kSvcVerify)
                k1_run<64, 4, true, true>(arena, alen, desc, n, out, status, nullptr, arena_w, blockIdx.x, gridDim.x);
            else if ((cmd & kSvcFrames) && (cmd & kSvcParse))
                k1_run<64, 4, false, true, false, 3>(arena, alen, desc, n, out, status, nullptr, arena_w, blockIdx.x,
                                                     gridDim.x, (const void*)s_aux);
            else if (cmd & kSvcFrames)
                k1_run<64, 4, false, true, false, 2>(arena, alen, desc, n, out, status, nullptr, arena_w, blockIdx.x, gridDim.x);
            else
                k1_run<64, 4, false, true, false, 1>(arena, alen, desc, n, out, status, nullptr, arena_w, blockIdx.x,
                                                     gridDim.x, pre, pre_fmt);
        }
        // the workgroup's stores are complete (barrier); thread 0 releases them system-wide and
        // counts the workgroup; the last participating workgroup publishes `done`
        __syncthreads();
        if (threadIdx.x == 0) {
#ifdef VPCSUM_SVC_STAMPS
            if (blockIdx.x == 0) mb->stamp[2] = __builtin_amdgcn_s_memrealtime();
#endif
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
#ifdef VPCSUM_SVC_STAMPS
            if (blockIdx.x == 0) mb->stamp[3] = __builtin_amdgcn_s_memrealtime();
#endif
            // a batch of one workgroup (up to 4 frames) publishes without the device counter.
            // The fence above has made this workgroup's results visible system-wide before the
            // count, so the count needs no release of its own, and neither does the `done` store
            // of a one-workgroup batch (one L2 write-back each).  With more workgroups `done`
            // keeps its release: it must not overtake the counter reset, or the next batch's
            // counts could land before it.  kSvcOptReleaseDone restores both (A/B tooling)
            uint32_t d = 0;
            if (nwg > 1)
                d = rel_done ? __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT)
                             : __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef VPCSUM_SVC_STAMPS
            if (blockIdx.x == 0) mb->stamp[4] = __builtin_amdgcn_s_memrealtime();
#endif
            if (d + 1 == nwg) {
                // the other workgroups' results were released at system scope by their own fences
                // before their (relaxed) counts; this acquire orders the reset and `done` after
                // them in the memory model as well (an L1 invalidate, no write-back)
                if (nwg > 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#ifdef VPCSUM_SVC_STAMPS
                mb->stamp[5] = __builtin_amdgcn_s_memrealtime();
                mb->stamp[6] = s_ts;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
#endif
                if (nwg > 1) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (rel_done || nwg > 1)
                    __hip_atomic_store(&mb->done, (uint32_t)cmd, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                else
                    __hip_atomic_store(&mb->done, (uint32_t)cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        }
        seen = (uint32_t)cmd;
        t0 = __builtin_amdgcn_s_memrealtime();
    }
}

hipError_t launch_service(SvcMailbox* d_mb, uint32_t* d_ctr, uint32_t seen, uint64_t idle_ticks, hipStream_t stream,
                          uint32_t grid, uint32_t poll) {
    hipLaunchKernelGGL(k_csum_service, dim3(grid), dim3(256), 0, stream, d_mb, d_ctr, seen, idle_ticks, poll);
    return hipGetLastError();
}

__global__ void k_spin_probe(uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(40);
}

hipError_t launch_spin_probe(uint32_t wgs, uint32_t threads, uint64_t ticks, hipStream_t stream) {
    hipLaunchKernelGGL(k_spin_probe, dim3(wgs), dim3(threads), 0, stream, ticks);
    return hipGetLastError();
}

// Grid of the grid-stride kernels: 12 workgroups per CU (2.4 waves of residency at 5 waves per
// SIMD) was the best grid-stride shape across C2 / C3 (tools/sweep.py --bpc).
static uint32_t default_grid() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    return (uint32_t)num_cus(dev) * 12u;
}
// Grid of K2 for dense small frames: one resident round of the build launched.  Workgroups of
// one K2 build resident per CU (its VGPR and LDS use: 6 for the unstaged compute build at 79
// VGPRs, which dense frames take; 5 for the verify build at 95 and the staging build at 92),
// looked up once per build.
static uint32_t resident_wgs(const void* kern) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 256, 0) != hipSuccess || nb <= 0) nb = 5;
    return (uint32_t)nb;
}
// Low-concurrency grid of K2 for batches of large packets: 2 workgroups per CU.
static uint32_t default_low_grid() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    return (uint32_t)num_cus(dev) * 2u;
}

template <int TEAM, int U, int TS = 0, int US = 1, int WPE = 1, int IL = 0, int ROT = 0, bool SF = false, bool WT = false, bool DS = false, bool WIN = false, bool WGS = false>
static hipError_t launch_d(const uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* desc, uint32_t n,
                           uint32_t* out, uint8_t* status, const uint8_t* flags_override, bool verify, bool nt,
                           uint8_t* arena_w, int grid, bool adapt, hipStream_t stream) {
    if ((!WIN && arena_len > kMaxBufArena) || ((uintptr_t)arena & 15))
        return launch_team<TEAM, U>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w,
                                    grid > 0 ? grid : default_grid(), stream);
    uint32_t need = (n + 255) / 256;   // 4 waves x 64 packets per workgroup
    uint32_t g = grid > 0 ? (uint32_t)grid : default_grid();
    // sampled low-concurrency grid: default grid only, not with IL (its units are per workgroup),
    // and only when the arena is large enough to hold n packets of >= 1 KiB without overlap
    // (otherwise the sample cannot succeed and its load latency would be pure cost)
    const uint32_t low_grid =
        (grid > 0 || IL == 1 || !adapt || arena_len < (uint64_t)n * 1024u) ? 0u : default_low_grid();
    // Dense small frames (at most 128 arena bytes per packet): one resident round of workgroups
    // beats the grid-stride default (C1 window units at 6 per CU: 4.91 vs 4.63 TB/s at 5 and
    // 4.65 at 12); the arena size alone tells, no sample needed.
    const bool dense = grid <= 0 && adapt && IL != 1 && arena_len <= (uint64_t)n * 128u;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const uint32_t cus = (uint32_t)num_cus(dev);
#define VPC_LAUNCH(V, N)                                                                                         \
    do {                                                                                                         \
        auto kern = k_csum_d<TEAM, U, TS, US, V, N, WPE, IL, ROT, SF, WT, DS, WIN, WGS>;                             \
        uint32_t gg = g;                                                                                         \
        if (dense) {                                                                                             \
            static const uint32_t res = resident_wgs((const void*)kern);                                         \
            gg = min(gg, res * cus);                                                                             \
        }                                                                                                        \
        if (gg > need) gg = need;                                                                                \
        if (gg == 0) gg = 1;                                                                                     \
        hipLaunchKernelGGL(kern, dim3(gg), dim3(256), 0, stream, arena, arena_len, (const uint4*)desc, n, out,   \
                           status, flags_override, arena_w, low_grid);                                            \
    } while (0)
    if (verify) {
        if (nt) VPC_LAUNCH(true, true); else VPC_LAUNCH(true, false);
    } else {
        if (nt) VPC_LAUNCH(false, true); else VPC_LAUNCH(false, false);
    }
#undef VPC_LAUNCH
    return hipGetLastError();
}

hipError_t launch_csum(const uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* desc, uint32_t n,
                       uint32_t* out, uint8_t* status, const uint8_t* flags_override, uint32_t mode,
                       uint8_t* arena_w, int team_log2, int grid_override, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const bool verify = (mode & VPCSUM_MODE_VERIFY) != 0;
    const int grid = grid_override;   // <= 0: each launcher's default
    // mode bit 13 (internal tuning): plain loads instead of non-temporal ones
    const bool nt = (mode & 0x2000u) == 0;
    // mode bit 14 (internal tuning): K2 without the sampled low-concurrency grid
    const bool adapt = (mode & 0x4000u) == 0;
    // variant = (lanes per packet, chunks in flight per lane); ids 2..6 are log2(lanes)
#define VPC_T(T, U) launch_team<T, U>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, \
                                      grid > 0 ? grid : (int)default_grid(), stream)
    switch (team_log2) {
        case 2: return VPC_T(4, 4);
        case 3: return VPC_T(8, 4);
        case 4: return VPC_T(16, 8);
        case 5: return VPC_T(32, 4);
        case 6: return VPC_T(64, 4);
        case 7: return VPC_T(4, 8);
        case 8: return VPC_T(8, 6);
        case 9: return VPC_T(8, 12);
        case 10: return VPC_T(16, 4);
        case 11: return VPC_T(8, 8);
        // zero-copy frames in host memory: one wave per packet, predicated loads (k1_run PRED)
        case 12: return launch_team<64, 4, true>(arena, arena_len, desc, n, out, status, flags_override, verify, nt,
                                                 arena_w, grid > 0 ? grid : (int)default_grid(), stream);
        case 40: return launch_d<8, 6>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        case 41: return launch_d<4, 12>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        case 43: return launch_d<16, 6>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        case 45: return launch_d<2, 12>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        case 46: return launch_d<8, 6, 2, 4>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        case 47: return launch_d<8, 6, 1, 4>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        case 48: return launch_d<8, 8, 2, 4>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        case 49: return launch_d<8, 6, 4, 4>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        case 50: return launch_d<8, 6, 2, 2>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        case 54: return launch_d<8, 4, 2, 2>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        case 58: return launch_d<8, 12, 2, 2>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        case 62: return launch_d<8, 6, 2, 2, 1, 1>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        case 66: return launch_d<8, 6, 2, 2, 1, 0, 1>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        // 70: the default; 72: the default without window units (A/B)
        case 72: return launch_d<kDefaultTeam, kDefaultUnroll, kSmallTeam, kSmallUnroll, 1, 0, kDefaultRot, false>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        case 74: return launch_d<kDefaultTeam, kDefaultUnroll, kSmallTeam, kSmallUnroll, 1, 0, kDefaultRot, true, true>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        // 76: the default without staged result stores (A/B)
        case 76: return launch_d<kDefaultTeam, kDefaultUnroll, kSmallTeam, kSmallUnroll, 1, 0, kDefaultRot, true, false, false>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        // 78: the team kernel with 64-bit loads, which serves arenas past 4 GiB (A/B, tooling)
        case 78: return launch_team<kDefaultTeam, kDefaultUnroll>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid > 0 ? grid : (int)default_grid(), stream);
        // 79: the staging build on every batch (round 3's r03w default, A/B)
        case 79: return launch_d<kDefaultTeam, kDefaultUnroll, kSmallTeam, kSmallUnroll, 1, 0, kDefaultRot, true, false, true>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        // 84: the default for non-dense batches (the staging build with workgroup-sorted units on
        // mixed batches); 79 is the same build without the workgroup sort
        case 84:
            if (arena_len > kMaxBufArena) return hipErrorInvalidValue;
            return launch_d<kDefaultTeam, kDefaultUnroll, kSmallTeam, kSmallUnroll, 1, 0, kDefaultRot, true, false, true, false, true>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        case 70:
        case 0:
            // Arenas past 4 GiB: K2 with a pass per 2-GiB window its units' packets start in (see
            // kWinBytes); not 16-B aligned: the team kernel (launch_d's fallback)
            if (arena_len > kMaxBufArena) {
                if (grid <= 0 && adapt && arena_len <= (uint64_t)n * 128u)
                    return launch_d<kDefaultTeam, kDefaultUnroll, kSmallTeam, kSmallUnroll, 1, 0, kDefaultRot, true, false, false, true>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
                return launch_d<kDefaultTeam, kDefaultUnroll, kSmallTeam, kSmallUnroll, 1, 0, kDefaultRot, true, false, true, true>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
            }
            // Dense small frames (at most 128 arena bytes per packet: C1) never stage their result
            // words: they take the build without staging and its smaller LDS
            if (grid <= 0 && adapt && arena_len <= (uint64_t)n * 128u)
                return launch_d<kDefaultTeam, kDefaultUnroll, kSmallTeam, kSmallUnroll, 1, 0, kDefaultRot, true, false, false>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
            // everything else: the staging build, whose mixed batches take workgroup-sorted units
            // (k2_run WGS)
            return launch_d<kDefaultTeam, kDefaultUnroll, kSmallTeam, kSmallUnroll, 1, 0, kDefaultRot, true, false, true, false, true>(arena, arena_len, desc, n, out, status, flags_override, verify, nt, arena_w, grid, adapt, stream);
        default: return hipErrorInvalidValue;   // unknown kernel variant id
    }
#undef VPC_T
}

// ------------------------------------------------------------------------------------------
// Parse kernel (one lane per frame): an Ethernet frame as the vswitch receives it (tap / XDP:
// PacketBuffer.init -> EthernetPacket.from(raw, allowPartial=true), EthernetPacket.java:25-94),
// reduced to what the checksum needs.  The EtherType picks Ipv4Packet.initPartial
// (Ipv4Packet.java:29-63, no version check) or Ipv6Packet.initPartial (Ipv6Packet.java:26-59, no
// version check unless an extension header forces the full Ipv6Packet.from, :69-159).  The L4
// part follows initPartial (TCP >= 20 B, UDP >= 8 B, ICMP >= 1 B) or, behind an extension header,
// the full from() (TCP options, the UDP length field, ICMP >= 8 B).  A frame whose IP packet the
// reference refuses (it becomes PacketBytes, EthernetPacket.java:60-64) gets S_BAD_DESC: no
// checksum applies to it.  Extension headers follow the reference's ExtHeader.from (8 + hdrExtLen
// bytes); a chain of two or more, and a TCP option of length 0, make the reference loop forever,
// and a TCP option of length 1 or an empty ICMP message make it throw: such frames are refused.
// Restated in Python by oracle/oracle.py:parse_ether (the tests compare the two frame by frame).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ bool v6_needs_next(int h) {
    return h == 0 || h == 60 || h == 43 || h == 44 || h == 51 || h == 50 || h == 135 || h == 139 || h == 140 ||
           h == 253 || h == 254;
}

// EtherIPPacket.initPartial / from (EtherIPPacket.java:32-71): >= 2 B, the inner Ethernet header,
// and an inner ARP that parses (ArpPacket.java:22-70); inner IP failures do not propagate.
__device__ bool pe_etherip(const uint8_t* s, uint32_t len) {
    if (len < 2) return false;
    const uint8_t* f = s + 2;
    const uint32_t L = len - 2;
    if (L < 14) return false;
    uint32_t typ = ld16(f + 12), hl = 14;
    if (typ == 0x8100) {
        if (L < 18) return false;
        typ = ld16(f + 16);
        hl = 18;
    }
    if (typ == 0x0806) {
        const uint32_t a = L - hl;
        if (a < 8) return false;
        const uint32_t hs = f[hl + 4], ps = f[hl + 5];
        if (a < 8 + 2 * (hs + ps)) return false;
    }
    return true;
}

// TcpPacket.from (TcpPacket.java:223-287) with the option walk and TcpOption.check (:602-640).
__device__ bool pe_tcp_from(const uint8_t* s, uint32_t len) {
    if (len < 20) return false;
    const uint32_t doff = ((s[12] >> 4) & 15u) * 4u;
    if (doff > len) return false;
    if (doff > 20) {
        uint32_t off = 20;
        while (off < doff) {   // at most 40 option bytes
            const uint32_t kind = s[off];
            if (kind == 0 || kind == 1) {
                off += 1;
                if (kind == 0) break;
                continue;
            }
            if (off + 1 >= doff) return false;
            const uint32_t ln = s[off + 1];
            if (off + ln > doff || ln < 2) return false;
            if ((kind == 3 && ln != 3) || (kind == 2 && ln != 4)) return false;
            off += ln;
        }
    }
    return true;
}

// The upper-layer packet of an IP packet: initPartial (partial = true; TcpPacket.java:187-199,
// UdpPacket.java:17-27, IcmpPacket.java:22-26) or the full from() (UdpPacket.java:40-60,
// IcmpPacket.java:33-45).  ICMPv6 exists only inside IPv6 (Ipv4Packet.java:146-163 maps 58 to
// PacketBytes); anything without a parser is PacketBytes and always accepted.
__device__ bool pe_l4(bool partial, int ver, int proto, const uint8_t* s, uint32_t len) {
    if (proto == 6) return partial ? len >= 20 : pe_tcp_from(s, len);
    if (proto == 17) return partial ? len >= 8 : (len >= 8 && ld16(s + 4) == len);
    if (proto == 1 || (ver == 6 && proto == 58)) return partial ? len >= 1 : len >= 8;
    if (proto == 97) return pe_etherip(s, len);
    return true;
}

// Ipv6Packet.from (Ipv6Packet.java:69-159) over avail bytes at b.
__device__ bool pe_ipv6_from(const uint8_t* b, uint32_t avail, uint32_t& total, int& l4o, int& proto) {
    if (avail < 40 || (b[0] >> 4) != 6) return false;
    const uint32_t pl = ld16(b + 4);
    const int nh = b[6];
    if (pl == 0 || 40 + pl > avail) return false;
    total = 40 + pl;
    proto = nh;
    l4o = 40;
    if (v6_needs_next(nh)) {
        if (pl < 8) return false;
        const int nxt = b[40], hlen = b[41];
        if (pl < (uint32_t)(8 + hlen) || v6_needs_next(nxt)) return false;
        proto = nxt;
        l4o = 40 + 8 + hlen;
    }
    const uint32_t seg = total - (uint32_t)l4o;
    if (proto == 59 && seg != 0) return false;   // IPv6_NEXT_HEADER_NO_NEXT_HEADER with bytes
    return pe_l4(false, 6, proto, b + l4o, seg);
}

// One frame at f (frame bytes: the arena, or a staged copy of at least its first 384 B -- no byte
// past offset 381 is ever read: 18 B of Ethernet / 802.1Q, 40 + 8 + 255 of IPv6 and its extension
// header, 60 of TCP header), o its arena offset, L its length, ok its bounds check: the descriptor
// (flags from w: egress, every flag must be honoured; ingress, those the frame allows) and the
// status byte (0 = parsed, S_BAD_DESC = refused).
__device__ __forceinline__ uint8_t parse_frame(const uint8_t* f, uint64_t o, uint32_t L, bool ok, uint8_t w, bool egress,
                                               vpcsum_desc_t& d) {
    d.l3_off = 0; d.l3_len = 0; d.l4_off = 0; d.l3_ver = 0; d.l4_proto = 0; d.flags = 0; d.rsv = 0;
    uint8_t st = VPCSUM_S_BAD_DESC;
    ok = ok && L >= 14;
    uint32_t hl = 14, typ = 0;
    if (ok) {
        typ = ld16(f + 12);
        if (typ == 0x8100) {
            if (L < 18) ok = false;
            else { typ = ld16(f + 16); hl = 18; }
        }
    }
    if (ok) {
        const uint8_t* b = f + hl;
        const uint32_t avail = L - hl;
        if (typ == 0x0800 && avail >= 20) {
            // Ipv4Packet.initPartial: the EtherType decided IPv4, the version nibble is not read
            const uint32_t ihl = b[0] & 15u;
            const uint32_t total = ld16(b + 2);
            if (avail >= ihl * 4 && ihl >= 5 && total >= ihl * 4 && total <= avail &&
                pe_l4(true, 4, b[9], b + ihl * 4, total - ihl * 4)) {
                d.l3_off = o + hl; d.l3_len = (uint16_t)total; d.l4_off = (uint16_t)(ihl * 4);
                d.l3_ver = 4; d.l4_proto = b[9];
                st = 0;
            }
        } else if (typ == 0x86DD && avail >= 40) {
            uint32_t total = 0;
            int l4o = 40, proto = b[6];
            bool good;
            if (v6_needs_next(b[6])) {
                good = pe_ipv6_from(b, avail, total, l4o, proto);   // initPartial defers to from()
            } else {
                const uint32_t pl = ld16(b + 4);
                total = 40 + pl;
                good = pl != 0 && total <= avail && pe_l4(true, 6, proto, b + 40, pl);
            }
            // l3_len is 16 bits: an IPv6 packet above 65535 B (payloadLength > 65495) cannot be
            // described (it never fits a umem frame); refused
            if (good && total <= 0xffff) {
                d.l3_off = o + hl; d.l3_len = (uint16_t)total; d.l4_off = (uint16_t)l4o;
                d.l3_ver = 6; d.l4_proto = (uint8_t)proto;
                st = 0;
            }
        }
    }
    if (st == 0) {
        // fwant (egress): the frame's own flags, all of which must be honoured -- a frame that
        // cannot take one (an IPv4 header sum on IPv6, an L4 sum its segment does not hold, a
        // pseudo-header sum for ICMPv4) is refused, so nothing is written and the caller hands
        // it back.  want (ingress): the sums the frame allows, of those asked.
        uint8_t fl = 0;
        const bool ip_ok = d.l3_ver == 4;
        const int fld = l4_field(d.l4_proto);
        const bool l4_ok = fld >= 0 && !(d.l3_ver == 4 && d.l4_proto == 58) && d.l3_len - d.l4_off >= fld + 2;
        if ((w & VPCSUM_F_IP) && ip_ok) fl |= VPCSUM_F_IP;
        if ((w & VPCSUM_F_L4) && l4_ok) fl |= VPCSUM_F_L4;
        else if ((w & VPCSUM_F_L4P) && l4_ok && d.l4_proto != 1) fl |= VPCSUM_F_L4P;
        if (egress && (fl != (w & (VPCSUM_F_IP | VPCSUM_F_L4 | VPCSUM_F_L4P)) ||
                      (w & ~(VPCSUM_F_IP | VPCSUM_F_L4 | VPCSUM_F_L4P)) || (fl & VPCSUM_F_L4 && fl & VPCSUM_F_L4P))) {
            st = VPCSUM_S_BAD_DESC;
            d.l3_off = 0; d.l3_len = 0; d.l4_off = 0; d.l3_ver = 0; d.l4_proto = 0;
            fl = 0;
        }
        d.flags = fl;
    }
    return st;
}

// The flow tuple the L4 input nodes read (vpcsum.h vpcsum_tuple_t) of a parsed frame, from its L3
// bytes at b: addresses at Ipv4Packet :51-54 (12, 16) / Ipv6Packet :47-50 (8, 24), ports and TCP
// flags at TcpPacket / UdpPacket.initPartial (0, 2, 12); zeros for a refused frame (st != 0).
__device__ __forceinline__ void frame_tuple(const uint8_t* b, const vpcsum_desc_t& d, uint32_t st, uint32_t t[10]) {
    for (int k = 0; k < 10; ++k) t[k] = 0;
    if (st != 0) return;
    auto put = [&](int dw0, const uint8_t* src, int nb) {   // bytes in memory order
        if (!((uintptr_t)src & 1)) {   // halfword loads where the field is 2-B aligned
            const uint16_t* h = (const uint16_t*)src;
            for (int k = 0; k < nb / 2; ++k) t[dw0 + (k >> 1)] |= (uint32_t)h[k] << (16 * (k & 1));
        } else {
            for (int k = 0; k < nb; ++k) t[dw0 + (k >> 2)] |= (uint32_t)src[k] << (8 * (k & 3));
        }
    };
    if (d.l3_ver == 4) {
        put(0, b + 12, 4);
        put(4, b + 16, 4);
    } else {
        put(0, b + 8, 16);
        put(4, b + 24, 16);
    }
    const uint8_t* l4 = b + d.l4_off;
    uint32_t w8 = d.l3_ver | ((uint32_t)d.l4_proto << 8);
    if (d.l4_proto == 6 || d.l4_proto == 17) {   // accepted: at least 8 / 20 bytes
        put(8, l4, 4);
        if (d.l4_proto == 6) w8 |= (uint32_t)(l4[13] & 0x3f) << 16;
    }
    t[9] = w8;
}

__global__ __launch_bounds__(256) void k_parse_ether(const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                    const uint64_t* __restrict__ foff,
                                                    const uint32_t* __restrict__ flen, uint32_t n, uint8_t want,
                                                    const uint8_t* __restrict__ fwant,
                                                    vpcsum_desc_t* __restrict__ desc, uint8_t* __restrict__ status,
                                                    vpcsum_tuple_t* __restrict__ tuples, uint2* __restrict__ hsum) {
    // 64 tuples of a wave are staged here and written as 10 coalesced 256-B stores
    __shared__ uint32_t s_tu[256 * 10];
    const uint32_t ln = threadIdx.x & 63u;
    // q: the wave's first frame (wave-uniform, so that every lane of the wave reaches the
    // tuple exchange, also in the batch's last, partial wave)
    for (uint32_t q = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); q < n; q += gridDim.x * blockDim.x) {
        const uint32_t p = q + ln;
        const bool act = p < n;
        const uint64_t o = act ? foff[p] : 0;
        const uint32_t L = act ? flen[p] : 0;
        vpcsum_desc_t d;
        const uint8_t w = act ? (fwant ? fwant[p] : want) : 0;
        const uint8_t st = parse_frame(arena + o, o, L, act && o <= arena_len && (uint64_t)L <= arena_len - o, w,
                                       fwant != nullptr, d);
        if (act) {
            desc[p] = d;
            if (status) status[p] = st;
            // the ingress header sum (vpcsum_hsum_t) from the same header bytes
            if (hsum)
                hsum[p] = st == 0 ? hsum_record(arena + d.l3_off, d.l3_ver, d.l4_proto, d.l3_len, d.l4_off, (int)(d.l3_off - o))
                                  : make_uint2(0u, 0u);
        }
        if (tuples) {
            // the flow tuple the L4 input nodes read (vpcsum.h vpcsum_tuple_t): addresses at
            // Ipv4Packet :51-54 (12, 16) / Ipv6Packet :47-50 (8, 24), ports and TCP flags at
            // TcpPacket / UdpPacket.initPartial (0, 2, 12); zeros for a refused frame
            uint32_t t[10];
            frame_tuple(arena + d.l3_off, d, st, t);
            uint32_t* wt = s_tu + (threadIdx.x & ~63u) * 10;   // this wave's 64 x 10 dwords
            for (int k = 0; k < 10; ++k) wt[ln * 10 + k] = t[k];
            wave_sync_lds();
            uint32_t* dst = (uint32_t*)(tuples + q);   // 4-B aligned (checked by the API)
            const uint32_t nd = min(64u, n - q) * 10u;
            for (uint32_t j = 0; j < 10; ++j) {
                const uint32_t i = j * 64u + ln;
                if (i < nd) dst[i] = wt[i];
            }
            wave_sync_lds();   // the slots are rewritten by the wave's next frames
        }
    }
}

hipError_t launch_parse_ether(const uint8_t* arena, uint64_t arena_len, const uint64_t* frame_off,
                              const uint32_t* frame_len, uint32_t n, uint8_t flags, vpcsum_desc_t* desc,
                              uint8_t* status, vpcsum_tuple_t* tuples, hipStream_t stream,
                              const uint8_t* frame_flags, vpcsum_hsum_t* hsum) {
    if (n == 0) return hipSuccess;
    uint32_t g = (n + 255) / 256;
    if (g > 65535u * 8) g = 65535u * 8;
    hipLaunchKernelGGL(k_parse_ether, dim3(g), dim3(256), 0, stream, arena, arena_len, frame_off, frame_len, n,
                       flags, frame_flags, desc, status, tuples, (uint2*)hsum);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Read-roof probe: plain streaming dwordx4 read of `bytes`, XOR-reduced per block.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_read_probe(const uint4* __restrict__ buf, uint64_t n16,
                                                   uint32_t* __restrict__ sink) {
    // Each workgroup streams one contiguous slab, 8 x 16 B per lane in flight, non-temporal
    // (the fastest pure-read shape measured by tools/bwlab.hip: ~6.9-7.0 TB/s on MI355X).
    uint32_t x = 0;
    const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per;
    const uint64_t hi = min(lo + per, n16);
    uint64_t i = lo + threadIdx.x;
    for (; i + 7 * 256 < hi; i += 8 * 256) {
        uint4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = ld_stream<true>(buf + i + u * 256);
#pragma unroll
        for (int u = 0; u < 8; ++u) x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < hi; i += 256) {
        const uint4 a = buf[i];
        x ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    for (int m = 32; m >= 1; m >>= 1) x ^= __shfl_xor(x, m, 64);
    if ((threadIdx.x & 63) == 0) atomicXor(&sink[blockIdx.x], x);
}

hipError_t launch_read_probe(const uint8_t* buf, uint64_t bytes, uint32_t* sink, uint32_t grid, hipStream_t stream) {
    if (grid == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        grid = num_cus(dev) * 8;
    }
    hipLaunchKernelGGL(k_read_probe, dim3(grid), dim3(256), 0, stream, (const uint4*)buf, bytes / 16, sink);
    return hipGetLastError();
}

// Pattern ceiling of a batch: the same 16-B chunk reads as K2's large tier (teams of 8 lanes,
// 6 non-temporal buffer loads in flight per lane, out-of-range chunks predicated off), and no
// checksum work.  Grid-stride over packets, one team per packet.
template <bool PIPE>
__global__ __launch_bounds__(256) void k_pattern_probe(const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                       const uint4* __restrict__ desc, uint32_t n,
                                                       uint32_t* __restrict__ sink, uint32_t order) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    constexpr int TEAM = 8, U = 6;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)arena, 0, (int)buf_records(arena_len), 0x00020000);
    const int tl = threadIdx.x & (TEAM - 1);
    const uint32_t nteams = gridDim.x * (256 / TEAM);
    uint32_t x = 0;
    // order 0: the grid's teams walk consecutive packets.  order 1: K2's order (a wave owns 64
    // consecutive packets, its 8 teams take them 8 at a time; units grid-strided).
    const uint32_t tpw = 64 / TEAM;
    const uint32_t wave = (blockIdx.x * 256 + threadIdx.x) >> 6, nwaves = gridDim.x * 4;
    const uint32_t tw = (threadIdx.x & 63) / TEAM;
    auto packet = [&](uint32_t i) -> uint32_t {   // i-th packet of this team, ~0u past the end
        uint32_t p;
        if (order == 0) {
            p = (blockIdx.x * 256 + threadIdx.x) / TEAM + i * nteams;
        } else {
            const uint32_t unit = wave + (i / 8) * nwaves;
            if (unit * 64 >= n) return ~0u;
            p = unit * 64 + (i % 8) * tpw + tw;
            if (p >= n) return ~1u;   // a hole in a partial unit: skip
        }
        return p < n ? p : ~0u;
    };
    auto issue = [&](v4u* v, uint32_t boff, int nch, int rr) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = (rr + u) * TEAM + tl;
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, k < nch ? boff + ((uint32_t)k << 4) : kOutOfRange, 0, 2);
        }
    };
    if (!PIPE) {
        for (uint32_t i = 0;; ++i) {
            const uint32_t p = packet(i);
            if (p == ~0u) break;
            if (p == ~1u) continue;
            const uint4 d = desc[p];
            const uint32_t boff = d.x & ~15u;
            const int nch = (int)(((d.x & 15) + (d.z & 0xffff) + 15) >> 4);
            for (int rr = 0; rr * TEAM < nch; rr += U) {
                v4u v[U];
                issue(v, boff, nch, rr);
#pragma unroll
                for (int u = 0; u < U; ++u) x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
            }
        }
    } else {
        // the next trip's loads are issued before the current trip is consumed, so the team
        // always has U loads per lane in flight (descriptors prefetched one packet ahead)
        uint32_t i = 0, p = packet(0);
        while (p == ~1u) p = packet(++i);
        if (p != ~0u) {
            uint4 d = desc[p];
            uint32_t pn = packet(i + 1), in = i + 1;
            while (pn == ~1u) pn = packet(++in);
            uint4 dn = pn != ~0u ? desc[pn] : make_uint4(0, 0, 0, 0);
            uint32_t boff = d.x & ~15u;
            int nch = (int)(((d.x & 15) + (d.z & 0xffff) + 15) >> 4);
            int rr = 0;
            v4u a[U], b[U];
            issue(a, boff, nch, rr);
            for (;;) {
                rr += U;
                bool last = false;
                if (rr * TEAM >= nch) {   // next packet
                    if (pn == ~0u) {
                        last = true;
                    } else {
                        d = dn;
                        boff = d.x & ~15u;
                        nch = (int)(((d.x & 15) + (d.z & 0xffff) + 15) >> 4);
                        rr = 0;
                        i = in;
                        pn = packet(i + 1), in = i + 1;
                        while (pn == ~1u) pn = packet(++in);
                        if (pn != ~0u) dn = desc[pn];
                    }
                }
                if (!last) issue(b, boff, nch, rr);
#pragma unroll
                for (int u = 0; u < U; ++u) x ^= a[u].x ^ a[u].y ^ a[u].z ^ a[u].w;
                if (last) break;
#pragma unroll
                for (int u = 0; u < U; ++u) a[u] = b[u];
            }
        }
    }
    for (int m = 32; m >= 1; m >>= 1) x ^= __shfl_xor(x, m, 64);
    if ((threadIdx.x & 63) == 0) atomicXor(&sink[blockIdx.x & 1023], x);
}

hipError_t launch_pattern_probe(const uint8_t* arena, uint64_t arena_len, const void* desc, uint32_t n, uint32_t* sink,
                                uint32_t grid, hipStream_t stream) {
    // tooling: grid bit 31 selects K2's packet order, bit 30 the software-pipelined trip stream
    const uint32_t order = grid >> 31;
    const bool pipe = (grid >> 30) & 1;
    grid &= 0x3fffffffu;
    if (grid == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        grid = num_cus(dev) * 8;
    }
    if (pipe)
        hipLaunchKernelGGL(k_pattern_probe<true>, dim3(grid), dim3(256), 0, stream, arena, arena_len, (const uint4*)desc,
                           n, sink, order);
    else
        hipLaunchKernelGGL(k_pattern_probe<false>, dim3(grid), dim3(256), 0, stream, arena, arena_len,
                           (const uint4*)desc, n, sink, order);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Synthetic workload generator: same bytes as oracle/csum_oracle.c:orc_synth_frame.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t rng(uint64_t seed, uint64_t pkt, uint64_t word) {
    const uint64_t ctr = (pkt << 20) | (word & 0xFFFFFull);
    return mix64(seed + (ctr + 1) * 0x9E3779B97F4A7C15ull);
}

struct Shape { int ver, proto, l3_len, l4_off; };

__device__ Shape shape_of(uint32_t workload, uint64_t seed, uint64_t pkt) {
    Shape s = {4, 6, 1500, 20};
    const uint64_t r = rng(seed, pkt, 0xFFFFF);
    switch (workload) {
        case VPCSUM_SYNTH_C1_UDP64: s.proto = 17; s.l3_len = 50; break;
        case VPCSUM_SYNTH_C2_TCP1500: break;
        case VPCSUM_SYNTH_C3_MIXED: {
            const int lens[3] = {64, 576, 1500};
            const int protos[3] = {17, 6, 1};
            s.l3_len = lens[r % 3];
            s.proto = protos[(r / 3) % 3];
            break;
        }
        case VPCSUM_SYNTH_C4_V6JUMBO: s.ver = 6; s.proto = 6; s.l3_len = 9000; s.l4_off = 40; break;
        case VPCSUM_SYNTH_C5_NAT1500: s.proto = (r & 1) ? 17 : 6; break;
        default: {
            const int protos4[4] = {6, 17, 1, 6};
            const int protos6[4] = {6, 17, 58, 17};
            s.ver = (r & 1) ? 6 : 4;
            if (s.ver == 4) {
                s.proto = protos4[(r >> 1) & 3];
                s.l4_off = 20 + 4 * (int)((r >> 3) % 11);
            } else {
                s.proto = protos6[(r >> 1) & 3];
                s.l4_off = 40;
            }
            const int minl4 = (s.proto == 6) ? 20 : 8;
            uint32_t span = 1600;
            if (((r >> 8) & 15) == 0) span = 9000;
            s.l3_len = s.l4_off + minl4 + (int)((r >> 12) % span);
            if (s.l3_len > 9000) s.l3_len = 9000;
            if (((r >> 40) & 63) == 0) s.l3_len = s.l4_off + minl4;
            break;
        }
    }
    return s;
}

// One block per packet: threads fill the payload 8 bytes at a time, then thread 0 writes
// the header fields (same order as the oracle: payload first, headers overwrite).  arena NULL:
// the descriptors alone.
__global__ __launch_bounds__(256) void k_synth(uint8_t* __restrict__ arena, uint32_t n, uint32_t stride,
                                              uint32_t l3_pad, uint32_t workload, uint64_t seed,
                                              uint64_t first, vpcsum_desc_t* __restrict__ desc) {
    if (!arena) {   // descriptors only: one lane per packet
        for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
            const Shape s = shape_of(workload, seed, first + p);
            vpcsum_desc_t d;
            d.l3_off = (uint64_t)p * stride + l3_pad;
            d.l3_len = (uint16_t)s.l3_len;
            d.l4_off = (uint16_t)s.l4_off;
            d.l3_ver = (uint8_t)s.ver;
            d.l4_proto = (uint8_t)s.proto;
            d.flags = (uint8_t)((s.ver == 4 ? VPCSUM_F_IP : 0) | VPCSUM_F_L4);
            d.rsv = 0;
            desc[p] = d;
        }
        return;
    }
    for (uint32_t p = blockIdx.x; p < n; p += gridDim.x) {
        const uint64_t pkt = first + p;
        const Shape s = shape_of(workload, seed, pkt);
        uint8_t* l3 = arena + (uint64_t)p * stride + l3_pad;
        const int nw = (s.l3_len + 7) >> 3;
        for (int w = threadIdx.x; w < nw; w += blockDim.x) {
            const uint64_t v = rng(seed, pkt, (uint64_t)w);
            const int b0 = w * 8;
            if ((((uintptr_t)(l3 + b0)) & 7) == 0 && b0 + 8 <= s.l3_len) {
                *(uint64_t*)(l3 + b0) = v;
            } else {
                for (int b = 0; b < 8 && b0 + b < s.l3_len; ++b) l3[b0 + b] = (uint8_t)(v >> (8 * b));
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            if (s.ver == 4) {
                l3[0] = (uint8_t)(0x40 | (s.l4_off / 4));
                l3[1] = 0;
                l3[2] = (uint8_t)(s.l3_len >> 8); l3[3] = (uint8_t)s.l3_len;
                l3[6] = 0x40; l3[7] = 0;
                l3[8] = 64; l3[9] = (uint8_t)s.proto;
                l3[10] = 0; l3[11] = 0;
            } else {
                const int pl = s.l3_len - 40;
                l3[0] = 0x60; l3[1] &= 0x0f;
                l3[4] = (uint8_t)(pl >> 8); l3[5] = (uint8_t)pl;
                l3[6] = (uint8_t)s.proto; l3[7] = 64;
            }
            uint8_t* l4 = l3 + s.l4_off;
            const int l4len = s.l3_len - s.l4_off;
            if (s.proto == 6) {
                l4[12] = 0x50; l4[13] = 0x10; l4[16] = 0; l4[17] = 0; l4[18] = 0; l4[19] = 0;
            } else if (s.proto == 17) {
                l4[4] = (uint8_t)(l4len >> 8); l4[5] = (uint8_t)l4len; l4[6] = 0; l4[7] = 0;
            } else {
                l4[0] = (s.proto == 58) ? 128 : 8; l4[1] = 0; l4[2] = 0; l4[3] = 0;
            }
            if (desc) {
                vpcsum_desc_t d;
                d.l3_off = (uint64_t)p * stride + l3_pad;
                d.l3_len = (uint16_t)s.l3_len;
                d.l4_off = (uint16_t)s.l4_off;
                d.l3_ver = (uint8_t)s.ver;
                d.l4_proto = (uint8_t)s.proto;
                d.flags = (uint8_t)((s.ver == 4 ? VPCSUM_F_IP : 0) | VPCSUM_F_L4);
                d.rsv = 0;
                desc[p] = d;
            }
        }
        __syncthreads();
    }
}

hipError_t launch_synth(uint8_t* arena, uint64_t arena_len, uint32_t n, uint32_t stride, uint32_t l3_pad,
                        uint32_t workload, uint64_t seed, uint64_t first_index, vpcsum_desc_t* desc,
                        hipStream_t stream) {
    if (n == 0) return hipSuccess;
    uint32_t g = n < 65536u ? n : 65536u;
    hipLaunchKernelGGL(k_synth, dim3(g), dim3(256), 0, stream, arena, n, stride, l3_pad, workload, seed,
                       first_index, desc);
    return hipGetLastError();
}

}  // namespace vpcsum
