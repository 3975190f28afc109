/*
 * csum_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of vproxy's Java checksum path, used as the parity checker for
 * libvpcsum.so and as the timed CPU baseline ("Java-algorithm C", kind "port") in
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this; the product path (vproxy_amd/, libvpcsum.so) never does.
 *
 * Parity pin: checked against every known-answer vector in the reference's TestPacket.java
 * (IP 0x76b8 / ICMP 0x4d5a, ICMPv6 0xd4ec, IP 0x87e4 / TCP 0xf3ff, IP 0x85f7 / TCP 0x0aa9,
 * IP 0x7f41 / UDP 0xdf0d, EtherIP 0xfc82 / 0x2c7a / 0xee43) and the 31 IPv4 frames of the
 * reference's pcap fixtures -- see tests/golden/ and tests/test_oracle_golden.py.
 *
 * Every function restates the Java code line by line (per-16-bit-word add, end-around carry
 * folded at EVERY step, odd tail byte as the high byte), not an optimised variant.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <pthread.h>
#include "../include/vpcsum.h"

/* Utils.calculateChecksumIntermediate -- base/src/main/java/io/vproxy/base/util/Utils.java:783-797 */
uint32_t orc_csum_intermediate(uint32_t sum, const uint8_t* a, uint32_t limit) {
    for (uint32_t i = 0; i < limit / 2; ++i) {
        sum += ((uint32_t)a[i * 2] << 8) | a[i * 2 + 1];       /* ByteArray.uint16: big endian */
        while (sum > 0xffff) {
            sum = (sum & 0xffff) + 1;
        }
    }
    if (limit % 2 != 0) {
        sum += ((uint32_t)a[limit - 1] << 8);
        while (sum > 0xffff) {
            sum = (sum & 0xffff) + 1;
        }
    }
    return sum;
}

/* Utils.calculateChecksumDoFinal -- Utils.java:799-801 */
uint32_t orc_csum_final(uint32_t sum) { return 0xffff - sum; }

/* Utils.calculateChecksum -- Utils.java:778-781 */
uint32_t orc_csum(const uint8_t* a, uint32_t limit) {
    return orc_csum_final(orc_csum_intermediate(0, a, limit));
}

/* Same per-step loop, but over a virtual concatenation pseudo || seg, with the 16-bit
 * checksum field at seg[fld..fld+1] read as zero (Java zeroes it in place with
 * raw.pktBuf.int16(off, 0) before summing, TcpPacket.java:476, UdpPacket.java:137,
 * IcmpPacket.java:69/129).  The pseudo header always has even length (12 or 40), so the
 * word grid continues unchanged across the concatenation (CompositeByteArray semantics). */
static uint32_t orc_sum_seg_zero_field(uint32_t sum, const uint8_t* seg, uint32_t len, uint32_t fld) {
    for (uint32_t i = 0; i < len / 2; ++i) {
        uint32_t o = i * 2;
        uint32_t b0 = (o == fld || o == fld + 1) ? 0 : seg[o];
        uint32_t b1 = (o + 1 == fld || o + 1 == fld + 1) ? 0 : seg[o + 1];
        sum += (b0 << 8) | b1;
        while (sum > 0xffff) sum = (sum & 0xffff) + 1;
    }
    if (len % 2 != 0) {
        uint32_t o = len - 1;
        uint32_t b0 = (o == fld || o == fld + 1) ? 0 : seg[o];
        sum += b0 << 8;
        while (sum > 0xffff) sum = (sum & 0xffff) + 1;
    }
    return sum;
}

/* Utils.buildPseudoIPv4Header -- Utils.java:758-766: src(4) dst(4) 0 proto len16 */
static void orc_pseudo4(const uint8_t* l3, uint32_t proto, uint32_t upper_len, uint8_t out[12]) {
    memcpy(out, l3 + 12, 4);
    memcpy(out + 4, l3 + 16, 4);
    out[8] = 0;
    out[9] = (uint8_t)proto;
    out[10] = (uint8_t)(upper_len >> 8);   /* ByteArray.int16 */
    out[11] = (uint8_t)upper_len;
}

/* Utils.buildPseudoIPv6Header -- Utils.java:768-776: src(16) dst(16) len32 0 0 0 nh */
static void orc_pseudo6(const uint8_t* l3, uint32_t proto, uint32_t upper_len, uint8_t out[40]) {
    memcpy(out, l3 + 8, 16);
    memcpy(out + 16, l3 + 24, 16);
    out[32] = (uint8_t)(upper_len >> 24);  /* ByteArray.int32 */
    out[33] = (uint8_t)(upper_len >> 16);
    out[34] = (uint8_t)(upper_len >> 8);
    out[35] = (uint8_t)upper_len;
    out[36] = 0; out[37] = 0; out[38] = 0;
    out[39] = (uint8_t)proto;
}

/* Ipv4Packet.__updateChecksum -- Ipv4Packet.java:209-217 (+ calculateChecksum :300-302):
 * zero [10..11], Utils.calculateChecksum(pktBuf, ihl*4). */
uint32_t orc_ipv4_header_csum(const uint8_t* l3, uint32_t ihl_bytes) {
    uint32_t sum = orc_sum_seg_zero_field(0, l3, ihl_bytes, 10);
    return orc_csum_final(sum);
}

/* Offset of the 16-bit checksum field inside the L4 header, or -1 when the protocol
 * carries none the reference computes.  TCP 16 (TcpPacket.java:476), UDP 6
 * (UdpPacket.java:137), ICMP/ICMPv6 2 (IcmpPacket.java:69, 129). */
int orc_l4_field(uint32_t proto) {
    switch (proto) {
        case 6: return 16;
        case 17: return 6;
        case 1: return 2;
        case 58: return 2;
        default: return -1;
    }
}

/* TcpPacket.updateChecksumWithIPv4/IPv6 (TcpPacket.java:475-485, 508-518),
 * UdpPacket.updateChecksumWithIPv4/IPv6 (UdpPacket.java:136-164: result 0 -> 0xffff),
 * IcmpPacket.__updateChecksum (v4, IcmpPacket.java:64-74: NO pseudo header) and
 * IcmpPacket.updateChecksumWithIPv6 (IcmpPacket.java:124-135: pseudo nh=58).
 * The pseudo-header length is the L4 buffer length, raw.pktBuf.length() (= l3_len - l4_off),
 * and its protocol is the constant of the class (Consts.java:24-29), not the header field. */
int orc_l4_csum(const uint8_t* l3, uint32_t l3_len, uint32_t l4_off, uint32_t ver, uint32_t proto,
                uint32_t* out) {
    int fld = orc_l4_field(proto);
    if (fld < 0) return -1;
    if (ver == 4 && proto == 58) return -1;   /* ICMPv6 only inside IPv6 */
    /* IPv6 + proto 1: Ipv6Packet.__updateChildrenChecksum (Ipv6Packet.java:232-234) calls
     * packet.updateChecksum() -> IcmpPacket v4 path -> no pseudo header (branch below). */
    if (l4_off > l3_len) return -1;
    uint32_t seg_len = l3_len - l4_off;
    if (seg_len < (uint32_t)fld + 2) return -1;
    const uint8_t* seg = l3 + l4_off;
    uint32_t sum = 0;
    if (proto == 1) {
        sum = orc_sum_seg_zero_field(0, seg, seg_len, (uint32_t)fld);
    } else if (ver == 4) {
        uint8_t ph[12];
        orc_pseudo4(l3, proto, seg_len, ph);
        sum = orc_csum_intermediate(0, ph, 12);
        sum = orc_sum_seg_zero_field(sum, seg, seg_len, (uint32_t)fld);
    } else {
        uint8_t ph[40];
        orc_pseudo6(l3, proto, seg_len, ph);
        sum = orc_csum_intermediate(0, ph, 40);
        sum = orc_sum_seg_zero_field(sum, seg, seg_len, (uint32_t)fld);
    }
    uint32_t c = orc_csum_final(sum);
    if (proto == 17 && c == 0) c = 0xffff;
    *out = c;
    return 0;
}

/* One descriptor, the batched restatement of the dirty-flag walk
 * (AbstractPacket.updateChecksum :58-65 -> Ipv4Packet.__updateChecksum/__updateChildrenChecksum
 * :209-234, Ipv6Packet :219-236).  Semantics mirror libvpcsum's kernel contract. */
void orc_process_one(const uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* d,
                     uint32_t mode, uint32_t* out_word, uint8_t* out_status, uint8_t* arena_w) {
    uint32_t ipc = 0, l4c = 0;
    uint8_t st = VPCSUM_S_DONE;
    uint64_t off = d->l3_off;
    uint32_t len = d->l3_len;
    if (off > arena_len || (uint64_t)len > arena_len - off) {
        if (out_word) *out_word = 0;
        if (out_status) *out_status = VPCSUM_S_BAD_DESC;
        return;
    }
    const uint8_t* l3 = arena + off;
    if (d->flags & VPCSUM_F_RAW) {
        ipc = orc_csum(l3, len);
        if (out_word) *out_word = ipc;
        if (out_status) *out_status = st;
        return;
    }
    int bad = 0;
    if (d->l3_ver == 4) {
        if (len < 20 || d->l4_off < 20 || d->l4_off > len || (d->l4_off & 3)) bad = 1;
    } else if (d->l3_ver == 6) {
        if (len < 40 || d->l4_off < 40 || d->l4_off > len) bad = 1;
    } else {
        bad = 1;
    }
    int do_l4 = 0, psonly = 0;
    if (!bad && (d->flags & VPCSUM_F_L4P)) {
        /* checksum offload: pseudo-header sum only (CHECKSUM_PARTIAL convention) */
        int fld = orc_l4_field(d->l4_proto);
        if ((d->flags & VPCSUM_F_L4) || fld < 0 || d->l4_proto == 1) bad = 1;
        else if (d->l3_ver == 4 && d->l4_proto == 58) bad = 1;
        else if (len - d->l4_off < (uint32_t)fld + 2) bad = 1;
        else do_l4 = 1, psonly = 1;
    }
    if (!bad && (d->flags & VPCSUM_F_L4)) {
        int fld = orc_l4_field(d->l4_proto);
        if (fld < 0) bad = 1;
        else if (d->l3_ver == 4 && d->l4_proto == 58) bad = 1;
        else if (len - d->l4_off < (uint32_t)fld + 2) bad = 1;
        else do_l4 = 1;
    }
    if (!bad && (d->flags & VPCSUM_F_IP) && d->l3_ver != 4) bad = 1;
    if (bad) {
        if (out_word) *out_word = 0;
        if (out_status) *out_status = VPCSUM_S_BAD_DESC;
        return;
    }
    int do_ip = (d->flags & VPCSUM_F_IP) != 0;
    if (do_ip) {
        ipc = orc_ipv4_header_csum(l3, d->l4_off);
        if (mode & VPCSUM_MODE_VERIFY) {
            uint32_t stored = ((uint32_t)l3[10] << 8) | l3[11];
            if (stored == ipc) st |= VPCSUM_S_IP_OK;
        }
    }
    if (do_l4) {
        int fld = orc_l4_field(d->l4_proto);
        if (psonly) {
            uint32_t seg_len = len - d->l4_off;
            uint8_t ph[40];
            if (d->l3_ver == 4) {
                orc_pseudo4(l3, d->l4_proto, seg_len, ph);
                l4c = orc_csum_intermediate(0, ph, 12);
            } else {
                orc_pseudo6(l3, d->l4_proto, seg_len, ph);
                l4c = orc_csum_intermediate(0, ph, 40);
            }
        } else {
            orc_l4_csum(l3, len, d->l4_off, d->l3_ver, d->l4_proto, &l4c);
        }
        if (mode & VPCSUM_MODE_VERIFY) {
            const uint8_t* f = l3 + d->l4_off + fld;
            uint32_t stored = ((uint32_t)f[0] << 8) | f[1];
            if (stored == l4c) st |= VPCSUM_S_L4_OK;
            if (!psonly && d->l4_proto == 17 && stored == 0) st |= VPCSUM_S_UDP_NOCSUM;
        }
    }
    if ((mode & VPCSUM_MODE_WRITE) && arena_w) {
        uint8_t* w = arena_w + off;
        if (do_ip) { w[10] = (uint8_t)(ipc >> 8); w[11] = (uint8_t)ipc; }
        if (do_l4) {
            int fld = orc_l4_field(d->l4_proto);
            w[d->l4_off + fld] = (uint8_t)(l4c >> 8);
            w[d->l4_off + fld + 1] = (uint8_t)l4c;
        }
    }
    if (out_word) *out_word = (ipc & 0xffff) | ((l4c & 0xffff) << 16);
    if (out_status) *out_status = st;
}

void orc_process_batch(const uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* d, uint32_t n,
                       uint32_t mode, uint32_t* out, uint8_t* status, uint8_t* arena_w) {
    for (uint32_t i = 0; i < n; ++i) {
        orc_process_one(arena, arena_len, d + i, mode, out ? out + i : NULL,
                        status ? status + i : NULL, arena_w);
    }
}

/* Multi-threaded CPU baseline: contiguous packet ranges, one pthread each (the reference
 * itself is single-threaded per Switch, Switch.java:170-199; N threads model N switches). */
typedef struct {
    const uint8_t* arena; uint64_t arena_len; const vpcsum_desc_t* d; uint32_t lo, hi;
    uint32_t mode; uint32_t* out; uint8_t* status; uint8_t* arena_w;
} orc_job;

static void* orc_job_run(void* p) {
    orc_job* j = (orc_job*)p;
    for (uint32_t i = j->lo; i < j->hi; ++i)
        orc_process_one(j->arena, j->arena_len, j->d + i, j->mode, j->out ? j->out + i : NULL,
                        j->status ? j->status + i : NULL, j->arena_w);
    return NULL;
}

/* arena_w (MODE_WRITE): the packets of one batch must not overlap (test infrastructure: the
 * threads write their own packets' fields) */
int orc_process_batch_mt_w(const uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* d, uint32_t n,
                           uint32_t mode, uint32_t* out, uint8_t* status, uint8_t* arena_w, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    orc_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].arena = arena; jobs[t].arena_len = arena_len; jobs[t].d = d;
        jobs[t].lo = (uint32_t)((uint64_t)n * t / nthreads);
        jobs[t].hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
        jobs[t].mode = mode; jobs[t].out = out; jobs[t].status = status; jobs[t].arena_w = arena_w;
        if (pthread_create(&th[t], NULL, orc_job_run, &jobs[t]) != 0) return -1;
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}

int orc_process_batch_mt(const uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* d, uint32_t n,
                         uint32_t mode, uint32_t* out, uint8_t* status, int nthreads) {
    return orc_process_batch_mt_w(arena, arena_len, d, n, mode, out, status, NULL, nthreads);
}

/* ---------------------------------------------------------------------------------------- */
/* NAT / TTL rewrite restated as Java does it: setters, then a FULL recompute of the sums they */
/* dirtied (SwitchUtils.applyNat SwitchUtils.java:522-542 -> getRawPacket(0)).               */
/* ---------------------------------------------------------------------------------------- */
/* The setters alone: returns 0 for a refused packet (status set, nothing written), else 1 with the
 * sums they dirtied in *ip_dirty / *l4_dirty (AbstractPacket.checksumSkipped). */
static int orc_nat_apply(uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* d, const vpcsum_nat_t* rw,
                         uint8_t* status, int* ip_dirty_out, int* l4_dirty_out) {
    uint64_t off = d->l3_off;
    int ver = d->l3_ver, proto = d->l4_proto;
    uint32_t len = d->l3_len, l4o = d->l4_off;
    int ok = off <= arena_len && (uint64_t)len <= arena_len - off;
    if (ok && ver == 4) ok = len >= 20 && l4o >= 20 && l4o <= len && !(l4o & 3);
    else if (ok && ver == 6) ok = len >= 40 && l4o >= 40 && l4o <= len;
    else ok = 0;
    if (!ok) {
        if (status) *status = VPCSUM_S_BAD_DESC;
        return 0;
    }
    uint8_t* l3 = arena + off;
    /* IPInputRoute.java:81-88: hop <= 1 is dropped (ICMP time exceeded), never decremented */
    if ((rw->mask & VPCSUM_NAT_DEC_TTL) &&
        ((rw->mask & VPCSUM_NAT_SET_TTL) ? rw->ttl : l3[ver == 4 ? 8 : 7]) <= 1) {
        if (status) *status = VPCSUM_S_BAD_DESC | VPCSUM_S_TTL_EXPIRED;
        return 0;
    }
    int fld = orc_l4_field((uint32_t)proto);
    /* the L4 packet carries a checksum field (TcpPacket / UdpPacket / IcmpPacket) */
    int l4sum = fld >= 0 && !(ver == 4 && proto == 58) && len - l4o >= (uint32_t)fld + 2;
    /* pseudoHeaderChanges: IPv4 dirties TCP / UDP (Ipv4Packet.java:236-240), IPv6 also ICMP /
     * ICMPv6 (Ipv6Packet.java:238-242) */
    int addr_dirty = l4sum && (proto == 6 || proto == 17 || (ver == 6 && (proto == 1 || proto == 58)));
    int ip_dirty = 0, l4_dirty = 0;
    if (ver == 4) {
        if (rw->mask & VPCSUM_NAT_SRC) { memcpy(l3 + 12, rw->src, 4); ip_dirty = 1; l4_dirty |= addr_dirty; } /* setSrc :433-445 */
        if (rw->mask & VPCSUM_NAT_DST) { memcpy(l3 + 16, rw->dst, 4); ip_dirty = 1; l4_dirty |= addr_dirty; } /* setDst :447-458 */
        if (rw->mask & VPCSUM_NAT_SET_TTL) { l3[8] = rw->ttl; ip_dirty = 1; }                     /* setTtl(ttl) :401-407 */
        if (rw->mask & VPCSUM_NAT_DEC_TTL) { l3[8] = (uint8_t)(l3[8] - 1); ip_dirty = 1; }         /* setTtl(ttl-1) */
    } else {
        if (rw->mask & VPCSUM_NAT_SRC) { memcpy(l3 + 8, rw->src, 16); l4_dirty |= addr_dirty; }   /* setSrc :374-384 */
        if (rw->mask & VPCSUM_NAT_DST) { memcpy(l3 + 24, rw->dst, 16); l4_dirty |= addr_dirty; }  /* setDst :386-396 */
        if (rw->mask & VPCSUM_NAT_SET_TTL) l3[7] = rw->ttl;                    /* setHopLimit: nothing dirty */
        if (rw->mask & VPCSUM_NAT_DEC_TTL) l3[7] = (uint8_t)(l3[7] - 1);
    }
    if (l4sum && (proto == 6 || proto == 17)) {   /* TcpPacket / UdpPacket.setSrcPort / setDstPort */
        if (rw->mask & VPCSUM_NAT_SPORT) { memcpy(l3 + l4o, rw->sport, 2); l4_dirty = 1; }
        if (rw->mask & VPCSUM_NAT_DPORT) { memcpy(l3 + l4o + 2, rw->dport, 2); l4_dirty = 1; }
    }
    *ip_dirty_out = ip_dirty;
    *l4_dirty_out = l4_dirty;
    return 1;
}

void orc_nat_java(uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* d, const vpcsum_nat_t* rw,
                  uint8_t* status) {
    int ip_dirty = 0, l4_dirty = 0;
    if (!orc_nat_apply(arena, arena_len, d, rw, status, &ip_dirty, &l4_dirty)) return;
    uint8_t* l3 = arena + d->l3_off;
    uint32_t len = d->l3_len, l4o = d->l4_off;
    int ver = d->l3_ver, proto = d->l4_proto;
    int fld = orc_l4_field((uint32_t)proto);
    /* getRawPacket(0): the dirty sums recomputed in full (AbstractPacket.java:15-22, 58-65) */
    if (ip_dirty) {
        uint32_t c = orc_ipv4_header_csum(l3, l4o);
        l3[10] = (uint8_t)(c >> 8); l3[11] = (uint8_t)c;
    }
    if (l4_dirty) {
        uint32_t c = 0;
        orc_l4_csum(l3, len, l4o, (uint32_t)ver, (uint32_t)proto, &c);
        l3[l4o + fld] = (uint8_t)(c >> 8); l3[l4o + fld + 1] = (uint8_t)c;
    }
    if (status) *status = VPCSUM_S_DONE;
}

/* Java's setters alone, without the recompute: the new bytes in the frame, the stored sums as they
 * were -- a NAT'd frame between SwitchUtils.applyNat (SwitchUtils.java:531-542) and its
 * getRawPacket(0) at egress, the input of the pre-image flush (VPCSUM_F_PRE).  Status as
 * orc_nat_java (S_DONE, or refused: nothing written).  Frames of one batch must not overlap. */
void orc_nat_setters_batch(uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* d, const vpcsum_nat_t* rw,
                           uint32_t n, uint8_t* status) {
    for (uint32_t i = 0; i < n; ++i) {
        int ip_dirty = 0, l4_dirty = 0;
        if (orc_nat_apply(arena, arena_len, d + i, rw + i, status ? status + i : NULL, &ip_dirty, &l4_dirty) && status)
            status[i] = VPCSUM_S_DONE;
    }
}

/* The 16-B IPv4 entry: the same setters (rsv[0] = the SET_TTL value); IPv6 is rejected. */
void orc_nat4_java(uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* d, const vpcsum_nat4_t* rw4,
                   uint8_t* status) {
    if (d->l3_ver != 4) {
        if (status) *status = VPCSUM_S_BAD_DESC;
        return;
    }
    vpcsum_nat_t rw;
    memset(&rw, 0, sizeof(rw));
    memcpy(rw.src, rw4->src, 4);
    memcpy(rw.dst, rw4->dst, 4);
    memcpy(rw.sport, rw4->sport, 2);
    memcpy(rw.dport, rw4->dport, 2);
    rw.mask = rw4->mask;
    rw.ttl = rw4->rsv[0];
    orc_nat_java(arena, arena_len, d, &rw, status);
}

/* Batches of the above, split over threads (the CPU baseline of BASELINE config C5; frames of
 * one batch must not overlap).  fmt 0: vpcsum_nat4_t entries, 1: vpcsum_nat_t. */
typedef struct {
    uint8_t* arena; uint64_t arena_len; const vpcsum_desc_t* d; const void* rw; int fmt;
    uint8_t* status; uint32_t lo, hi;
} orc_nat_job;

static void* orc_nat_job_run(void* p) {
    orc_nat_job* j = (orc_nat_job*)p;
    for (uint32_t i = j->lo; i < j->hi; ++i) {
        if (j->fmt == 0)
            orc_nat4_java(j->arena, j->arena_len, j->d + i, (const vpcsum_nat4_t*)j->rw + i, j->status ? j->status + i : NULL);
        else
            orc_nat_java(j->arena, j->arena_len, j->d + i, (const vpcsum_nat_t*)j->rw + i, j->status ? j->status + i : NULL);
    }
    return NULL;
}

int orc_nat_java_batch(uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* d, const void* rw, int fmt,
                       uint32_t n, uint8_t* status, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    orc_nat_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].arena = arena; jobs[t].arena_len = arena_len; jobs[t].d = d; jobs[t].rw = rw; jobs[t].fmt = fmt;
        jobs[t].status = status;
        jobs[t].lo = (uint32_t)((uint64_t)n * t / nthreads);
        jobs[t].hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
        if (pthread_create(&th[t], NULL, orc_nat_job_run, &jobs[t]) != 0) return -1;
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}

int orc_nat4_java_batch(uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* d, const vpcsum_nat4_t* rw,
                        uint32_t n, uint8_t* status, int nthreads) {
    return orc_nat_java_batch(arena, arena_len, d, rw, 0, n, status, nthreads);
}

/* ---------------------------------------------------------------------------------------- */
/* Synthetic workloads (splitmix64, seed 0x20241020).  Counter-based so any    */
/* packet can be regenerated independently; libvpcsum's GPU generator must match this.      */
/* ---------------------------------------------------------------------------------------- */
static inline uint64_t orc_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
/* splitmix64 output number (ctr+1) of the stream seeded with `seed` */
uint64_t orc_rng(uint64_t seed, uint64_t pkt, uint64_t word) {
    uint64_t ctr = (pkt << 20) | (word & 0xFFFFFull);
    return orc_mix64(seed + (ctr + 1) * 0x9E3779B97F4A7C15ull);
}

/* Packet shape of packet `pkt` for a workload. */
typedef struct { uint32_t ver, proto, l3_len, l4_off; } orc_shape;

static orc_shape orc_shape_of(uint32_t workload, uint64_t seed, uint64_t pkt) {
    orc_shape s = {4, 6, 1500, 20};
    uint64_t r = orc_rng(seed, pkt, 0xFFFFF);
    switch (workload) {
        case VPCSUM_SYNTH_C1_UDP64: s.proto = 17; s.l3_len = 50; break;
        case VPCSUM_SYNTH_C2_TCP1500: break;
        case VPCSUM_SYNTH_C3_MIXED: {
            static const uint32_t lens[3] = {64, 576, 1500};
            static const uint32_t protos[3] = {17, 6, 1};
            s.l3_len = lens[r % 3];
            s.proto = protos[(r / 3) % 3];
            break;
        }
        case VPCSUM_SYNTH_C4_V6JUMBO: s.ver = 6; s.proto = 6; s.l3_len = 9000; s.l4_off = 40; break;
        case VPCSUM_SYNTH_C5_NAT1500: s.proto = (r & 1) ? 17 : 6; break;
        default: { /* FUZZ */
            static const uint32_t protos4[4] = {6, 17, 1, 6};
            static const uint32_t protos6[4] = {6, 17, 58, 17};
            s.ver = (r & 1) ? 6 : 4;
            if (s.ver == 4) {
                s.proto = protos4[(r >> 1) & 3];
                s.l4_off = 20 + 4 * (uint32_t)((r >> 3) % 11);       /* ihl 5..15 */
            } else {
                s.proto = protos6[(r >> 1) & 3];
                s.l4_off = 40;                                       /* no ext headers */
            }
            uint32_t minl4 = (s.proto == 6) ? 20 : 8;
            uint32_t span = 1600;
            if (((r >> 8) & 15) == 0) span = 9000;                   /* occasional jumbo */
            s.l3_len = s.l4_off + minl4 + (uint32_t)((r >> 12) % span);
            if (s.l3_len > 9000) s.l3_len = 9000;
            if (((r >> 40) & 63) == 0) s.l3_len = s.l4_off + minl4;  /* header-only */
            break;
        }
    }
    return s;
}

/* Write packet `pkt` (L3 at frame + l3_pad) and its descriptor.  Bytes outside
 * [l3_pad, l3_pad + l3_len) are left untouched.  Checksum fields are zero. */
void orc_synth_frame(uint8_t* frame, uint32_t l3_pad, uint32_t workload, uint64_t seed, uint64_t pkt,
                     uint64_t frame_off, vpcsum_desc_t* desc) {
    orc_shape s = orc_shape_of(workload, seed, pkt);
    uint8_t* l3 = frame + l3_pad;
    for (uint32_t b = 0; b < s.l3_len; ++b) {
        uint64_t w = orc_rng(seed, pkt, b >> 3);
        l3[b] = (uint8_t)(w >> (8 * (b & 7)));
    }
    if (s.ver == 4) {
        l3[0] = (uint8_t)(0x40 | (s.l4_off / 4));
        l3[1] = 0;
        l3[2] = (uint8_t)(s.l3_len >> 8); l3[3] = (uint8_t)s.l3_len;
        l3[6] = 0x40; l3[7] = 0;
        l3[8] = 64; l3[9] = (uint8_t)s.proto;
        l3[10] = 0; l3[11] = 0;
    } else {
        uint32_t pl = s.l3_len - 40;
        l3[0] = 0x60; l3[1] &= 0x0f;
        l3[4] = (uint8_t)(pl >> 8); l3[5] = (uint8_t)pl;
        l3[6] = (uint8_t)s.proto; l3[7] = 64;
    }
    uint8_t* l4 = l3 + s.l4_off;
    uint32_t l4len = s.l3_len - s.l4_off;
    if (s.proto == 6) {
        l4[12] = 0x50; l4[13] = 0x10; l4[16] = 0; l4[17] = 0; l4[18] = 0; l4[19] = 0;
    } else if (s.proto == 17) {
        l4[4] = (uint8_t)(l4len >> 8); l4[5] = (uint8_t)l4len; l4[6] = 0; l4[7] = 0;
    } else {
        l4[0] = (s.proto == 58) ? 128 : 8; l4[1] = 0; l4[2] = 0; l4[3] = 0;
    }
    if (desc) {
        desc->l3_off = frame_off + l3_pad;
        desc->l3_len = (uint16_t)s.l3_len;
        desc->l4_off = (uint16_t)s.l4_off;
        desc->l3_ver = (uint8_t)s.ver;
        desc->l4_proto = (uint8_t)s.proto;
        desc->flags = (uint8_t)((s.ver == 4 ? VPCSUM_F_IP : 0) | VPCSUM_F_L4);
        desc->rsv = 0;
    }
}

void orc_synth_batch(uint8_t* arena, uint32_t n, uint32_t stride, uint32_t l3_pad, uint32_t workload,
                     uint64_t seed, uint64_t first_index, vpcsum_desc_t* desc) {
    for (uint32_t i = 0; i < n; ++i) {
        orc_synth_frame(arena + (uint64_t)i * stride, l3_pad, workload, seed, first_index + i,
                        (uint64_t)i * stride, desc ? desc + i : NULL);
    }
}

/* The same split over threads (frames are independent). */
typedef struct {
    uint8_t* arena; uint32_t stride, l3_pad, workload; uint64_t seed, first; vpcsum_desc_t* desc; uint32_t lo, hi;
} orc_synth_job;

static void* orc_synth_job_run(void* p) {
    orc_synth_job* j = (orc_synth_job*)p;
    for (uint32_t i = j->lo; i < j->hi; ++i)
        orc_synth_frame(j->arena + (uint64_t)i * j->stride, j->l3_pad, j->workload, j->seed, j->first + i,
                        (uint64_t)i * j->stride, j->desc ? j->desc + i : NULL);
    return NULL;
}

int orc_synth_batch_mt(uint8_t* arena, uint32_t n, uint32_t stride, uint32_t l3_pad, uint32_t workload,
                       uint64_t seed, uint64_t first_index, vpcsum_desc_t* desc, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    orc_synth_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        orc_synth_job j = {arena, stride, l3_pad, workload, seed, first_index, desc,
                           (uint32_t)((uint64_t)n * t / nthreads), (uint32_t)((uint64_t)n * (t + 1) / nthreads)};
        jobs[t] = j;
        if (pthread_create(&th[t], NULL, orc_synth_job_run, &jobs[t]) != 0) return -1;
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}
