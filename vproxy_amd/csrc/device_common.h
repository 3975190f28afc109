// device_common.h -- device helpers shared by the kernels of libvpcsum (kernels.hip, nat.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "vpcsum.h"

namespace vpcsum {

// Bytes of the dword at relative byte position d that fall inside [lo, hi).
__device__ __forceinline__ uint32_t bmask(int d, int lo, int hi) {
    int s = min(max(lo - d, 0), 4);
    int e = min(max(hi - d, 0), 4);
    uint32_t me = e >= 4 ? 0xffffffffu : ((1u << (e << 3)) - 1u);
    uint32_t ms = s >= 4 ? 0xffffffffu : ((1u << (s << 3)) - 1u);
    return me & ~ms;
}

// Bytes of the dword at relative position d that lie before `hi`.
__device__ __forceinline__ uint32_t tailmask(int d, int hi) {
    const int e = min(max(hi - d, 0), 4);
    return e >= 4 ? 0xffffffffu : ((1u << (e << 3)) - 1u);
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// Packet bytes are read exactly once: non-temporal loads keep them from displacing the
// descriptors and the next packets' lines in L2 / MALL (measured +10% on this pattern,
// tools/bwlab.hip).
// (address space 1 so hipcc emits global_load_dwordx4, not flat_load: flat loads count on
// lgkmcnt too and force vmcnt(0)+lgkmcnt(0) waits that serialise the U loads in flight.)
typedef __attribute__((address_space(1))) const u32x4_t gu32x4_t;
template <bool NT>
__device__ __forceinline__ uint4 ld_stream(const uint4* q) {
    const u32x4_t v = NT ? __builtin_nontemporal_load((gu32x4_t*)q) : *(gu32x4_t*)q;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// End-around-carry fold of a 64-bit sum of LE words to 16 bits; 0 only for 0.
__device__ __forceinline__ uint32_t fold64(uint64_t x) {
    uint64_t t = (x & 0xffffffffull) + (x >> 32);
    t = (t & 0xffff) + (t >> 16);
    t = (t & 0xffff) + (t >> 16);
    t = (t & 0xffff) + (t >> 16);
    return (uint32_t)t;
}
__device__ __forceinline__ uint32_t fold32(uint32_t x) {
    x = (x & 0xffff) + (x >> 16);
    x = (x & 0xffff) + (x >> 16);
    return x;
}
__device__ __forceinline__ uint32_t bswap16(uint32_t v) { return ((v & 0xff) << 8) | (v >> 8); }
// A sum taken over a byte range that starts at an even absolute address is byte-swapped
// relative to the big-endian word grid of that range (RFC 1071 byte-order independence).
__device__ __forceinline__ uint32_t orient(uint32_t v, int start) { return (start & 1) ? v : bswap16(v); }

__device__ __forceinline__ int l4_field(int proto) {
    return proto == 6 ? 16 : proto == 17 ? 6 : (proto == 1 || proto == 58) ? 2 : -1;
}

// Internal flag set by the NAT kernel on descriptors it rejected (strict-Java mode hands its
// per-packet dirty flags to the checksum kernel through flags_override).
constexpr int kFlagRejected = 0x80;

// Buffer addressing: the packet bytes come in through buffer loads on ONE wave-uniform descriptor
// spanning the arena; an offset outside the descriptor's range returns zeros without touching
// memory.  Needs a 16-B aligned arena < 4 GiB.
constexpr uint32_t kOutOfRange = 0xFFFFFF00u;
constexpr uint64_t kMaxBufArena = 0xFFFF0000ull;
// The range check zeroes any dword that reaches past num_records, so the descriptor covers the
// arena rounded up to 16 B: the 16-B aligned block holding the last arena byte is readable
// (it never crosses a page), and bytes past the arena end are masked by the packet bounds.
__device__ __forceinline__ uint32_t buf_records(uint64_t arena_len) {
    return (uint32_t)((arena_len + 15) & ~15ull);
}

__device__ __forceinline__ uint32_t ld16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
__device__ __forceinline__ void st16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

// Big-endian 16-bit store of a checksum field into a frame, non-temporal (written once; a plain
// store of a partial line costs far more beside the nt read stream -- measured 2x on an
// earlier team-per-packet kernel).
__device__ __forceinline__ void st_be16_nt(uint8_t* p, uint32_t v) {
    typedef __attribute__((address_space(1))) uint16_t g16;
    typedef __attribute__((address_space(1))) uint8_t g8;
    if (((uintptr_t)p & 1) == 0) {
        __builtin_nontemporal_store((uint16_t)(((v & 0xff) << 8) | ((v >> 8) & 0xff)), (g16*)p);
    } else {
        __builtin_nontemporal_store((uint8_t)(v >> 8), (g8*)p);
        __builtin_nontemporal_store((uint8_t)v, (g8*)(p + 1));
    }
}

// The same with a plain store (written through L2: two fields of one line leave in one write-back).
__device__ __forceinline__ void st_be16(uint8_t* p, uint32_t v) {
    typedef __attribute__((address_space(1))) uint16_t g16;
    typedef __attribute__((address_space(1))) uint8_t g8;
    if (((uintptr_t)p & 1) == 0) {
        *(g16*)p = (uint16_t)(((v & 0xff) << 8) | ((v >> 8) & 0xff));
    } else {
        *(g8*)p = (uint8_t)(v >> 8);
        *(g8*)(p + 1) = (uint8_t)v;
    }
}

// VPCSUM_F_PRE descriptors belong to the pre-image kernel (nat.hip k_pre): the checksum kernels
// read none of their bytes and write nothing into their frames (flags 0: out 0, S_DONE).
__device__ __forceinline__ int csum_flags(int fl) { return (fl & VPCSUM_F_PRE) ? 0 : fl; }

}  // namespace vpcsum
