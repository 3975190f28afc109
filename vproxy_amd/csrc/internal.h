// Internal launch interface between the C-ABI layer (api.cpp) and the kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include "vpcsum.h"

namespace vpcsum {

// Lanes per packet ("team") for the checksum kernel.  0 = auto.
// mode bits 8..11 carry an explicit log2(team) (tuning / tests); see api.cpp.
hipError_t launch_csum(const uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* desc, uint32_t n,
                       uint32_t* out, uint8_t* status, const uint8_t* flags_override, uint32_t mode,
                       uint8_t* arena_w, int team_log2, int grid_override, hipStream_t stream);

// Low-latency service (k_csum_service): a small persistent grid that polls this host-pinned,
// device-mapped, uncached mailbox instead of being launched per batch.  The host writes the
// batch's descriptors into the service's own pinned buffers, the parameter block when it
// changed, then the command word; the grid writes `done` = seq when the batch is finished.
// The command word shares its 64-B line with the first kSvcInlineDesc descriptors of every
// batch, each tagged with the batch sequence (low byte, in the descriptor's rsv byte): the
// poller reads the whole line in one request, so a flush of up to kSvcInlineDesc frames needs
// no separate descriptor read over PCIe.
constexpr int kSvcInlineDesc = 3;
struct alignas(64) SvcMailbox {
    uint64_t cmd;        // host: seq (bits 0..31, 0 = none yet) | n (32..54) | kSvcHsum | kSvcParse | kSvcFrames | kSvcPre | kSvcPreFmt | kSvcInline |
                         // kSvcStop | kSvcVerify | kSvcParams
    uint64_t rsv0;
    vpcsum_desc_t idesc[kSvcInlineDesc];   // host: descriptors 0..2 of the batch, rsv = (uint8_t)seq
    alignas(64) uint64_t arena;   // line 1, device addresses, read when kSvcParams: arena, then
    uint64_t arena_len, arena_w, desc, out, status, opts, pre;   // opts: kSvcOpt* (tooling); pre: the
                                                                 // service's aux buffer: pre-images (kSvcPre
                                                                 // batches) or parse results (kSvcParse)
    alignas(64) uint32_t done;   // device: last completed batch
    uint32_t pad_;
    uint64_t stamp[7];           // VPCSUM_SVC_STAMPS builds only: s_memrealtime per batch step
};
static_assert(sizeof(vpcsum_desc_t) * kSvcInlineDesc + 16 == 64, "SvcMailbox command line: one 64-B line");
static_assert(offsetof(SvcMailbox, arena) == 64 && offsetof(SvcMailbox, done) == 128, "SvcMailbox line layout");
constexpr uint64_t kSvcInline = 1ull << 60, kSvcStop = 1ull << 61, kSvcVerify = 1ull << 62, kSvcParams = 1ull << 63;
constexpr uint64_t kSvcOptClampLoads = 1;   // A/B: the frame loads of a batch clamp instead of predicate
constexpr uint64_t kSvcOptReleaseDone = 2;  // A/B: release semantics on the completion count and `done`
// a batch with VPCSUM_F_PRE frames: their pre-images are in the buffer `pre` names, 16-B
// vpcsum_pre4_t entries, or 48-B vpcsum_pre_t ones with kSvcPreFmt
constexpr uint64_t kSvcPre = 1ull << 58, kSvcPreFmt = 1ull << 59;
// a batch of raw egress frames (vpcsum_ctx_egress_frames): the descriptor buffer (and the inline
// descriptors) hold SvcFrameRec records, each frame is parsed on the GPU before it is summed
constexpr uint64_t kSvcFrames = 1ull << 57;
// with kSvcFrames: parse only (vpcsum_ctx_parse_frames) -- descriptors at the aux buffer's start,
// tuples after kSvcBatchMax descriptors, status bytes; no sums
constexpr uint64_t kSvcParse = 1ull << 56;
// with kSvcFrames | kSvcVerify: each frame's ingress header sum (vpcsum_hsum_t) to the aux buffer
// (vpcsum_ctx_verify_frames_hsum)
constexpr uint64_t kSvcHsum = 1ull << 55;
struct SvcFrameRec {
    uint64_t off;    // the frame's offset in the arena
    uint32_t len;    // its length
    uint8_t flags;   // the VPCSUM_F_* sums it needs
    uint8_t pad[2];
    uint8_t tag;     // the inline records' batch tag (vpcsum_desc_t's rsv byte)
};
static_assert(sizeof(SvcFrameRec) == sizeof(vpcsum_desc_t), "a frame record takes a descriptor's slot");
constexpr uint32_t kSvcMaxPkts = (1u << 23) - 1;   // the command's n field (bits 32..54)
constexpr uint32_t kSvcBatchMax = 512;              // largest batch the host hands to the service (api.cpp)
constexpr int kServiceGrid = 32;   // workgroups: 4 waves each, one packet per wave and round (default)
hipError_t launch_service(SvcMailbox* d_mb, uint32_t* d_ctr, uint32_t seen, uint64_t idle_ticks, hipStream_t stream,
                          uint32_t grid = kServiceGrid, uint32_t poll = 0);
// Tooling: a resident grid of `wgs` workgroups x `threads` that only sleeps (s_sleep) for `ticks`
// (100 MHz) -- no memory traffic: the control for "a resident kernel on another queue" A/Bs.
hipError_t launch_spin_probe(uint32_t wgs, uint32_t threads, uint64_t ticks, hipStream_t stream);

// NAT / TTL rewrites (nat.hip).  fmt 0: rw is vpcsum_nat4_t[n], fmt 1: vpcsum_nat_t[n].  With
// VPCSUM_NAT_STRICT_JAVA the kernel only rewrites and stores Java's dirty flags in flags_out.
hipError_t launch_nat(uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* desc, const void* rw, int fmt,
                      uint32_t n, uint8_t* status, uint8_t* flags_out, uint32_t nat_mode, hipStream_t stream);
// NAT's memory operations without the rewrite (tooling: the C5 pattern ceiling)
hipError_t launch_nat_probe(uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* desc, const void* rw, int fmt,
                            uint32_t n, hipStream_t stream);
// pre-image egress sums (K6, VPCSUM_F_PRE descriptors only); fmt 0: vpcsum_pre4_t, 1: vpcsum_pre_t;
// mode: VPCSUM_MODE_WRITE plus the tuning bits of vpcsum_pre_async
hipError_t launch_pre(uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* desc, const void* pre, int fmt, uint32_t n,
                      uint32_t* out, uint8_t* status, uint32_t mode, hipStream_t stream);
// strict mode, after the recompute: S_TTL_EXPIRED on the packets refused for their TTL
hipError_t launch_nat_ttl_status(const uint8_t* arena, uint64_t arena_len, const vpcsum_desc_t* desc, const void* rw,
                                 int fmt, uint32_t n, uint8_t* status, hipStream_t stream);

hipError_t launch_parse_ether(const uint8_t* arena, uint64_t arena_len, const uint64_t* frame_off,
                              const uint32_t* frame_len, uint32_t n, uint8_t flags, vpcsum_desc_t* desc,
                              uint8_t* status, vpcsum_tuple_t* tuples, hipStream_t stream,
                              const uint8_t* frame_flags = nullptr, vpcsum_hsum_t* hsum = nullptr);

hipError_t launch_read_probe(const uint8_t* buf, uint64_t bytes, uint32_t* sink, uint32_t grid, hipStream_t stream);
hipError_t launch_pattern_probe(const uint8_t* arena, uint64_t arena_len, const void* desc, uint32_t n, uint32_t* sink,
                                uint32_t grid, hipStream_t stream);

hipError_t launch_synth(uint8_t* arena, uint64_t arena_len, uint32_t n, uint32_t stride, uint32_t l3_pad,
                        uint32_t workload, uint64_t seed, uint64_t first_index, vpcsum_desc_t* desc,
                        hipStream_t stream);

int num_cus(int device);

}  // namespace vpcsum
