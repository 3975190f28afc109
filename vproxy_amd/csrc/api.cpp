// api.cpp -- the C-ABI of libvpcsum.so (declared in include/vpcsum.h).
//
// Device-resident entry points validate arguments and launch the kernels of kernels.hip on
// the caller's stream.  The context API is what the Java side drives (io.vproxy.vpcsum.VPCsum,
// java/io/vproxy/vpcsum/VPCsum.java): host arena + descriptors in, checksums out, with the
// batch flushed once per Iface.completeTx (core/.../vswitch/iface/XDPIface.java:227-243).
// Errors: plain functions return <0 and set a thread-local message; PNI functions store the
// exception in env->ex exactly as the PNI runtime expects (base/src/main/c-generated/pni.h:74-82).
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "internal.h"
#include "vpcsum.h"

namespace vpcsum {

// The thread's last error message: a fixed buffer, so that reporting a failure never allocates
// (an out-of-memory failure must still leave its message)
static thread_local char g_err[1024];

static int fail(const char* fmt, ...) {
    char buf[sizeof(g_err)];   // the arguments may point into g_err itself
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    memcpy(g_err, buf, sizeof(g_err));
    return -1;
}

static int hipfail(hipError_t e, const char* what) {
    return fail("%s: %s (%d)", what, hipGetErrorString(e), (int)e);
}

// Every extern "C" entry point catches what the C++ runtime may throw (std::bad_alloc from the
// bookkeeping containers, ...): an exception must never unwind into a C or JVM caller.  The entry
// returns -1 with the message set (PNI: the exception stored in env->ex).
#define VPC_CATCH(what)                                                                 \
    catch (const std::bad_alloc&) { return fail("%s: out of host memory", what); }     \
    catch (...) { return fail("%s: internal error (C++ exception)", what); }
#define VPC_CATCH_PNI(what)                                                             \
    catch (const std::bad_alloc&) {                                                     \
        fail("%s: out of host memory", what);                                           \
        return pni_throw(env, "java.lang.OutOfMemoryError");                            \
    }                                                                                   \
    catch (...) {                                                                       \
        fail("%s: internal error (C++ exception)", what);                               \
        return pni_throw(env, "java.io.IOException");                                   \
    }

#define VPC_CHECK(expr, what)                         \
    do {                                              \
        hipError_t e__ = (expr);                      \
        if (e__ != hipSuccess) return hipfail(e__, what); \
    } while (0)

// Makes `device` current for one entry point and gives the caller its own current device back on
// every exit path: a torch or Java caller working on another device never sees it change.
struct DeviceScope {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceScope(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != device) err = hipSetDevice(device);
    }
    ~DeviceScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};

#define VPC_ON_DEVICE(dev)                                                      \
    DeviceScope dscope__(dev);                                                  \
    if (dscope__.err != hipSuccess) return hipfail(dscope__.err, "hipSetDevice")

int num_cus(int device) {
    static std::mutex mu;
    static std::vector<int> cache;
    std::lock_guard<std::mutex> lk(mu);
    if (device < 0) device = 0;
    if ((int)cache.size() <= device) cache.resize(device + 1, 0);
    if (cache[device] == 0) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || v <= 0) v = 256;
        cache[device] = v;
    }
    return cache[device];
}

// Per-slot staging of one in-flight batch of a context.
struct Slot {
    uint8_t* d_arena = nullptr;
    vpcsum_desc_t* d_desc = nullptr;
    uint32_t* d_out = nullptr;
    uint8_t* d_status = nullptr;
    vpcsum_desc_t* h_desc = nullptr;   // pinned staging
    uint32_t* h_out = nullptr;         // pinned staging
    uint8_t* h_status = nullptr;       // pinned staging
    uint8_t* h_arena = nullptr;        // pinned staging for unregistered arenas
    vpcsum_desc_t* dh_desc = nullptr;  // device-side addresses of the pinned staging
    uint32_t* dh_out = nullptr;
    uint8_t* dh_status = nullptr;
    uint64_t* h_foff = nullptr;        // pinned staging of received-frame offsets / lengths
    uint32_t* h_flen = nullptr;
    uint64_t* dh_foff = nullptr;
    uint32_t* dh_flen = nullptr;
    vpcsum_nat_t* h_rw = nullptr;      // NAT rewrite tables: pinned staging (mapped) and device copy,
    vpcsum_nat_t* dh_rw = nullptr;     // allocated with the context's first NAT batch
    vpcsum_nat_t* d_rw = nullptr;
    vpcsum_tuple_t* h_tu = nullptr;    // flow tuples of a parse batch: pinned (mapped), allocated
    vpcsum_tuple_t* dh_tu = nullptr;   // with the context's first parse batch
    vpcsum_hsum_t* h_hs = nullptr;     // ingress header sums of a verify batch: pinned (mapped),
    vpcsum_hsum_t* dh_hs = nullptr;    // allocated with the context's first such batch
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    int kind = 0;                      // current batch: 0 checksums, 1 NAT rewrite, 2 parse
    bool zero_copy = false;            // current batch ran on the host frames in place
    uint32_t svc_seq = 0;              // != 0: the batch went to the low-latency service
    // the batch currently owned by this slot
    uint64_t ticket = 0;
    bool busy = false;
    uint32_t n = 0;
    uint32_t mode = 0;
    uint8_t* user_arena = nullptr;
    const vpcsum_desc_t* user_desc = nullptr;
    uint32_t* user_out = nullptr;
    uint8_t* user_status = nullptr;
    vpcsum_desc_t* user_desc_out = nullptr;   // parse batch: where descriptors and tuples go
    vpcsum_tuple_t* user_tuples = nullptr;
    vpcsum_hsum_t* user_hsum = nullptr;       // verify batch with header sums: where they go
};

}  // namespace vpcsum

struct Registered {
    uint8_t* host;
    uint64_t len;
    uint8_t* dev;    // device-side address of the page-locked mapping (zero-copy access)
    uint8_t* key;    // the process-wide page-lock this entry holds a reference on (hostlock_acquire);
                     // nullptr: a mapping of its group's lock (the group holds the reference)
};

// ------------------------------------------------------------------------------------------
// Process-wide registry of the host ranges libvpcsum page-locks.  HIP keys a host registration by
// its start address (tools/reg_probe.py, profiles/r06c_reg_probe.jsonl): a second hipHostRegister
// of a registered start -- same length or longer -- returns success without mapping anything new,
// the first hipHostUnregister then drops the registration for both holders, and the second fails.
// Two contexts (or a context and a group) registering one umem therefore left the survivor with a
// mapping HIP had torn down, and its zero-copy kernels -- or a later pageable copy HIP resolves
// through the orphaned registration -- reading unmapped memory (DESIGN_HISTORY.md "Round 6: the
// intermittent fault").  So every page-lock goes through here: a range inside a live lock shares
// it (reference counted), a range that partially overlaps one or that HIP already holds as
// page-locked memory of another owner is refused, and hipHostUnregister runs once, with the last
// reference.  Locks are mapped on every device (portable), so a share across devices is valid.
// ------------------------------------------------------------------------------------------
struct HostLock {
    uint8_t* host;
    uint64_t len;
    uint32_t refs;
};
static std::mutex g_lock_mu;
static std::vector<HostLock> g_locks;

static bool hip_holds_pinned(const uint8_t* p) {
    hipPointerAttribute_t a;
    const bool pinned = hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost;
    (void)hipGetLastError();   // an unknown (pageable) pointer leaves an error behind
    return pinned;
}

using vpcsum::fail;
using vpcsum::hipfail;

// A reference on the page-lock of [p, p+len) (see HostLock): *key = the lock's start, for
// hostlock_release.  Caller is on the device the mapping is wanted for.
static int hostlock_acquire(uint8_t* p, uint64_t len, uint8_t** key, const char* what) {
    std::lock_guard<std::mutex> lk(g_lock_mu);
    for (auto& h : g_locks) {
        if (p >= h.host && p + len <= h.host + h.len) {   // inside a live lock: share it
            ++h.refs;
            *key = h.host;
            return 0;
        }
        if (p < h.host + h.len && h.host < p + len)
            return fail("%s: [%p, +%llu) overlaps the arena [%p, +%llu) page-locked earlier: register one range "
                        "that covers both",
                        what, (void*)p, (unsigned long long)len, (void*)h.host, (unsigned long long)h.len);
    }
    if (hip_holds_pinned(p) || hip_holds_pinned(p + len - 1))
        return fail("%s: %p is already page-locked outside libvpcsum (hipHostMalloc / hipHostRegister): its owner "
                    "controls that lock's lifetime; pass the memory unregistered (staged) instead",
                    what, (void*)p);
    g_locks.reserve(g_locks.size() + 1);   // may throw: before anything is pinned
    VPC_CHECK(hipHostRegister(p, len, hipHostRegisterMapped | hipHostRegisterPortable), "hipHostRegister");
    g_locks.push_back({p, len, 1});
    *key = p;
    return 0;
}

// Drop one reference; the last one unpins (a failure is reported: the caller must not free the
// memory as if it were unpinned).
static int hostlock_release(uint8_t* key, const char* what) {
    std::lock_guard<std::mutex> lk(g_lock_mu);
    for (size_t i = 0; i < g_locks.size(); ++i) {
        if (g_locks[i].host != key) continue;
        if (--g_locks[i].refs) return 0;
        g_locks.erase(g_locks.begin() + i);
        const hipError_t e = hipHostUnregister(key);
        if (e != hipSuccess) return fail("%s: hipHostUnregister(%p): %s", what, (void*)key, hipGetErrorString(e));
        return 0;
    }
    return fail("%s: %p holds no page-lock of libvpcsum", what, (void*)key);
}

// Zero-copy batches (frames read over PCIe) of at most this many packets run one wave per packet.
constexpr uint32_t kZeroCopyWaveTeams = 4096;
// kSvcBatchMax (internal.h): the largest batch handed to the low-latency service (128 waves, one
// packet each per round); larger ones are launched with a grid of their size, which is faster from
// ~1000 packets on (tools/flush_latency.cpp: 1024 packets 55 us launched vs 58 us through the
// service, profiles/r05m_flush_latency.json).

// The service's aux buffer: kSvcBatchMax pre-images of 48 B, or kSvcBatchMax descriptors followed
// by kSvcBatchMax tuples (a parse batch, kSvcParse)
constexpr size_t kSvcAuxBytes = (size_t)vpcsum::kSvcBatchMax * (sizeof(vpcsum_desc_t) + sizeof(vpcsum_tuple_t));
static_assert(kSvcAuxBytes >= (size_t)vpcsum::kSvcBatchMax * sizeof(vpcsum_pre_t), "aux buffer holds a batch of pre-images");

// Low-latency service of a context (kernels.hip k_csum_service).
struct Service {
    vpcsum::SvcMailbox* mb = nullptr;    // host-pinned, coherent (uncached on the GPU), mapped
    vpcsum::SvcMailbox* dmb = nullptr;   // its device address
    uint32_t* ctr = nullptr;             // device: workgroups finished with the current batch,
                                         // then (8-B aligned, ctr + 2) the command relay
    hipStream_t stream = nullptr;
    // the service's own descriptor / result buffers (pinned, coherent, mapped) and their device
    // addresses: the same for every batch, so the parameter block rarely changes
    vpcsum_desc_t* h_desc = nullptr;
    uint32_t* h_out = nullptr;
    uint8_t* h_status = nullptr;
    vpcsum_desc_t* dh_desc = nullptr;
    uint32_t* dh_out = nullptr;
    uint8_t* dh_status = nullptr;
    void* h_pre = nullptr;               // the aux buffer (kSvcAuxBytes): pre-images of a batch with F_PRE
                                         // frames, or a parse batch's descriptors and tuples
    void* dh_pre = nullptr;
    uint64_t par[3] = {0, 0, 0};         // arena, arena_len, arena_w last published
    bool par_valid = false;
    uint32_t posted = 0;                 // last batch published (seq)
    uint64_t idle_ticks = 0;             // 100 MHz ticks
    uint32_t grid = vpcsum::kServiceGrid;   // workgroups (VPCSUM_SVC_GRID: A/B tooling)
    uint32_t poll = 1;                      // relay poll mode: relaxed loads (VPCSUM_SVC_POLL: A/B tooling)
    bool quiesce = false;                   // stop an idle grid before launched batches (VPCSUM_SVC_QUIESCE)
    bool on = false;
    std::chrono::steady_clock::time_point last_post;   // the last batch posted (svc_quiesce)
    bool inline_desc = true;             // descriptors of <= kSvcInlineDesc frames ride in the command line
                                         // (VPCSUM_SVC_INLINE=0 turns it off: A/B tooling)
#ifdef VPCSUM_SVC_STAMPS
    std::chrono::steady_clock::time_point t_post;
    uint32_t t_n = 0;
#endif
};

struct vpcsum_ctx {
    int device = 0;
    Service svc;
    uint64_t svc_batches = 0;    // batches run by the service (lifetime of the context)
    uint64_t svc_launches = 0;   // service grids launched (first start, idle restarts, re-runs)
    uint64_t max_arena = 0;
    uint32_t max_pkts = 0;
    vpcsum::Slot slots[2];
    uint64_t next_ticket = 1;
    std::vector<Registered> registered;
    std::mutex mu;
};

using namespace vpcsum;

extern "C" {

int vpcsum_abi_version(void) { return VPCSUM_ABI_VERSION; }

const char* vpcsum_last_error(void) { return g_err; }

int vpcsum_device_count(int* out_n) {
    try {
        if (!out_n) return fail("vpcsum_device_count: out_n is NULL");
        int n = 0;
        VPC_CHECK(hipGetDeviceCount(&n), "hipGetDeviceCount");
        *out_n = n;
        return 0;
    } VPC_CATCH("vpcsum_device_count")
}

int vpcsum_set_device(int device) {
    try {
        VPC_CHECK(hipSetDevice(device), "hipSetDevice");
        return 0;
    } VPC_CATCH("vpcsum_set_device")
}

// kernel variant id: bits 8..12 low, bits 24..26 high (0..255; 0 = default)
static int team_from_mode(uint32_t mode) { return (int)(((mode >> 8) & 0x1f) | (((mode >> 24) & 0x7) << 5)); }

int vpcsum_compute_async(const uint8_t* d_arena, uint64_t arena_len, const vpcsum_desc_t* d_desc, uint32_t n,
                         uint32_t* d_out, uint8_t* d_status, uint32_t mode, void* stream) {
    try {
        if (n == 0) return 0;
        if (!d_arena || !d_desc) return fail("vpcsum_compute_async: NULL arena or descriptors");
        // tuning hints (not part of the stable ABI): bits 8..12 + 24..26 kernel variant, bit 13
        // plain (temporal) loads, bit 14 no sampled low-concurrency grid, bits 16..23 workgroups
        // per CU.
        if (mode & ~(0x07ff7fffu | VPCSUM_MODE_VERIFY | VPCSUM_MODE_WRITE)) return fail("vpcsum_compute_async: bad mode 0x%x", mode);
        uint8_t* w = (mode & VPCSUM_MODE_WRITE) ? const_cast<uint8_t*>(d_arena) : nullptr;
        int grid = 0;
        if ((mode >> 16) & 0xff) {
            int dev = 0;
            VPC_CHECK(hipGetDevice(&dev), "hipGetDevice");
            grid = num_cus(dev) * (int)((mode >> 16) & 0xff);
        }
        VPC_CHECK(launch_csum(d_arena, arena_len, d_desc, n, d_out, d_status, nullptr, mode, w, team_from_mode(mode), grid,
                              (hipStream_t)stream),
                  "vpcsum_compute_async launch");
        return 0;
    } VPC_CATCH("vpcsum_compute_async")
}

// NAT on device memory: the rewrite kernel, then (strict Java) the full recompute of the sums it
// dirtied, written in place -- Java's getRawPacket(0) after the setters.
}  // extern "C"

// Two batches in flight on the device API (vpcsum.h vpcsum_pipe_*): launches alternate between two
// streams of the pipe's own, forked from the caller's stream at vpcsum_pipe_begin and joined back
// into it at vpcsum_pipe_join, so that one launch's ramp-up and drain overlap its neighbour's.
struct vpcsum_pipe {
    int device = 0;
    hipStream_t caller = nullptr;
    hipStream_t s[2] = {nullptr, nullptr};
    hipEvent_t fork = nullptr;
    hipEvent_t done[2] = {nullptr, nullptr};
    uint32_t next = 0;
};

static void pipe_free(vpcsum_pipe* p) {
    for (int i = 0; i < 2; ++i) {
        if (p->s[i]) {
            (void)hipStreamSynchronize(p->s[i]);
            (void)hipStreamDestroy(p->s[i]);
        }
        if (p->done[i]) (void)hipEventDestroy(p->done[i]);
    }
    if (p->fork) (void)hipEventDestroy(p->fork);
    delete p;
}

extern "C" {

int vpcsum_pipe_create(void* stream, vpcsum_pipe_t** out) {
    try {
        if (!out) return fail("vpcsum_pipe_create: out is NULL");
        vpcsum_pipe* p = new vpcsum_pipe();
        p->caller = (hipStream_t)stream;
        hipError_t e = hipGetDevice(&p->device);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->s[0], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->s[1], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&p->fork, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&p->done[0], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&p->done[1], hipEventDisableTiming);
        if (e != hipSuccess) {
            pipe_free(p);
            return hipfail(e, "vpcsum_pipe_create");
        }
        *out = p;
        return 0;
    } VPC_CATCH("vpcsum_pipe_create")
}

int vpcsum_pipe_begin(vpcsum_pipe_t* p) {
    try {
        if (!p) return fail("vpcsum_pipe_begin: NULL pipe");
        VPC_ON_DEVICE(p->device);
        VPC_CHECK(hipEventRecord(p->fork, p->caller), "vpcsum_pipe_begin: hipEventRecord");
        for (int i = 0; i < 2; ++i) VPC_CHECK(hipStreamWaitEvent(p->s[i], p->fork, 0), "vpcsum_pipe_begin: hipStreamWaitEvent");
        return 0;
    } VPC_CATCH("vpcsum_pipe_begin")
}

int vpcsum_pipe_compute_async(vpcsum_pipe_t* p, const uint8_t* d_arena, uint64_t arena_len, const vpcsum_desc_t* d_desc,
                              uint32_t n, uint32_t* d_out, uint8_t* d_status, uint32_t mode) {
    try {
        if (!p) return fail("vpcsum_pipe_compute_async: NULL pipe");
        VPC_ON_DEVICE(p->device);
        const int rc = vpcsum_compute_async(d_arena, arena_len, d_desc, n, d_out, d_status, mode, p->s[p->next & 1]);
        if (rc == 0) ++p->next;
        return rc;
    } VPC_CATCH("vpcsum_pipe_compute_async")
}

int vpcsum_pipe_join(vpcsum_pipe_t* p) {
    try {
        if (!p) return fail("vpcsum_pipe_join: NULL pipe");
        VPC_ON_DEVICE(p->device);
        for (int i = 0; i < 2; ++i) {
            VPC_CHECK(hipEventRecord(p->done[i], p->s[i]), "vpcsum_pipe_join: hipEventRecord");
            VPC_CHECK(hipStreamWaitEvent(p->caller, p->done[i], 0), "vpcsum_pipe_join: hipStreamWaitEvent");
        }
        return 0;
    } VPC_CATCH("vpcsum_pipe_join")
}

int vpcsum_pipe_destroy(vpcsum_pipe_t* p) {
    try {
        if (!p) return 0;
        DeviceScope on_dev(p->device);
        pipe_free(p);
        return 0;
    } VPC_CATCH("vpcsum_pipe_destroy")
}

static int nat_run(uint8_t* d_arena, uint64_t arena_len, const vpcsum_desc_t* d_desc, const void* d_rw, int fmt,
                   uint32_t n, uint8_t* d_status, uint32_t nat_mode, hipStream_t s) {
    if (nat_mode & VPCSUM_NAT_STRICT_JAVA) {
        // pass 1: rewrite fields, record which sums went dirty (Java's checksumSkipped())
        VPC_CHECK(launch_nat(d_arena, arena_len, d_desc, d_rw, fmt, n, nullptr, d_status, nat_mode, s), "nat launch");
        // pass 2: full recompute of the dirty sums, written in place (getRawPacket(0))
        VPC_CHECK(launch_csum(d_arena, arena_len, d_desc, n, nullptr, d_status, d_status, VPCSUM_MODE_WRITE, d_arena,
                              0, 0, s),
                  "nat recompute launch");
        // pass 3: the TTL-expired packets (refused, untouched) get S_TTL_EXPIRED next to S_BAD_DESC
        VPC_CHECK(launch_nat_ttl_status(d_arena, arena_len, d_desc, d_rw, fmt, n, d_status, s), "nat ttl status launch");
        return 0;
    }
    VPC_CHECK(launch_nat(d_arena, arena_len, d_desc, d_rw, fmt, n, d_status, nullptr, nat_mode, s), "nat launch");
    return 0;
}

static int nat_async(const char* what, uint8_t* d_arena, uint64_t arena_len, const vpcsum_desc_t* d_desc,
                     const void* d_rw, int fmt, uint32_t n, uint8_t* d_status, uint32_t nat_mode, void* stream) {
    if (n == 0) return 0;
    if (!d_arena || !d_desc || !d_rw) return fail("%s: NULL arena, descriptors or rewrite table", what);
    // tuning hints (not part of the stable ABI; nat.hip, above nat_chunks_sel): bit 8 byte-access
    // kernel, bits 12..14 packets per lane of the wide kernel (the quad kernel clamps 4 to 2), bits
    // 16..17 window chunks, bits 18..22 workgroups per CU, bit 23 the lane layout of the wide kernel
    // instead of quads, bits 24..25 the quad kernel's forced occupancy (6 / 8 waves: may spill)
    if (nat_mode & ~(VPCSUM_NAT_STRICT_JAVA | 0x100u | 0x7000u | 0x3ff0000u)) return fail("%s: bad nat_mode 0x%x", what, nat_mode);
    if ((nat_mode & VPCSUM_NAT_STRICT_JAVA) && !d_status) return fail("%s: strict-java mode needs a status buffer", what);
    if ((nat_mode & VPCSUM_NAT_STRICT_JAVA) && fmt == 2) return fail("%s: records take VPCSUM_NAT_RFC1624 only", what);
    return nat_run(d_arena, arena_len, d_desc, d_rw, fmt, n, d_status, nat_mode, (hipStream_t)stream);
}

int vpcsum_nat4_pattern_probe_async(uint8_t* d_arena, uint64_t arena_len, const vpcsum_desc_t* d_desc,
                                    const vpcsum_nat4_t* d_rw, uint32_t n, void* stream) {
    try {
        if (n == 0) return 0;
        if (!d_arena || !d_desc || !d_rw) return fail("vpcsum_nat4_pattern_probe_async: NULL argument");
        VPC_CHECK(launch_nat_probe(d_arena, arena_len, d_desc, d_rw, 0, n, (hipStream_t)stream),
                  "vpcsum_nat4_pattern_probe_async launch");
        return 0;
    } VPC_CATCH("vpcsum_nat4_pattern_probe_async")
}

int vpcsum_nat4_async(uint8_t* d_arena, uint64_t arena_len, const vpcsum_desc_t* d_desc, const vpcsum_nat4_t* d_rw,
                      uint32_t n, uint8_t* d_status, uint32_t nat_mode, void* stream) {
    try {
        return nat_async("vpcsum_nat4_async", d_arena, arena_len, d_desc, d_rw, 0, n, d_status, nat_mode, stream);
    } VPC_CATCH("vpcsum_nat4_async")
}

int vpcsum_nat4r_async(uint8_t* d_arena, uint64_t arena_len, const vpcsum_nat4_rec_t* d_rec, uint32_t n,
                       uint8_t* d_status, uint32_t nat_mode, void* stream) {
    try {
        return nat_async("vpcsum_nat4r_async", d_arena, arena_len, (const vpcsum_desc_t*)d_rec, d_rec, 2, n, d_status,
                         nat_mode, stream);
    } VPC_CATCH("vpcsum_nat4r_async")
}

int vpcsum_nat4r_pattern_probe_async(uint8_t* d_arena, uint64_t arena_len, const vpcsum_nat4_rec_t* d_rec,
                                     uint32_t n, void* stream) {
    try {
        if (n == 0) return 0;
        if (!d_arena || !d_rec) return fail("vpcsum_nat4r_pattern_probe_async: NULL argument");
        VPC_CHECK(launch_nat_probe(d_arena, arena_len, (const vpcsum_desc_t*)d_rec, d_rec, 2, n, (hipStream_t)stream),
                  "vpcsum_nat4r_pattern_probe_async launch");
        return 0;
    } VPC_CATCH("vpcsum_nat4r_pattern_probe_async")
}

int vpcsum_nat_async(uint8_t* d_arena, uint64_t arena_len, const vpcsum_desc_t* d_desc, const vpcsum_nat_t* d_rw,
                     uint32_t n, uint8_t* d_status, uint32_t nat_mode, void* stream) {
    try {
        return nat_async("vpcsum_nat_async", d_arena, arena_len, d_desc, d_rw, 1, n, d_status, nat_mode, stream);
    } VPC_CATCH("vpcsum_nat_async")
}

int vpcsum_pre_async(uint8_t* d_arena, uint64_t arena_len, const vpcsum_desc_t* d_desc, const void* d_pre,
                     uint32_t pre_fmt, uint32_t n, uint32_t* d_out, uint8_t* d_status, uint32_t mode, void* stream) {
    try {
        if (n == 0) return 0;
        if (!d_arena || !d_desc || !d_pre) return fail("vpcsum_pre_async: NULL arena, descriptors or pre-images");
        if (pre_fmt > VPCSUM_PRE_FMT_PRE) return fail("vpcsum_pre_async: bad pre_fmt %u", pre_fmt);
        // tuning hints (not part of the stable ABI; nat.hip launch_pre): bit 8 byte accesses on the
        // frames, bits 12..13 packets per lane (2: two; default one), bits 16..17 window chunks (2:
        // four, 16-B entries only), bits 18..22 workgroups per CU, bit 23 the memory-pattern probe
        // (16-B entries: the same loads and stores, the stored sums written back unchanged), bit 24
        // non-temporal field stores
        if (mode & ~(VPCSUM_MODE_WRITE | 0x100u | 0x3000u | 0x1ff0000u)) return fail("vpcsum_pre_async: bad mode 0x%x", mode);
        VPC_CHECK(launch_pre(d_arena, arena_len, d_desc, d_pre, (int)pre_fmt, n, d_out, d_status, mode, (hipStream_t)stream),
                  "vpcsum_pre_async launch");
        return 0;
    } VPC_CATCH("vpcsum_pre_async")
}

int vpcsum_parse_ether_async(const uint8_t* d_arena, uint64_t arena_len, const uint64_t* d_frame_off,
                             const uint32_t* d_frame_len, uint32_t n, uint8_t flags, vpcsum_desc_t* d_desc,
                             uint8_t* d_status, void* stream) {
    try {
        if (n == 0) return 0;
        if (!d_arena || !d_frame_off || !d_frame_len || !d_desc) return fail("vpcsum_parse_ether_async: NULL argument");
        VPC_CHECK(launch_parse_ether(d_arena, arena_len, d_frame_off, d_frame_len, n, flags, d_desc, d_status, nullptr,
                                     (hipStream_t)stream),
                  "parse launch");
        return 0;
    } VPC_CATCH("vpcsum_parse_ether_async")
}

int vpcsum_parse_ether_tuples_async(const uint8_t* d_arena, uint64_t arena_len, const uint64_t* d_frame_off,
                                    const uint32_t* d_frame_len, uint32_t n, uint8_t flags, vpcsum_desc_t* d_desc,
                                    uint8_t* d_status, vpcsum_tuple_t* d_tuples, void* stream) {
    try {
        if (n == 0) return 0;
        if (!d_arena || !d_frame_off || !d_frame_len || !d_desc || !d_tuples)
            return fail("vpcsum_parse_ether_tuples_async: NULL argument");
        if ((uintptr_t)d_tuples & 3) return fail("vpcsum_parse_ether_tuples_async: tuples not 4-byte aligned");
        VPC_CHECK(launch_parse_ether(d_arena, arena_len, d_frame_off, d_frame_len, n, flags, d_desc, d_status, d_tuples,
                                     (hipStream_t)stream),
                  "parse launch");
        return 0;
    } VPC_CATCH("vpcsum_parse_ether_tuples_async")
}

int vpcsum_parse_ether_hsum_async(const uint8_t* d_arena, uint64_t arena_len, const uint64_t* d_frame_off,
                                  const uint32_t* d_frame_len, uint32_t n, uint8_t flags, vpcsum_desc_t* d_desc,
                                  uint8_t* d_status, vpcsum_hsum_t* d_hsum, void* stream) {
    try {
        if (n == 0) return 0;
        if (!d_arena || !d_frame_off || !d_frame_len || !d_desc || !d_hsum)
            return fail("vpcsum_parse_ether_hsum_async: NULL argument");
        if ((uintptr_t)d_hsum & 7) return fail("vpcsum_parse_ether_hsum_async: header sums not 8-byte aligned");
        VPC_CHECK(launch_parse_ether(d_arena, arena_len, d_frame_off, d_frame_len, n, flags, d_desc, d_status, nullptr,
                                     (hipStream_t)stream, nullptr, d_hsum),
                  "parse launch");
        return 0;
    } VPC_CATCH("vpcsum_parse_ether_hsum_async")
}

int vpcsum_read_probe_async(const uint8_t* d_buf, uint64_t bytes, uint32_t* d_sink, uint32_t grid, void* stream) {
    try {
        if (!d_buf || !d_sink) return fail("vpcsum_read_probe_async: NULL argument");
        VPC_CHECK(launch_read_probe(d_buf, bytes, d_sink, grid, (hipStream_t)stream), "read probe launch");
        return 0;
    } VPC_CATCH("vpcsum_read_probe_async")
}

int vpcsum_pattern_probe_async(const uint8_t* d_arena, uint64_t arena_len, const vpcsum_desc_t* d_desc, uint32_t n,
                               uint32_t* d_sink, uint32_t grid, void* stream) {
    try {
        if (n == 0) return 0;
        if (!d_arena || !d_desc || !d_sink) return fail("vpcsum_pattern_probe_async: NULL argument");
        if (arena_len >= (1ull << 32)) return fail("vpcsum_pattern_probe_async: arena must be < 4 GiB");
        VPC_CHECK(launch_pattern_probe(d_arena, arena_len, d_desc, n, d_sink, grid, (hipStream_t)stream),
                  "pattern probe launch");
        return 0;
    } VPC_CATCH("vpcsum_pattern_probe_async")
}

int vpcsum_synth_async(uint8_t* d_arena, uint64_t arena_len, uint32_t n, uint32_t stride, uint32_t l3_pad,
                       uint32_t workload, uint64_t seed, uint64_t first_index, vpcsum_desc_t* d_desc, void* stream) {
    try {
        if (n == 0) return 0;
        if (!d_arena && !d_desc) return fail("vpcsum_synth_async: NULL arena and descriptors");
        if (workload < VPCSUM_SYNTH_C1_UDP64 || workload > VPCSUM_SYNTH_C5_NAT1500) return fail("vpcsum_synth_async: bad workload %u", workload);
        const uint32_t maxlen = (workload == VPCSUM_SYNTH_C4_V6JUMBO || workload == VPCSUM_SYNTH_FUZZ) ? 9000
                                : (workload == VPCSUM_SYNTH_C1_UDP64) ? 50 : 1500;
        if ((uint64_t)l3_pad + maxlen > stride) return fail("vpcsum_synth_async: stride %u < l3_pad %u + %u", stride, l3_pad, maxlen);
        if (d_arena && (uint64_t)n * stride > arena_len) return fail("vpcsum_synth_async: arena too small");
        VPC_CHECK(launch_synth(d_arena, arena_len, n, stride, l3_pad, workload, seed, first_index, d_desc,
                               (hipStream_t)stream),
                  "synth launch");
        return 0;
    } VPC_CATCH("vpcsum_synth_async")
}

int vpcsum_spin_probe_async(uint32_t workgroups, uint32_t threads, uint32_t micros, void* stream) {
    try {
        if (workgroups == 0 || workgroups > 65535 || threads == 0 || threads > 1024 || (threads & 63))
            return fail("vpcsum_spin_probe_async: bad shape %u x %u", workgroups, threads);
        VPC_CHECK(launch_spin_probe(workgroups, threads, (uint64_t)micros * 100u, (hipStream_t)stream), "spin probe launch");
        return 0;
    } VPC_CATCH("vpcsum_spin_probe_async")
}

int vpcsum_event_create(void** ev) {
    try {
        if (!ev) return fail("vpcsum_event_create: NULL");
        hipEvent_t e;
        VPC_CHECK(hipEventCreate(&e), "hipEventCreate");
        *ev = (void*)e;
        return 0;
    } VPC_CATCH("vpcsum_event_create")
}
int vpcsum_event_destroy(void* ev) {
    try {
        VPC_CHECK(hipEventDestroy((hipEvent_t)ev), "hipEventDestroy");
        return 0;
    } VPC_CATCH("vpcsum_event_destroy")
}
int vpcsum_event_record(void* ev, void* stream) {
    try {
        VPC_CHECK(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream), "hipEventRecord");
        return 0;
    } VPC_CATCH("vpcsum_event_record")
}
int vpcsum_event_elapsed_ms(void* start, void* end, float* ms) {
    try {
        if (!ms) return fail("vpcsum_event_elapsed_ms: NULL");
        VPC_CHECK(hipEventSynchronize((hipEvent_t)end), "hipEventSynchronize");
        VPC_CHECK(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end), "hipEventElapsedTime");
        return 0;
    } VPC_CATCH("vpcsum_event_elapsed_ms")
}
int vpcsum_stream_sync(void* stream) {
    try {
        VPC_CHECK(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize");
        return 0;
    } VPC_CATCH("vpcsum_stream_sync")
}

// ------------------------------------------------------------------------------------------
// Context (host memory) API
// ------------------------------------------------------------------------------------------
static void slot_free(Slot& s) {
    if (s.d_arena) (void)hipFree(s.d_arena);
    if (s.d_desc) (void)hipFree(s.d_desc);
    if (s.d_out) (void)hipFree(s.d_out);
    if (s.d_status) (void)hipFree(s.d_status);
    if (s.h_desc) (void)hipHostFree(s.h_desc);
    if (s.h_out) (void)hipHostFree(s.h_out);
    if (s.h_status) (void)hipHostFree(s.h_status);
    if (s.h_arena) (void)hipHostFree(s.h_arena);
    if (s.h_foff) (void)hipHostFree(s.h_foff);
    if (s.h_flen) (void)hipHostFree(s.h_flen);
    if (s.h_rw) (void)hipHostFree(s.h_rw);
    if (s.d_rw) (void)hipFree(s.d_rw);
    if (s.h_tu) (void)hipHostFree(s.h_tu);
    if (s.h_hs) (void)hipHostFree(s.h_hs);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s = Slot();
}

static int slot_finish(vpcsum_ctx* c, Slot& s);

static void svc_free(vpcsum_ctx* c) {
    Service& v = c->svc;
    if (v.mb) __atomic_store_n(&v.mb->cmd, kSvcStop, __ATOMIC_RELEASE);
    if (v.stream) {
        (void)hipStreamSynchronize(v.stream);   // the grid sees kSvcStop within a poll interval
        (void)hipStreamDestroy(v.stream);
    }
    if (v.ctr) (void)hipFree(v.ctr);
    if (v.mb) (void)hipHostFree(v.mb);
    if (v.h_desc) (void)hipHostFree(v.h_desc);
    if (v.h_out) (void)hipHostFree(v.h_out);
    if (v.h_status) (void)hipHostFree(v.h_status);
    if (v.h_pre) (void)hipHostFree(v.h_pre);
    c->svc = Service();
}

int vpcsum_ctx_set_service(vpcsum_ctx_t* c, uint32_t idle_us) {
    try {
        if (!c) return fail("vpcsum_ctx_set_service: NULL context");
        std::lock_guard<std::mutex> lk(c->mu);
        VPC_ON_DEVICE(c->device);
        for (auto& s : c->slots)
            if (s.busy && slot_finish(c, s) != 0) return -1;
        svc_free(c);
        if (idle_us == 0) return 0;
        Service& v = c->svc;
        const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
        hipError_t e = hipSuccess;
        if ((e = hipHostMalloc((void**)&v.mb, sizeof(SvcMailbox), fl)) != hipSuccess ||
            (e = hipHostGetDevicePointer((void**)&v.dmb, v.mb, 0)) != hipSuccess ||
            (e = hipHostMalloc((void**)&v.h_desc, (size_t)c->max_pkts * sizeof(vpcsum_desc_t), fl)) != hipSuccess ||
            (e = hipHostMalloc((void**)&v.h_out, (size_t)c->max_pkts * 4, fl)) != hipSuccess ||
            (e = hipHostMalloc((void**)&v.h_status, (size_t)c->max_pkts, fl)) != hipSuccess ||
            (e = hipHostMalloc((void**)&v.h_pre, kSvcAuxBytes, fl)) != hipSuccess ||
            (e = hipHostGetDevicePointer((void**)&v.dh_pre, v.h_pre, 0)) != hipSuccess ||
            (e = hipHostGetDevicePointer((void**)&v.dh_desc, v.h_desc, 0)) != hipSuccess ||
            (e = hipHostGetDevicePointer((void**)&v.dh_out, v.h_out, 0)) != hipSuccess ||
            (e = hipHostGetDevicePointer((void**)&v.dh_status, v.h_status, 0)) != hipSuccess ||
            (e = hipMalloc((void**)&v.ctr, 16)) != hipSuccess ||   // counter + command relay
            (e = hipStreamCreateWithFlags(&v.stream, hipStreamNonBlocking)) != hipSuccess) {
            svc_free(c);
            return hipfail(e, "vpcsum_ctx_set_service allocation");
        }
        memset((void*)v.mb, 0, sizeof(SvcMailbox));
        v.mb->desc = (uint64_t)(uintptr_t)v.dh_desc;
        v.mb->out = (uint64_t)(uintptr_t)v.dh_out;
        v.mb->status = (uint64_t)(uintptr_t)v.dh_status;
        v.mb->pre = (uint64_t)(uintptr_t)v.dh_pre;
        v.idle_ticks = (uint64_t)idle_us * 100u;   // s_memrealtime runs at 100 MHz
        const char* gs = getenv("VPCSUM_SVC_GRID");   // A/B tooling: the grid's workgroups (1..256)
        if (gs && atoi(gs) >= 1 && atoi(gs) <= 256) v.grid = (uint32_t)atoi(gs);
        const char* pm = getenv("VPCSUM_SVC_POLL");   // 0: round 5's acquire loads
        if (pm) v.poll = (uint32_t)atoi(pm) & 7u;
        const char* q = getenv("VPCSUM_SVC_QUIESCE");
        v.quiesce = q && q[0] == '1';
        const char* inl = getenv("VPCSUM_SVC_INLINE");
        v.inline_desc = !(inl && inl[0] == '0');
        const char* clamp = getenv("VPCSUM_SVC_CLAMP");   // A/B tooling: 1 = clamped frame loads
        const char* reld = getenv("VPCSUM_SVC_RELEASE_DONE");   // A/B tooling: 1 = release on count / done
        v.mb->opts = ((clamp && clamp[0] == '1') ? kSvcOptClampLoads : 0) | ((reld && reld[0] == '1') ? kSvcOptReleaseDone : 0);
        v.on = true;
        return 0;
    } VPC_CATCH("vpcsum_ctx_set_service")
}

int vpcsum_ctx_stats(vpcsum_ctx_t* c, uint64_t* service_batches, uint64_t* service_launches) {
    try {
        if (!c) return fail("vpcsum_ctx_stats: NULL context");
        std::lock_guard<std::mutex> lk(c->mu);
        if (service_batches) *service_batches = c->svc_batches;
        if (service_launches) *service_launches = c->svc_launches;
        return 0;
    } VPC_CATCH("vpcsum_ctx_stats")
}

int vpcsum_ctx_create(int device, uint64_t max_arena_bytes, uint32_t max_pkts, vpcsum_ctx_t** out) {
    try {
        if (!out) return fail("vpcsum_ctx_create: out is NULL");
        if (max_arena_bytes == 0 || max_pkts == 0) return fail("vpcsum_ctx_create: zero capacity");
        VPC_ON_DEVICE(device);
        vpcsum_ctx* c = new vpcsum_ctx();
        c->device = device;
        c->max_arena = max_arena_bytes;
        c->max_pkts = max_pkts;
        for (auto& s : c->slots) {
            hipError_t e = hipSuccess;
            if ((e = hipMalloc((void**)&s.d_arena, max_arena_bytes + 64)) != hipSuccess ||
                (e = hipMalloc((void**)&s.d_desc, (size_t)max_pkts * sizeof(vpcsum_desc_t))) != hipSuccess ||
                (e = hipMalloc((void**)&s.d_out, (size_t)max_pkts * 4)) != hipSuccess ||
                (e = hipMalloc((void**)&s.d_status, (size_t)max_pkts)) != hipSuccess ||
                (e = hipHostMalloc((void**)&s.h_desc, (size_t)max_pkts * sizeof(vpcsum_desc_t), hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess ||
                (e = hipHostMalloc((void**)&s.h_out, (size_t)max_pkts * 4, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess ||
                (e = hipHostMalloc((void**)&s.h_status, (size_t)max_pkts, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess ||
                (e = hipHostGetDevicePointer((void**)&s.dh_desc, s.h_desc, 0)) != hipSuccess ||
                (e = hipHostGetDevicePointer((void**)&s.dh_out, s.h_out, 0)) != hipSuccess ||
                (e = hipHostGetDevicePointer((void**)&s.dh_status, s.h_status, 0)) != hipSuccess ||
                (e = hipHostMalloc((void**)&s.h_arena, max_arena_bytes + 64, 0)) != hipSuccess ||
                (e = hipHostMalloc((void**)&s.h_foff, (size_t)max_pkts * 8, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess ||
                (e = hipHostMalloc((void**)&s.h_flen, (size_t)max_pkts * 4, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess ||
                (e = hipHostGetDevicePointer((void**)&s.dh_foff, s.h_foff, 0)) != hipSuccess ||
                (e = hipHostGetDevicePointer((void**)&s.dh_flen, s.h_flen, 0)) != hipSuccess ||
                (e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess ||
                (e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming)) != hipSuccess) {
                for (auto& t : c->slots) slot_free(t);
                delete c;
                return hipfail(e, "vpcsum_ctx_create allocation");
            }
        }
        *out = c;
        return 0;
    } VPC_CATCH("vpcsum_ctx_create")
}

int vpcsum_ctx_destroy(vpcsum_ctx_t* c) {
    try {
        if (!c) return 0;
        DeviceScope on_dev(c->device);
        int rc = 0;
        {
            std::lock_guard<std::mutex> lk(c->mu);
            // batches still in flight complete first, as a wait would: their out / status (and a
            // staged batch's frames) reach the caller's buffers before anything is freed.  A failure
            // is reported, and the context is destroyed all the same.
            for (auto& s : c->slots)
                if (s.busy && slot_finish(c, s) != 0) rc = -1;
            svc_free(c);
            for (auto& s : c->slots) {
                if (s.stream) (void)hipStreamSynchronize(s.stream);
                slot_free(s);
            }
            // every page-lock reference this context holds goes, each failure reported (the caller
            // may free the arena once this returns: a range HIP still held as registered would be taken
            // for pinned memory by a later copy from whatever is allocated there)
            for (auto& r : c->registered)
                if (r.key && hostlock_release(r.key, "vpcsum_ctx_destroy") != 0) rc = -1;
        }
        delete c;
        return rc;
    } VPC_CATCH("vpcsum_ctx_destroy")
}

int vpcsum_ctx_register_arena(vpcsum_ctx_t* c, void* h_arena, uint64_t len) {
    try {
        if (!c || !h_arena || len == 0) return fail("vpcsum_ctx_register_arena: bad argument");
        std::lock_guard<std::mutex> lk(c->mu);
        VPC_ON_DEVICE(c->device);
        for (auto& r : c->registered)
            if (r.host == (uint8_t*)h_arena) return fail("vpcsum_ctx_register_arena: %p is registered already", h_arena);
        c->registered.reserve(c->registered.size() + 1);   // may throw: before anything is pinned
        uint8_t* key = nullptr;
        if (hostlock_acquire((uint8_t*)h_arena, len, &key, "vpcsum_ctx_register_arena") != 0) return -1;
        void* dev = nullptr;
        hipError_t e = hipHostGetDevicePointer(&dev, h_arena, 0);
        if (e != hipSuccess) {
            (void)hostlock_release(key, "vpcsum_ctx_register_arena");
            return hipfail(e, "hipHostGetDevicePointer");
        }
        c->registered.push_back({(uint8_t*)h_arena, len, (uint8_t*)dev, key});
        return 0;
    } VPC_CATCH("vpcsum_ctx_register_arena")
}

// A zero-copy batch (launched or on the service grid) may still read and write frames of a
// registered arena in place: finish every such batch of the context before a mapping goes away,
// and make the service re-read its parameters (they may name that arena) with its next batch.
// Caller holds c->mu on c's device.
static int ctx_quiesce_zero_copy(vpcsum_ctx* c) {
    for (auto& s : c->slots)
        if (s.busy && s.zero_copy && slot_finish(c, s) != 0) return -1;
    c->svc.par_valid = false;
    return 0;
}

int vpcsum_ctx_unregister_arena(vpcsum_ctx_t* c, void* h_arena) {
    try {
        if (!c || !h_arena) return fail("vpcsum_ctx_unregister_arena: bad argument");
        std::lock_guard<std::mutex> lk(c->mu);
        VPC_ON_DEVICE(c->device);
        for (size_t i = 0; i < c->registered.size(); ++i) {
            if (c->registered[i].host == (uint8_t*)h_arena) {
                if (ctx_quiesce_zero_copy(c) != 0) return -1;
                uint8_t* key = c->registered[i].key;
                c->registered.erase(c->registered.begin() + i);
                return key ? hostlock_release(key, "vpcsum_ctx_unregister_arena") : 0;
            }
        }
        return fail("vpcsum_ctx_unregister_arena: arena not registered");
    } VPC_CATCH("vpcsum_ctx_unregister_arena")
}

// Device-side address of host range [p, p+len) if it lies in an arena registered with this context.
static uint8_t* mapped_dev(vpcsum_ctx* c, const uint8_t* p, uint64_t len) {
    for (auto& r : c->registered)
        if (p >= r.host && p + len <= r.host + r.len) return r.dev + (p - r.host);
    return nullptr;
}

// Whether the staged path may DMA straight from [p, p+len): only when this context registered it
// (its own registration or its group's), so the page-lock outlives the copy -- vpcsum_ctx_unregister
// and destroy finish the context's batches before they unpin.  Memory page-locked by anyone else
// (another context, hipHostMalloc, another library) is copied through the pinned staging first: its
// owner may unpin or free it while the copy is in flight, which the library cannot see (round 5's
// version trusted hipPointerGetAttributes here; DESIGN_HISTORY.md "Round 6: the intermittent fault").
static bool is_registered(vpcsum_ctx* c, const uint8_t* p, uint64_t len) { return mapped_dev(c, p, len) != nullptr; }

static uint32_t svc_done(const Service& v) { return __atomic_load_n(&v.mb->done, __ATOMIC_ACQUIRE); }

// (Re)start the service grid: it treats batches after `seen` as new.  Only called while no grid
// of this context runs (stream idle), so the finished-wave counter can be cleared first.
static int svc_launch(vpcsum_ctx* c, uint32_t seen) {
    Service& v = c->svc;
    VPC_CHECK(hipMemsetAsync(v.ctr, 0, 16, v.stream), "service counter / relay reset");
    VPC_CHECK(launch_service(v.dmb, v.ctr, seen, v.idle_ticks, v.stream, v.grid, v.poll), "service launch");
    ++c->svc_launches;
    return 0;
}

// Wait until the service has completed batch `seq`.  A grid that left on its idle timeout while
// the batch was being posted may have done part of it: once the stream is idle the batch is run
// again from the start by a fresh grid (the sums do not read the fields they write).
#ifdef VPCSUM_SVC_STAMPS
// tooling build: per-batch durations of the service's steps (ns), medians per batch size at exit
static std::map<uint32_t, std::vector<uint64_t>> g_stamp_d[7];
static void stamps_print() {
    static const char* name[7] = {"host_post_to_done_seen_ns", "wg0_params_ns", "wg0_k1_ns", "wg0_release_ns",
                                  "wg0_atomic_ns", "wg0_seen_to_done_store_ns", "last_wg_seen_after_wg0_ns"};
    for (auto& kv : g_stamp_d[0]) {
        fprintf(stderr, "{\"n\": %u", kv.first);
        for (int i = 0; i < 7; ++i) {
            auto v = g_stamp_d[i][kv.first];
            std::sort(v.begin(), v.end());
            fprintf(stderr, ", \"%s\": %llu", name[i], (unsigned long long)v[v.size() / 2]);
        }
        fprintf(stderr, "}\n");
    }
}
#endif

static int svc_wait(vpcsum_ctx* c, uint32_t seq) {
    Service& v = c->svc;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 1; (int32_t)(svc_done(v) - seq) < 0; ++spin) {
        __builtin_ia32_pause();
        if ((spin & 255) != 0) continue;
        if (hipStreamQuery(v.stream) == hipSuccess && (int32_t)(svc_done(v) - seq) < 0) {
            if (svc_launch(c, seq - 1) != 0) return -1;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10))
            return fail("vpcsum service: batch %u not completed within 10 s", seq);
    }
#ifdef VPCSUM_SVC_STAMPS
    {
        static bool reg = false;
        if (!reg) { reg = true; atexit(stamps_print); }
        const uint64_t* s = (const uint64_t*)v.mb->stamp;
        const uint64_t s0 = s[0];
        const uint32_t n = v.t_n;
        g_stamp_d[0][n].push_back((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
            std::chrono::steady_clock::now() - v.t_post).count());
        for (int i = 1; i <= 4; ++i) g_stamp_d[i][n].push_back((s[i] - s[i - 1]) * 10);
        g_stamp_d[5][n].push_back((s[5] - s0) * 10);
        g_stamp_d[6][n].push_back((s[6] - s0) * 10);
    }
#endif
    return 0;
}

static int slot_finish(vpcsum_ctx* c, Slot& s) {
    if (!s.busy) return 0;
    if (s.svc_seq) {
        if (svc_wait(c, s.svc_seq) != 0) return -1;
    } else {
        VPC_CHECK(hipEventSynchronize(s.done), "hipEventSynchronize");
    }
    if (s.kind == 1) {
        // NAT: a staged batch's rewritten headers (L3 header through the L4 checksum field)
        // go back into the caller's frames; zero-copy batches rewrote them in place
        if (!s.zero_copy && s.user_arena) {
            for (uint32_t i = 0; i < s.n; ++i) {
                if (s.h_status[i] & VPCSUM_S_BAD_DESC) continue;
                const vpcsum_desc_t& d = s.user_desc[i];
                const int fld = d.l4_proto == 6 ? 16 : d.l4_proto == 17 ? 6 : (d.l4_proto == 1 || d.l4_proto == 58) ? 2 : -1;
                uint32_t end = d.l3_ver == 4 ? 20 : 40;
                if (fld >= 0 && d.l3_len >= d.l4_off + fld + 2) end = std::max<uint32_t>(end, d.l4_off + fld + 2u);
                end = std::min<uint32_t>(end, d.l3_len);
                memcpy(s.user_arena + d.l3_off, s.h_arena + s.h_desc[i].l3_off, end);
            }
        }
        if (s.user_status) memcpy(s.user_status, s.h_status, s.n);
        s.busy = false;
        return 0;
    }
    if (s.kind == 2) {   // parse: descriptors, status and tuples were written to the pinned staging
        const bool svc = s.svc_seq != 0;   // or, through the service grid, to its aux buffer
        const uint8_t* aux = (const uint8_t*)c->svc.h_pre;
        if (s.user_desc_out)
            memcpy(s.user_desc_out, svc ? aux : (const uint8_t*)s.h_desc, (size_t)s.n * sizeof(vpcsum_desc_t));
        if (s.user_status) memcpy(s.user_status, svc ? c->svc.h_status : s.h_status, s.n);
        if (s.user_tuples)
            memcpy(s.user_tuples, svc ? aux + (size_t)kSvcBatchMax * sizeof(vpcsum_desc_t) : (const uint8_t*)s.h_tu,
                   (size_t)s.n * sizeof(vpcsum_tuple_t));
        s.busy = false;
        s.svc_seq = 0;
        return 0;
    }
    const uint32_t* res_out = s.svc_seq ? c->svc.h_out : s.h_out;
    const uint8_t* res_status = s.svc_seq ? c->svc.h_status : s.h_status;
    if (s.user_out) memcpy(s.user_out, res_out, (size_t)s.n * 4);
    if (s.user_status) memcpy(s.user_status, res_status, s.n);
    if (s.user_hsum)   // a verify batch's header sums: the service's aux buffer, or the slot's staging
        memcpy(s.user_hsum, s.svc_seq ? (const void*)c->svc.h_pre : (const void*)s.h_hs, (size_t)s.n * sizeof(vpcsum_hsum_t));
    s.user_hsum = nullptr;
    if ((s.mode & VPCSUM_MODE_WRITE) && s.user_arena && !s.zero_copy) {
        // place the GPU results into the caller's frames (big endian, as ByteArray.int16)
        for (uint32_t i = 0; i < s.n; ++i) {
            const vpcsum_desc_t& d = s.user_desc[i];
            if (res_status[i] & VPCSUM_S_BAD_DESC) continue;
            uint8_t* l3 = s.user_arena + d.l3_off;
            const uint32_t w = res_out[i];
            if (d.flags & VPCSUM_F_IP) { l3[10] = (uint8_t)(w >> 8); l3[11] = (uint8_t)w; }
            if (d.flags & (VPCSUM_F_L4 | VPCSUM_F_L4P)) {
                const int fld = d.l4_proto == 6 ? 16 : d.l4_proto == 17 ? 6 : 2;
                l3[d.l4_off + fld] = (uint8_t)(w >> 24);
                l3[d.l4_off + fld + 1] = (uint8_t)(w >> 16);
            }
        }
    }
    s.busy = false;
    s.svc_seq = 0;
    return 0;
}

// The slot's per-packet entry staging (NAT rewrites, pre-images: at most 48 B each), pinned and
// mapped plus a device copy, allocated with the context's first batch that carries entries.
static int slot_rw_alloc(vpcsum_ctx* c, Slot& s, const char* what) {
    if (s.h_rw) return 0;
    hipError_t e = hipSuccess;
    const size_t bytes = (size_t)c->max_pkts * sizeof(vpcsum_nat_t);
    if ((e = hipHostMalloc((void**)&s.h_rw, bytes, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void**)&s.dh_rw, s.h_rw, 0)) != hipSuccess ||
        (e = hipMalloc((void**)&s.d_rw, bytes)) != hipSuccess) {
        if (s.h_rw) (void)hipHostFree(s.h_rw);
        if (s.d_rw) (void)hipFree(s.d_rw);
        s.h_rw = s.dh_rw = s.d_rw = nullptr;
        return hipfail(e, what);
    }
    return 0;
}

static int l4_field_host(int proto) { return proto == 6 ? 16 : proto == 17 ? 6 : (proto == 1 || proto == 58) ? 2 : -1; }

// The service runs one batch at a time: the previous one done, its results handed over, before its
// buffers are refilled.
static int svc_drain(vpcsum_ctx* c) {
    for (auto& o : c->slots)
        if (o.busy && o.svc_seq && slot_finish(c, o) != 0) return -1;
    return 0;
}

// Before a launched zero-copy batch (more than kSvcBatchMax frames, or a form the grid does not
// take), round 5 stopped a resident grid that had had no batch for kSvcKeep: with an idle grid
// resident, launched batches ran 6-50% slower.  The cause (round 6, tools/svc_interference.cpp,
// profiles/r06e_svc_interference.json, r06f_svc_poll.json) was the grid's relay pollers: 31
// workgroups re-reading the relay word with an agent-scope ACQUIRE load, each one a cache
// invalidate, while a sleeping grid of the same shape cost nothing.  With relaxed relay loads (the
// acquire fence after the poll orders the batch, kernels.hip k_csum_service) a resident grid costs
// the launched batches nothing measurable, so it stays: the stop is now opt-in
// (VPCSUM_SVC_QUIESCE=1, the A/B of round 5's policy) and a small flush after a large one no
// longer pays a grid launch.
constexpr auto kSvcKeep = std::chrono::microseconds(1000);
static int svc_quiesce(vpcsum_ctx* c) {
    Service& v = c->svc;
    if (!v.quiesce || !v.on || hipStreamQuery(v.stream) == hipSuccess) return 0;   // off, or no grid resident
    if (std::chrono::steady_clock::now() - v.last_post < kSvcKeep) return 0;
    if (svc_drain(c) != 0) return -1;
    __atomic_store_n(&v.mb->cmd, kSvcStop | v.posted, __ATOMIC_RELEASE);
    VPC_CHECK(hipStreamSynchronize(v.stream), "service stop");
    return 0;
}

// Hand a zero-copy batch to the low-latency service (c->svc.on, n <= kSvcBatchMax): one batch at
// a time; descriptors (and pre-images) into the service's buffers, the parameter block if it
// changed, then the command word.  `base` is the device address of h_arena[0].  Caller holds c->mu
// on c's device; slot s (ticket t) is free.
// frames: h_desc is the service's own buffer, filled with SvcFrameRec records (raw frames); parse:
// the frames are parsed only (vpcsum_ctx_parse_frames).
static int svc_post(vpcsum_ctx* c, Slot& s, uint64_t t, uint8_t* h_arena, uint64_t arena_len, uint8_t* base,
                    const vpcsum_desc_t* h_desc, uint32_t n, uint32_t* h_out, uint8_t* h_status, uint32_t mode,
                    const void* h_pre, uint32_t pre_fmt, uint64_t* ticket, bool frames = false, bool parse = false,
                    bool hsum = false) {
    Service& v = c->svc;
    SvcMailbox* mb = v.mb;
    if (!frames) memcpy(v.h_desc, h_desc, (size_t)n * sizeof(vpcsum_desc_t));
    uint64_t cmd = (frames ? kSvcFrames : 0) | (parse ? kSvcParse : 0) | (hsum ? kSvcHsum : 0);
    if (h_pre) {
        // the pre-images, each F_PRE frame's stored L4 sum copied into its entry's spare bytes
        // (vpcsum_pre4_t rsv[1..2], vpcsum_pre_t rsv[0..1]): the kernel takes the sum from there,
        // so a batch re-run by a fresh grid (svc_wait) computes from the same input
        const size_t esz = pre_fmt == VPCSUM_PRE_FMT_PRE ? sizeof(vpcsum_pre_t) : sizeof(vpcsum_pre4_t);
        const size_t at = pre_fmt == VPCSUM_PRE_FMT_PRE ? offsetof(vpcsum_pre_t, rsv) : offsetof(vpcsum_pre4_t, rsv) + 1;
        memcpy(v.h_pre, h_pre, (size_t)n * esz);
        for (uint32_t i = 0; i < n; ++i) {
            const vpcsum_desc_t& d = h_desc[i];
            const int fld = l4_field_host(d.l4_proto);
            if (!(d.flags & VPCSUM_F_PRE) || fld < 0 || d.l3_off > arena_len || d.l3_len > arena_len - d.l3_off ||
                (uint32_t)d.l4_off + fld + 2u > d.l3_len)
                continue;   // no L4 sum to update, or refused by the kernel
            memcpy((uint8_t*)v.h_pre + (size_t)i * esz + at, h_arena + d.l3_off + d.l4_off + fld, 2);
        }
        cmd |= kSvcPre | (pre_fmt == VPCSUM_PRE_FMT_PRE ? kSvcPreFmt : 0);
    }
    const uint64_t par[3] = {(uint64_t)(uintptr_t)base, arena_len, (mode & VPCSUM_MODE_WRITE) ? (uint64_t)(uintptr_t)base : 0};
    if (!v.par_valid || memcmp(par, v.par, sizeof(par)) != 0) {
        mb->arena = par[0];
        mb->arena_len = par[1];
        mb->arena_w = par[2];
        memcpy(v.par, par, sizeof(par));
        v.par_valid = true;
        cmd |= kSvcParams;
    }
    const uint32_t seq = v.posted + 1 ? v.posted + 1 : 1;
    // the first descriptors ride in the command's line, tagged with the batch.  All of them are
    // rewritten for every batch, so a stale one always carries the previous batch's tag; the high
    // word (with the tag) is stored after the low one.
    for (int k = 0; k < kSvcInlineDesc; ++k) {
        vpcsum_desc_t d;
        if ((uint32_t)k < n) memcpy(&d, &h_desc[k], sizeof(d));
        else memset(&d, 0, sizeof(d));
        d.rsv = (uint8_t)seq;
        uint64_t w[2];
        memcpy(w, &d, sizeof(w));
        uint64_t* dst = reinterpret_cast<uint64_t*>(&mb->idesc[k]);
        __atomic_store_n(&dst[0], w[0], __ATOMIC_RELAXED);
        __atomic_store_n(&dst[1], w[1], __ATOMIC_RELEASE);
    }
    cmd |= seq | ((uint64_t)n << 32) | ((mode & VPCSUM_MODE_VERIFY) ? kSvcVerify : 0) |
           (v.inline_desc && n <= (uint32_t)kSvcInlineDesc ? kSvcInline : 0);
#ifdef VPCSUM_SVC_STAMPS
    v.t_post = std::chrono::steady_clock::now();
    v.t_n = n;
#endif
    __atomic_store_n(&mb->cmd, cmd, __ATOMIC_RELEASE);
    v.posted = seq;
    v.last_post = std::chrono::steady_clock::now();
    ++c->svc_batches;
    if (hipStreamQuery(v.stream) == hipSuccess && svc_launch(c, seq - 1) != 0) return -1;
    s.zero_copy = true;
    s.svc_seq = seq;
    s.kind = 0;
    s.busy = true;
    s.ticket = t;
    s.n = n;
    s.mode = mode;
    s.user_arena = h_arena;
    s.user_desc = h_desc;
    s.user_out = h_out;
    s.user_status = h_status;
    *ticket = t;
    return 0;
}

// A small batch of raw frames (egress, RX verify or RX parse) to the service grid: one SvcFrameRec
// per frame in the service's descriptor buffer -- offset, length, and the frame's own flags
// (h_flags) or `flags` for all -- then svc_post.  The results stay in the service's buffers until
// slot_finish hands them over; the frames themselves are written in place through the mapping.
static int svc_post_frames(vpcsum_ctx* c, Slot& s, uint64_t t, const uint8_t* h_arena, uint64_t arena_len, uint8_t* base,
                           const uint64_t* h_off, const uint32_t* h_len, const uint8_t* h_flags, uint8_t flags,
                           uint32_t n, uint32_t* h_out, uint8_t* h_status, uint32_t mode, bool parse, uint64_t* ticket,
                           bool hsum = false) {
    if (svc_drain(c) != 0) return -1;
    SvcFrameRec* r = reinterpret_cast<SvcFrameRec*>(c->svc.h_desc);
    for (uint32_t i = 0; i < n; ++i) {
        SvcFrameRec x;
        memset(&x, 0, sizeof(x));
        x.off = h_off[i];
        x.len = h_len[i];
        x.flags = h_flags ? h_flags[i] : flags;
        memcpy(&r[i], &x, sizeof(x));
    }
    if (svc_post(c, s, t, const_cast<uint8_t*>(h_arena), arena_len, base, c->svc.h_desc, n, h_out, h_status, mode, nullptr,
                 0, ticket, true, parse, hsum) != 0)
        return -1;
    s.user_arena = nullptr;
    s.user_desc = nullptr;
    return 0;
}

int vpcsum_ctx_submit(vpcsum_ctx_t* c, uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc, uint32_t n,
                      uint32_t* h_out, uint8_t* h_status, uint32_t mode, uint64_t* ticket) {
    try {
        if (!c || !ticket) return fail("vpcsum_ctx_submit: NULL context or ticket");
        if (n > c->max_pkts) return fail("vpcsum_ctx_submit: %u packets > capacity %u", n, c->max_pkts);
        if (n && (!h_arena || !h_desc)) return fail("vpcsum_ctx_submit: NULL arena or descriptors");
        if (mode & ~(VPCSUM_MODE_VERIFY | VPCSUM_MODE_WRITE)) return fail("vpcsum_ctx_submit: bad mode 0x%x", mode);
        std::lock_guard<std::mutex> lk(c->mu);
        VPC_ON_DEVICE(c->device);
        const uint64_t t = c->next_ticket++;
        Slot& s = c->slots[t & 1];
        if (s.busy && slot_finish(c, s) != 0) return -1;

        // byte span the descriptors touch (16-B aligned so device alignment == host alignment)
        uint64_t lo = UINT64_MAX, hi = 0, used = 0;
        for (uint32_t i = 0; i < n; ++i) {
            const vpcsum_desc_t& d = h_desc[i];
            if (d.l3_off > arena_len || d.l3_len > arena_len - d.l3_off) continue;   // kernel flags it BAD
            lo = std::min(lo, d.l3_off);
            hi = std::max(hi, d.l3_off + d.l3_len);
            used += d.l3_len + 16;
        }
        if (lo == UINT64_MAX) { lo = 0; hi = 0; }
        lo &= ~(uint64_t)15;
        const uint64_t span = hi - lo;
        s.zero_copy = false;

        uint8_t* dev_arena = span ? mapped_dev(c, h_arena + lo, span) : nullptr;
        if (dev_arena) {
            // Zero-copy: the frames live in a page-locked, mapped arena (an AF_XDP umem).  The
            // kernel reads them over PCIe in place, takes the descriptors from and writes the
            // results to pinned staging, and with MODE_WRITE stores the checksum fields straight
            // into the frames -- no DMA copy in either direction.
            uint8_t* base = dev_arena - lo;   // device address of h_arena[0]
            if (c->svc.on && n <= kSvcBatchMax) {
                if (svc_drain(c) != 0) return -1;
                return svc_post(c, s, t, h_arena, arena_len, base, h_desc, n, h_out, h_status, mode, nullptr, 0, ticket);
            }
            if (svc_quiesce(c) != 0) return -1;
            memcpy(s.h_desc, h_desc, (size_t)n * sizeof(vpcsum_desc_t));
            // up to kZeroCopyWaveTeams packets: one wave per packet (variant 12, 64 lanes x 4
            // predicated loads), so the batch is a few PCIe round trips deep instead of K2's per-unit
            // iterations, and no chunk is read twice over PCIe
            const int variant = n <= kZeroCopyWaveTeams ? 12 : 0;
            // no out words asked for (an ingress verify: the status bytes are the result): none written
            VPC_CHECK(launch_csum(base, arena_len, s.dh_desc, n, h_out ? s.dh_out : nullptr, s.dh_status, nullptr,
                                  mode & VPCSUM_MODE_VERIFY, (mode & VPCSUM_MODE_WRITE) ? base : nullptr, variant, 0,
                                  s.stream),
                      "checksum launch (zero-copy)");
            s.zero_copy = true;
        } else {
            const bool gather = span > 2 * used + (64u << 10);
            uint64_t dev_len = span;
            if (gather) {
                // sparse batch in a large pageable arena: gather the touched 16-B blocks only
                uint64_t pos = 0;
                for (uint32_t i = 0; i < n; ++i) {
                    const vpcsum_desc_t& d = h_desc[i];
                    s.h_desc[i] = d;
                    if (d.l3_off > arena_len || d.l3_len > arena_len - d.l3_off) { s.h_desc[i].l3_off = UINT64_MAX; continue; }
                    const uint64_t a0 = d.l3_off & ~(uint64_t)15;
                    const uint64_t a1 = std::min<uint64_t>((d.l3_off + d.l3_len + 15) & ~(uint64_t)15, arena_len);
                    if (pos + (a1 - a0) > c->max_arena) return fail("vpcsum_ctx_submit: gathered batch exceeds capacity");
                    memcpy(s.h_arena + pos, h_arena + a0, a1 - a0);
                    s.h_desc[i].l3_off = pos + (d.l3_off - a0);
                    pos += (a1 - a0 + 15) & ~(uint64_t)15;
                }
                dev_len = pos;
            } else {
                if (span > c->max_arena) return fail("vpcsum_ctx_submit: batch spans %llu bytes > capacity %llu",
                                                     (unsigned long long)span, (unsigned long long)c->max_arena);
                // descriptors rebased to the device copy of [lo, hi)
                for (uint32_t i = 0; i < n; ++i) {
                    s.h_desc[i] = h_desc[i];
                    if (h_desc[i].l3_off >= lo) s.h_desc[i].l3_off = h_desc[i].l3_off - lo;
                    else s.h_desc[i].l3_off = UINT64_MAX;   // out of span -> BAD in the kernel
                }
            }
            VPC_CHECK(hipMemcpyAsync(s.d_desc, s.h_desc, (size_t)n * sizeof(vpcsum_desc_t), hipMemcpyHostToDevice, s.stream),
                      "H2D descriptors");
            if (dev_len) {
                const uint8_t* src = gather ? s.h_arena : h_arena + lo;
                if (!gather && !is_registered(c, src, span)) {
                    memcpy(s.h_arena, src, span);   // pageable -> pinned staging
                    src = s.h_arena;
                }
                VPC_CHECK(hipMemcpyAsync(s.d_arena, src, dev_len, hipMemcpyHostToDevice, s.stream), "H2D arena");
            }
            // the out words travel when the caller asked for them or MODE_WRITE places them in the frames
            const bool want_out = h_out || (mode & VPCSUM_MODE_WRITE);
            VPC_CHECK(launch_csum(s.d_arena, dev_len, s.d_desc, n, want_out ? s.d_out : nullptr, s.d_status, nullptr,
                                  mode & VPCSUM_MODE_VERIFY, nullptr, 0, 0, s.stream),
                      "checksum launch");
            if (want_out)
                VPC_CHECK(hipMemcpyAsync(s.h_out, s.d_out, (size_t)n * 4, hipMemcpyDeviceToHost, s.stream), "D2H out");
            VPC_CHECK(hipMemcpyAsync(s.h_status, s.d_status, n, hipMemcpyDeviceToHost, s.stream), "D2H status");
        }
        VPC_CHECK(hipEventRecord(s.done, s.stream), "hipEventRecord");
        s.kind = 0;
        s.busy = true;
        s.ticket = t;
        s.n = n;
        s.mode = mode;
        s.user_arena = h_arena;
        s.user_desc = h_desc;
        s.user_out = h_out;
        s.user_status = h_status;
        *ticket = t;
        return 0;
    } VPC_CATCH("vpcsum_ctx_submit")
}

int vpcsum_ctx_submit_pre(vpcsum_ctx_t* c, uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc,
                          const void* h_pre, uint32_t pre_fmt, uint32_t n, uint32_t* h_out, uint8_t* h_status,
                          uint32_t mode, uint64_t* ticket) {
    try {
        if (!c || !ticket) return fail("vpcsum_ctx_submit_pre: NULL context or ticket");
        if (n > c->max_pkts) return fail("vpcsum_ctx_submit_pre: %u packets > capacity %u", n, c->max_pkts);
        if (n && (!h_arena || !h_desc || !h_pre)) return fail("vpcsum_ctx_submit_pre: NULL arena, descriptors or pre-images");
        if (pre_fmt > VPCSUM_PRE_FMT_PRE) return fail("vpcsum_ctx_submit_pre: bad pre_fmt %u", pre_fmt);
        if (mode & ~VPCSUM_MODE_WRITE) return fail("vpcsum_ctx_submit_pre: bad mode 0x%x (COMPUTE or WRITE)", mode);
        uint32_t npre = 0;
        for (uint32_t i = 0; i < n; ++i) npre += (h_desc[i].flags & VPCSUM_F_PRE) ? 1u : 0u;
        // no pre-image in the batch: a plain submit (the service grid may take it)
        if (npre == 0) return vpcsum_ctx_submit(c, h_arena, arena_len, h_desc, n, h_out, h_status, mode, ticket);
        const size_t esz = pre_fmt == VPCSUM_PRE_FMT_PRE ? sizeof(vpcsum_pre_t) : sizeof(vpcsum_pre4_t);
        const bool full = npre < n;   // descriptors the checksum kernel sums in full
        std::lock_guard<std::mutex> lk(c->mu);
        VPC_ON_DEVICE(c->device);
        const uint64_t t = c->next_ticket++;
        Slot& s = c->slots[t & 1];
        if (s.busy && slot_finish(c, s) != 0) return -1;
        uint64_t lo = UINT64_MAX, hi = 0;
        for (uint32_t i = 0; i < n; ++i) {
            const vpcsum_desc_t& d = h_desc[i];
            if (d.l3_off > arena_len || d.l3_len > arena_len - d.l3_off) continue;   // the kernels flag it BAD
            lo = std::min(lo, d.l3_off);
            hi = std::max(hi, d.l3_off + d.l3_len);
        }
        if (lo == UINT64_MAX) { lo = 0; hi = 0; }
        lo &= ~(uint64_t)15;
        uint8_t* dev_arena = hi > lo ? mapped_dev(c, h_arena + lo, hi - lo) : nullptr;
        const uint32_t wr = mode & VPCSUM_MODE_WRITE;
        // a small flush from the registered umem: the service grid, F_PRE frames and the others in
        // one batch (kernels.hip svc_pre_packet)
        if (dev_arena && c->svc.on && n <= kSvcBatchMax) {
            if (svc_drain(c) != 0) return -1;
            return svc_post(c, s, t, h_arena, arena_len, dev_arena - lo, h_desc, n, h_out, h_status, mode, h_pre, pre_fmt,
                            ticket);
        }
        if (slot_rw_alloc(c, s, "vpcsum_ctx_submit_pre allocation") != 0) return -1;
        memcpy(s.h_rw, h_pre, (size_t)n * esz);
        if (dev_arena) {
            // registered arena (umem): in place; an F_PRE packet's header is all that crosses PCIe
            if (svc_quiesce(c) != 0) return -1;
            uint8_t* base = dev_arena - lo;
            memcpy(s.h_desc, h_desc, (size_t)n * sizeof(vpcsum_desc_t));
            if (full)
                VPC_CHECK(launch_csum(base, arena_len, s.dh_desc, n, s.dh_out, s.dh_status, nullptr, VPCSUM_MODE_COMPUTE,
                                      wr ? base : nullptr, n <= kZeroCopyWaveTeams ? 12 : 0, 0, s.stream),
                          "checksum launch (zero-copy)");
            VPC_CHECK(launch_pre(base, arena_len, s.dh_desc, s.dh_rw, (int)pre_fmt, n, s.dh_out, s.dh_status, wr, s.stream),
                      "pre-image launch (zero-copy)");
            s.zero_copy = true;
        } else {
            // staged: each packet's 16-B blocks gathered into the pinned staging -- of an F_PRE
            // packet only its header through the L4 checksum field (its descriptor's l3_len cut to
            // that: the kernel reads no further), unless it is UDP with a stored 0, which is summed
            // in full
            uint64_t pos = 0;
            for (uint32_t i = 0; i < n; ++i) {
                const vpcsum_desc_t& d = h_desc[i];
                s.h_desc[i] = d;
                if (d.l3_off > arena_len || d.l3_len > arena_len - d.l3_off) { s.h_desc[i].l3_off = UINT64_MAX; continue; }
                uint32_t take = d.l3_len;
                const int fld = l4_field_host(d.l4_proto);
                if ((d.flags & VPCSUM_F_PRE) && fld >= 0 && (uint32_t)d.l4_off + fld + 2u <= d.l3_len) {
                    const uint8_t* f = h_arena + d.l3_off + d.l4_off + fld;
                    if (!(d.l4_proto == 17 && f[0] == 0 && f[1] == 0)) {
                        // through the checksum field, or through the L4 header a header-sum entry covers
                        const uint8_t* e = (const uint8_t*)h_pre + (size_t)i * esz;
                        const uint8_t emask = e[pre_fmt == VPCSUM_PRE_FMT_PRE ? offsetof(vpcsum_pre_t, mask)
                                                                               : offsetof(vpcsum_pre4_t, mask)];
                        const uint32_t hl = (emask & VPCSUM_PRE_HSUM) ? e[offsetof(vpcsum_hsum_t, hlen)] : 0u;
                        take = std::max<uint32_t>(d.l3_ver == 4 ? 20u : 40u,
                                                  (uint32_t)d.l4_off + std::max<uint32_t>(fld + 2u, hl));
                        take = std::min<uint32_t>(take, d.l3_len);
                        s.h_desc[i].l3_len = (uint16_t)take;
                        if (emask & VPCSUM_PRE_HSUM) {
                            // the kernel checks the record's segment length against the descriptor's,
                            // which is cut here: check it against the real one on the host, and hand the
                            // kernel the cut length (or, on a mismatch, a record it refuses)
                            vpcsum_hsum_t hs;
                            uint8_t* se = (uint8_t*)s.h_rw + (size_t)i * esz;
                            memcpy(&hs, se, sizeof(hs));
                            if (hs.l4_len == (uint32_t)d.l3_len - d.l4_off) hs.l4_len = (uint16_t)(take - d.l4_off);
                            else hs.l2_len = 0;
                            memcpy(se, &hs, sizeof(hs));
                        }
                    }
                }
                const uint64_t a0 = d.l3_off & ~(uint64_t)15;
                const uint64_t a1 = std::min<uint64_t>((d.l3_off + take + 15) & ~(uint64_t)15, arena_len);
                if (pos + (a1 - a0) > c->max_arena) return fail("vpcsum_ctx_submit_pre: gathered batch exceeds capacity");
                memcpy(s.h_arena + pos, h_arena + a0, a1 - a0);
                s.h_desc[i].l3_off = pos + (d.l3_off - a0);
                pos += (a1 - a0 + 15) & ~(uint64_t)15;
            }
            VPC_CHECK(hipMemcpyAsync(s.d_desc, s.h_desc, (size_t)n * sizeof(vpcsum_desc_t), hipMemcpyHostToDevice, s.stream),
                      "H2D descriptors");
            VPC_CHECK(hipMemcpyAsync(s.d_rw, s.h_rw, (size_t)n * esz, hipMemcpyHostToDevice, s.stream), "H2D pre-images");
            if (pos) VPC_CHECK(hipMemcpyAsync(s.d_arena, s.h_arena, pos, hipMemcpyHostToDevice, s.stream), "H2D frames");
            if (full)
                VPC_CHECK(launch_csum(s.d_arena, pos, s.d_desc, n, s.d_out, s.d_status, nullptr, VPCSUM_MODE_COMPUTE, nullptr,
                                      0, 0, s.stream),
                          "checksum launch");
            // the sums go back through out: slot_finish writes them into the caller's frames
            VPC_CHECK(launch_pre(s.d_arena, pos, s.d_desc, s.d_rw, (int)pre_fmt, n, s.d_out, s.d_status, 0, s.stream),
                      "pre-image launch");
            VPC_CHECK(hipMemcpyAsync(s.h_out, s.d_out, (size_t)n * 4, hipMemcpyDeviceToHost, s.stream), "D2H out");
            VPC_CHECK(hipMemcpyAsync(s.h_status, s.d_status, n, hipMemcpyDeviceToHost, s.stream), "D2H status");
            s.zero_copy = false;
        }
        VPC_CHECK(hipEventRecord(s.done, s.stream), "hipEventRecord");
        s.kind = 0;
        s.svc_seq = 0;
        s.busy = true;
        s.ticket = t;
        s.n = n;
        s.mode = mode;
        s.user_arena = h_arena;
        s.user_desc = h_desc;
        s.user_out = h_out;
        s.user_status = h_status;
        *ticket = t;
        return 0;
    } VPC_CATCH("vpcsum_ctx_submit_pre")
}

int vpcsum_ctx_wait(vpcsum_ctx_t* c, uint64_t ticket) {
    try {
        if (!c) return fail("vpcsum_ctx_wait: NULL context");
        std::lock_guard<std::mutex> lk(c->mu);
        VPC_ON_DEVICE(c->device);
        Slot& s = c->slots[ticket & 1];
        if (!s.busy || s.ticket != ticket) {
            if (ticket == 0 || ticket >= c->next_ticket) return fail("vpcsum_ctx_wait: unknown ticket %llu", (unsigned long long)ticket);
            return 0;   // already completed
        }
        return slot_finish(c, s);
    } VPC_CATCH("vpcsum_ctx_wait")
}

// vpcsum_ctx_verify_frames / _hsum: h_hsum NULL = no header sums
static int ctx_verify_frames(vpcsum_ctx_t* c, const uint8_t* h_arena, uint64_t arena_len, const uint64_t* h_frame_off,
                             const uint32_t* h_frame_len, uint32_t n, uint32_t* h_out, uint8_t* h_status,
                             vpcsum_hsum_t* h_hsum, uint64_t* ticket, const char* what) {
    if (!c || !ticket) return fail("%s: NULL context or ticket", what);
    if (n > c->max_pkts) return fail("%s: %u frames > capacity %u", what, n, c->max_pkts);
    if (n && (!h_arena || !h_frame_off || !h_frame_len || !h_status))
        return fail("%s: NULL arena, frame table or status", what);
    std::lock_guard<std::mutex> lk(c->mu);
    VPC_ON_DEVICE(c->device);
    uint8_t* base = n ? mapped_dev(c, h_arena, arena_len) : nullptr;
    if (n && !base) return fail("%s: the arena must be registered (vpcsum_ctx_register_arena)", what);
    const uint64_t t = c->next_ticket++;
    Slot& s = c->slots[t & 1];
    if (s.busy && slot_finish(c, s) != 0) return -1;
    if (h_hsum && n && !s.h_hs) {
        hipError_t e = hipHostMalloc((void**)&s.h_hs, (size_t)c->max_pkts * sizeof(vpcsum_hsum_t),
                                     hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&s.dh_hs, s.h_hs, 0);
        if (e != hipSuccess) {
            if (s.h_hs) (void)hipHostFree(s.h_hs);
            s.h_hs = s.dh_hs = nullptr;
            return hipfail(e, what);
        }
    }
    if (n && c->svc.on && n <= kSvcBatchMax) {
        // a small received batch: the service grid parses and verifies each frame
        // (kernels.hip svc_frame_packet), the sums into its own buffer (copied out only with h_out),
        // the header sums into its aux buffer
        if (svc_post_frames(c, s, t, h_arena, arena_len, base, h_frame_off, h_frame_len, nullptr, VPCSUM_F_IP | VPCSUM_F_L4,
                            n, h_out, h_status, VPCSUM_MODE_VERIFY, false, ticket, h_hsum != nullptr) != 0)
            return -1;
        s.user_hsum = h_hsum;
        return 0;
    }
    if (n) {
        // parse the frames where they lie (zero-copy), then verify the descriptors it built
        if (svc_quiesce(c) != 0) return -1;
        memcpy(s.h_foff, h_frame_off, (size_t)n * 8);
        memcpy(s.h_flen, h_frame_len, (size_t)n * 4);
        VPC_CHECK(launch_parse_ether(base, arena_len, s.dh_foff, s.dh_flen, n, VPCSUM_F_IP | VPCSUM_F_L4, s.d_desc,
                                     nullptr, nullptr, s.stream, nullptr, h_hsum ? s.dh_hs : nullptr),
                  "parse launch");
        // h_out NULL: the status bytes alone (the out words are 4 of the 5 result bytes a packet writes)
        VPC_CHECK(launch_csum(base, arena_len, s.d_desc, n, h_out ? s.dh_out : nullptr, s.dh_status, nullptr,
                              VPCSUM_MODE_VERIFY, nullptr, n <= kZeroCopyWaveTeams ? 12 : 0, 0, s.stream),
                  "verify launch");
    }
    VPC_CHECK(hipEventRecord(s.done, s.stream), "hipEventRecord");
    s.zero_copy = true;
    s.svc_seq = 0;
    s.kind = 0;
    s.busy = true;
    s.ticket = t;
    s.n = n;
    s.mode = VPCSUM_MODE_VERIFY;
    s.user_arena = nullptr;
    s.user_desc = nullptr;
    s.user_out = h_out;
    s.user_status = h_status;
    s.user_hsum = n ? h_hsum : nullptr;
    *ticket = t;
    return 0;
}

int vpcsum_ctx_verify_frames(vpcsum_ctx_t* c, const uint8_t* h_arena, uint64_t arena_len, const uint64_t* h_frame_off,
                             const uint32_t* h_frame_len, uint32_t n, uint32_t* h_out, uint8_t* h_status,
                             uint64_t* ticket) {
    try {
        return ctx_verify_frames(c, h_arena, arena_len, h_frame_off, h_frame_len, n, h_out, h_status, nullptr, ticket,
                                 "vpcsum_ctx_verify_frames");
    } VPC_CATCH("vpcsum_ctx_verify_frames")
}

int vpcsum_ctx_verify_frames_hsum(vpcsum_ctx_t* c, const uint8_t* h_arena, uint64_t arena_len, const uint64_t* h_frame_off,
                                  const uint32_t* h_frame_len, uint32_t n, uint32_t* h_out, uint8_t* h_status,
                                  vpcsum_hsum_t* h_hsum, uint64_t* ticket) {
    try {
        if (n && !h_hsum) return fail("vpcsum_ctx_verify_frames_hsum: NULL header-sum array");
        return ctx_verify_frames(c, h_arena, arena_len, h_frame_off, h_frame_len, n, h_out, h_status, h_hsum, ticket,
                                 "vpcsum_ctx_verify_frames_hsum");
    } VPC_CATCH("vpcsum_ctx_verify_frames_hsum")
}

int vpcsum_ctx_egress_frames(vpcsum_ctx_t* c, uint8_t* h_arena, uint64_t arena_len, const uint64_t* h_frame_off,
                             const uint32_t* h_frame_len, const uint8_t* h_frame_flags, uint32_t n, uint32_t* h_out,
                             uint8_t* h_status, uint64_t* ticket) {
    try {
        if (!c || !ticket) return fail("vpcsum_ctx_egress_frames: NULL context or ticket");
        if (n > c->max_pkts) return fail("vpcsum_ctx_egress_frames: %u frames > capacity %u", n, c->max_pkts);
        if (n && (!h_arena || !h_frame_off || !h_frame_len || !h_frame_flags))
            return fail("vpcsum_ctx_egress_frames: NULL arena, frame table or flags");
        std::lock_guard<std::mutex> lk(c->mu);
        VPC_ON_DEVICE(c->device);
        uint8_t* base = n ? mapped_dev(c, h_arena, arena_len) : nullptr;
        if (n && !base) return fail("vpcsum_ctx_egress_frames: the arena must be registered (vpcsum_ctx_register_arena)");
        const uint64_t t = c->next_ticket++;
        Slot& s = c->slots[t & 1];
        if (s.busy && slot_finish(c, s) != 0) return -1;
        if (n && c->svc.on && n <= kSvcBatchMax) {
            // a small flush: the service grid parses and sums each frame (kernels.hip svc_frame_packet)
            return svc_post_frames(c, s, t, h_arena, arena_len, base, h_frame_off, h_frame_len, h_frame_flags, 0, n, h_out,
                                   h_status, VPCSUM_MODE_WRITE, false, ticket);
        }
        if (n) {
            if (svc_quiesce(c) != 0) return -1;
            // the frames' own flags ride in the status staging: the parse reads them before the
            // checksum kernel, later on the same stream, overwrites them with the statuses
            memcpy(s.h_foff, h_frame_off, (size_t)n * 8);
            memcpy(s.h_flen, h_frame_len, (size_t)n * 4);
            memcpy(s.h_status, h_frame_flags, n);
            VPC_CHECK(launch_parse_ether(base, arena_len, s.dh_foff, s.dh_flen, n, 0, s.d_desc, nullptr, nullptr, s.stream,
                                         s.dh_status),
                      "parse launch");
            VPC_CHECK(launch_csum(base, arena_len, s.d_desc, n, s.dh_out, s.dh_status, nullptr, VPCSUM_MODE_COMPUTE, base,
                                  n <= kZeroCopyWaveTeams ? 12 : 0, 0, s.stream),
                      "checksum launch");
        }
        VPC_CHECK(hipEventRecord(s.done, s.stream), "hipEventRecord");
        s.zero_copy = true;
        s.svc_seq = 0;
        s.kind = 0;
        s.busy = true;
        s.ticket = t;
        s.n = n;
        s.mode = VPCSUM_MODE_WRITE;
        s.user_arena = nullptr;   // written in place through the mapping
        s.user_desc = nullptr;
        s.user_out = h_out;
        s.user_status = h_status;
        *ticket = t;
        return 0;
    } VPC_CATCH("vpcsum_ctx_egress_frames")
}

int vpcsum_ctx_parse_frames(vpcsum_ctx_t* c, const uint8_t* h_arena, uint64_t arena_len, const uint64_t* h_frame_off,
                            const uint32_t* h_frame_len, uint32_t n, vpcsum_desc_t* h_desc, uint8_t* h_status,
                            vpcsum_tuple_t* h_tuples, uint64_t* ticket) {
    try {
        if (!c || !ticket) return fail("vpcsum_ctx_parse_frames: NULL context or ticket");
        if (n > c->max_pkts) return fail("vpcsum_ctx_parse_frames: %u frames > capacity %u", n, c->max_pkts);
        if (n && (!h_arena || !h_frame_off || !h_frame_len)) return fail("vpcsum_ctx_parse_frames: NULL arena or frame table");
        std::lock_guard<std::mutex> lk(c->mu);
        VPC_ON_DEVICE(c->device);
        uint8_t* base = n ? mapped_dev(c, h_arena, arena_len) : nullptr;
        if (n && !base) return fail("vpcsum_ctx_parse_frames: the arena must be registered (vpcsum_ctx_register_arena)");
        const uint64_t t = c->next_ticket++;
        Slot& s = c->slots[t & 1];
        if (s.busy && slot_finish(c, s) != 0) return -1;
        if (!s.h_tu) {
            hipError_t e = hipHostMalloc((void**)&s.h_tu, (size_t)c->max_pkts * sizeof(vpcsum_tuple_t),
                                         hipHostMallocMapped | hipHostMallocCoherent);
            if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&s.dh_tu, s.h_tu, 0);
            if (e != hipSuccess) {
                if (s.h_tu) (void)hipHostFree(s.h_tu);
                s.h_tu = s.dh_tu = nullptr;
                return hipfail(e, "vpcsum_ctx_parse_frames allocation");
            }
        }
        if (n && c->svc.on && n <= kSvcBatchMax) {
            // a small received batch: the service grid parses each frame (kernels.hip svc_frame_packet)
            if (svc_post_frames(c, s, t, h_arena, arena_len, base, h_frame_off, h_frame_len, nullptr,
                                VPCSUM_F_IP | VPCSUM_F_L4, n, nullptr, h_status, 0, true, ticket) != 0)
                return -1;
            s.kind = 2;
            s.user_desc_out = h_desc;
            s.user_tuples = h_tuples;
            return 0;
        }
        if (n) {
            // parsed where the frames lie (zero-copy); results straight into the pinned staging
            if (svc_quiesce(c) != 0) return -1;
            memcpy(s.h_foff, h_frame_off, (size_t)n * 8);
            memcpy(s.h_flen, h_frame_len, (size_t)n * 4);
            VPC_CHECK(launch_parse_ether(base, arena_len, s.dh_foff, s.dh_flen, n, VPCSUM_F_IP | VPCSUM_F_L4, s.dh_desc,
                                         s.dh_status, s.dh_tu, s.stream),
                      "parse launch");
        }
        VPC_CHECK(hipEventRecord(s.done, s.stream), "hipEventRecord");
        s.zero_copy = true;
        s.svc_seq = 0;
        s.kind = 2;
        s.busy = true;
        s.ticket = t;
        s.n = n;
        s.mode = 0;
        s.user_arena = nullptr;
        s.user_desc = nullptr;
        s.user_out = nullptr;
        s.user_status = h_status;
        s.user_desc_out = h_desc;
        s.user_tuples = h_tuples;
        *ticket = t;
        return 0;
    } VPC_CATCH("vpcsum_ctx_parse_frames")
}

int vpcsum_ctx_nat_submit(vpcsum_ctx_t* c, uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc,
                          const vpcsum_nat_t* h_rw, uint32_t n, uint8_t* h_status, uint32_t nat_mode, uint64_t* ticket) {
    try {
        if (!c || !ticket) return fail("vpcsum_ctx_nat_submit: NULL context or ticket");
        if (n > c->max_pkts) return fail("vpcsum_ctx_nat_submit: %u packets > capacity %u", n, c->max_pkts);
        if (n && (!h_arena || !h_desc || !h_rw)) return fail("vpcsum_ctx_nat_submit: NULL arena, descriptors or rewrites");
        if (nat_mode & ~(VPCSUM_NAT_STRICT_JAVA | 0x100u)) return fail("vpcsum_ctx_nat_submit: bad nat_mode 0x%x", nat_mode);
        std::lock_guard<std::mutex> lk(c->mu);
        VPC_ON_DEVICE(c->device);
        const uint64_t t = c->next_ticket++;
        Slot& s = c->slots[t & 1];
        if (s.busy && slot_finish(c, s) != 0) return -1;
        if (slot_rw_alloc(c, s, "vpcsum_ctx_nat_submit") != 0) return -1;
        uint64_t lo = UINT64_MAX, hi = 0;
        for (uint32_t i = 0; i < n; ++i) {
            const vpcsum_desc_t& d = h_desc[i];
            if (d.l3_off > arena_len || d.l3_len > arena_len - d.l3_off) continue;   // the kernel flags it BAD
            lo = std::min(lo, d.l3_off);
            hi = std::max(hi, d.l3_off + d.l3_len);
        }
        if (lo == UINT64_MAX) { lo = 0; hi = 0; }
        lo &= ~(uint64_t)15;
        uint8_t* dev_arena = hi > lo ? mapped_dev(c, h_arena + lo, hi - lo) : nullptr;
        memcpy(s.h_rw, h_rw, (size_t)n * sizeof(vpcsum_nat_t));
        if (dev_arena) {
            // the frames live in a registered (page-locked, mapped) arena: rewritten where they lie
            if (svc_quiesce(c) != 0) return -1;
            memcpy(s.h_desc, h_desc, (size_t)n * sizeof(vpcsum_desc_t));
            if (n && nat_run(dev_arena - lo, arena_len, s.dh_desc, s.dh_rw, 1, n, s.dh_status, nat_mode, s.stream) != 0)
                return -1;
            s.zero_copy = true;
        } else {
            // staged: each packet's 16-B blocks gathered into the pinned staging, rewritten on the
            // device, and the whole gathered batch copied back (the headers return at wait)
            uint64_t pos = 0;
            for (uint32_t i = 0; i < n; ++i) {
                const vpcsum_desc_t& d = h_desc[i];
                s.h_desc[i] = d;
                if (d.l3_off > arena_len || d.l3_len > arena_len - d.l3_off) { s.h_desc[i].l3_off = UINT64_MAX; continue; }
                const uint64_t a0 = d.l3_off & ~(uint64_t)15;
                const uint64_t a1 = std::min<uint64_t>((d.l3_off + d.l3_len + 15) & ~(uint64_t)15, arena_len);
                if (pos + (a1 - a0) > c->max_arena) return fail("vpcsum_ctx_nat_submit: batch exceeds the staging capacity");
                memcpy(s.h_arena + pos, h_arena + a0, a1 - a0);
                s.h_desc[i].l3_off = pos + (d.l3_off - a0);
                pos += (a1 - a0 + 15) & ~(uint64_t)15;
            }
            if (n) {
                VPC_CHECK(hipMemcpyAsync(s.d_desc, s.h_desc, (size_t)n * sizeof(vpcsum_desc_t), hipMemcpyHostToDevice, s.stream),
                          "H2D descriptors");
                VPC_CHECK(hipMemcpyAsync(s.d_rw, s.h_rw, (size_t)n * sizeof(vpcsum_nat_t), hipMemcpyHostToDevice, s.stream),
                          "H2D rewrites");
                if (pos) VPC_CHECK(hipMemcpyAsync(s.d_arena, s.h_arena, pos, hipMemcpyHostToDevice, s.stream), "H2D frames");
                if (nat_run(s.d_arena, pos, s.d_desc, s.d_rw, 1, n, s.d_status, nat_mode, s.stream) != 0) return -1;
                if (pos) VPC_CHECK(hipMemcpyAsync(s.h_arena, s.d_arena, pos, hipMemcpyDeviceToHost, s.stream), "D2H frames");
                VPC_CHECK(hipMemcpyAsync(s.h_status, s.d_status, n, hipMemcpyDeviceToHost, s.stream), "D2H status");
            }
            s.zero_copy = false;
        }
        VPC_CHECK(hipEventRecord(s.done, s.stream), "hipEventRecord");
        s.kind = 1;
        s.svc_seq = 0;
        s.busy = true;
        s.ticket = t;
        s.n = n;
        s.mode = nat_mode;
        s.user_arena = h_arena;
        s.user_desc = h_desc;
        s.user_out = nullptr;
        s.user_status = h_status;
        *ticket = t;
        return 0;
    } VPC_CATCH("vpcsum_ctx_nat_submit")
}

int vpcsum_ctx_pipeline(vpcsum_ctx_t* c, uint8_t* h_arena, uint32_t stride, uint32_t copy_bytes,
                        const vpcsum_desc_t* h_desc, uint32_t n, uint32_t* h_out, uint32_t mode, uint32_t chunks) {
    try {
        if (!c || !h_arena || !h_desc || !h_out) return fail("vpcsum_ctx_pipeline: NULL argument");
        if (chunks == 0) chunks = 1;
        if (copy_bytes > stride) return fail("vpcsum_ctx_pipeline: copy_bytes > stride");
        if (mode & ~(VPCSUM_MODE_VERIFY | VPCSUM_MODE_WRITE)) return fail("vpcsum_ctx_pipeline: bad mode");
        std::lock_guard<std::mutex> lk(c->mu);
        VPC_ON_DEVICE(c->device);
        for (auto& s : c->slots)
            if (s.busy && slot_finish(c, s) != 0) return -1;
        const uint32_t per = (n + chunks - 1) / chunks;
        if (per > c->max_pkts || (uint64_t)per * stride > c->max_arena)
            return fail("vpcsum_ctx_pipeline: chunk of %u frames exceeds context capacity", per);
        const bool pinned = is_registered(c, h_arena, (uint64_t)n * stride);
        if (!pinned) return fail("vpcsum_ctx_pipeline: host arena must be registered (vpcsum_ctx_register_arena)");
        // MODE_WRITE: the kernels read the device copy and store the checksum fields straight into the
        // host frames through the registered arena's mapping (2-B posted PCIe writes), so the frames
        // need no copy back
        uint8_t* w = nullptr;
        if (mode & VPCSUM_MODE_WRITE) {
            w = mapped_dev(c, h_arena, (uint64_t)n * stride);
            if (!w) return fail("vpcsum_ctx_pipeline: MODE_WRITE needs the arena registered with this context");
        }
        const bool desc_pinned = is_registered(c, (const uint8_t*)h_desc, (uint64_t)n * sizeof(vpcsum_desc_t));
        const bool out_pinned = is_registered(c, (const uint8_t*)h_out, (uint64_t)n * 4);
        if (!desc_pinned || !out_pinned) return fail("vpcsum_ctx_pipeline: descriptors and out must be registered");
        // each chunk's device view starts at frame i0, and only the first copy_bytes of every frame
        // are copied: a descriptor must lie inside the copied part of a frame of its own chunk
        // (below the view it would address memory before the device slot)
        for (uint32_t i = 0; i < n; ++i) {
            const uint64_t i0 = (uint64_t)(i / per) * per;
            const uint64_t off = h_desc[i].l3_off;
            if (off < i0 * stride || off >= (uint64_t)n * stride || off % stride + h_desc[i].l3_len > copy_bytes)
                return fail("vpcsum_ctx_pipeline: descriptor %u [%llu, +%u) outside the copied frames", i,
                            (unsigned long long)off, (unsigned)h_desc[i].l3_len);
        }
        // a failure after some chunks were queued drains both streams before it returns: the queued
        // copies and in-place writes land in the caller's registered buffers
    #define VPC_CHECK_DRAIN(expr, what)                                                  \
        do {                                                                             \
            hipError_t e__ = (expr);                                                     \
            if (e__ != hipSuccess) {                                                     \
                const int rc__ = hipfail(e__, what);                                     \
                for (auto& q__ : c->slots) (void)hipStreamSynchronize(q__.stream);       \
                return rc__;                                                             \
            }                                                                            \
        } while (0)
        for (uint32_t k = 0; k < chunks; ++k) {
            const uint32_t i0 = k * per;
            if (i0 >= n) break;
            const uint32_t m = std::min(per, n - i0);
            Slot& s = c->slots[k & 1];
            // descriptors of this chunk address the device slot as frame (i - i0) * stride: the
            // caller's descriptors are relative to frame i0 once i0 * stride is subtracted
            VPC_CHECK_DRAIN(hipMemcpyAsync(s.d_desc, h_desc + i0, (size_t)m * sizeof(vpcsum_desc_t), hipMemcpyHostToDevice,
                                     s.stream),
                      "pipeline H2D desc");
            VPC_CHECK_DRAIN(hipMemcpy2DAsync(s.d_arena, stride, h_arena + (uint64_t)i0 * stride, stride, copy_bytes, m,
                                       hipMemcpyHostToDevice, s.stream),
                      "pipeline H2D frames");
            VPC_CHECK_DRAIN(launch_csum(s.d_arena - (uint64_t)i0 * stride, (uint64_t)(i0 + m) * stride, s.d_desc, m, s.d_out,
                                  nullptr, nullptr, mode & VPCSUM_MODE_VERIFY, w, 0, 0, s.stream),
                      "pipeline launch");
            VPC_CHECK_DRAIN(hipMemcpyAsync(h_out + i0, s.d_out, (size_t)m * 4, hipMemcpyDeviceToHost, s.stream), "pipeline D2H");
        }
    #undef VPC_CHECK_DRAIN
        hipError_t es = hipSuccess;   // both streams are joined, the first error is reported
        for (auto& s : c->slots) {
            const hipError_t e2 = hipStreamSynchronize(s.stream);
            if (es == hipSuccess) es = e2;
        }
        VPC_CHECK(es, "pipeline sync");
        return 0;
    } VPC_CATCH("vpcsum_ctx_pipeline")
}

// ------------------------------------------------------------------------------------------
// Device groups (SURVEY.md §8(b) vpcsum_init(dev_mask), §8(e)): one context per GPU; a host batch
// is cut into contiguous descriptor ranges of nearly equal byte totals, one per GPU, each run by
// its own context (own streams, own staging); wait joins them.  No data crosses devices.
// ------------------------------------------------------------------------------------------
}  // extern "C"

struct vpcsum_group {
    std::vector<vpcsum_ctx*> ctx;
    struct Reg { uint8_t* host; uint8_t* key; };
    std::vector<Reg> reg;          // arenas the group registered: their page-lock references (portable
                                   // locks: every device maps them), one per arena
    uint64_t next_ticket = 1;
    struct Pending { uint64_t ticket = 0; std::vector<uint64_t> sub; };
    Pending slots[2];
    std::mutex mu;
};

static int vpcsum_group_wait_locked(vpcsum_group* g, vpcsum_group::Pending& slot) {
    int rc = 0;
    for (size_t d = 0; d < slot.sub.size(); ++d)
        if (vpcsum_ctx_wait(g->ctx[d], slot.sub[d]) != 0) rc = -1;   // every device joins, first error kept
    slot.ticket = 0;
    return rc;
}

extern "C" {

int vpcsum_group_create_list(const int* devices, int ndev, uint64_t max_arena_bytes, uint32_t max_pkts,
                             vpcsum_group_t** out) {
    try {
        if (!out || !devices || ndev <= 0 || ndev > 64) return fail("vpcsum_group_create_list: bad argument");
        std::unique_ptr<vpcsum_group> g(new vpcsum_group());
        g->ctx.reserve(ndev);   // the push_backs below cannot throw once a context exists
        for (int i = 0; i < ndev; ++i) {
            vpcsum_ctx_t* c = nullptr;
            if (vpcsum_ctx_create(devices[i], max_arena_bytes, max_pkts, &c) != 0) {
                char e[1024];
                snprintf(e, sizeof(e), "%s", g_err);
                vpcsum_group_destroy(g.release());
                return fail("%s", e);
            }
            g->ctx.push_back(c);
        }
        *out = g.release();
        return 0;
    } VPC_CATCH("vpcsum_group_create_list")
}

int vpcsum_group_create(uint64_t dev_mask, uint64_t max_arena_bytes, uint32_t max_pkts, vpcsum_group_t** out) {
    try {
        int n = 0;
        VPC_CHECK(hipGetDeviceCount(&n), "hipGetDeviceCount");
        std::vector<int> devs;
        for (int d = 0; d < 64 && d < n; ++d)
            if (dev_mask >> d & 1) devs.push_back(d);
        if (devs.empty() || (n < 64 && (dev_mask >> n) != 0))
            return fail("vpcsum_group_create: mask 0x%llx names no device or one beyond the %d present",
                        (unsigned long long)dev_mask, n);
        return vpcsum_group_create_list(devs.data(), (int)devs.size(), max_arena_bytes, max_pkts, out);
    } VPC_CATCH("vpcsum_group_create")
}

int vpcsum_group_destroy(vpcsum_group_t* g) {
    try {
        if (!g) return 0;
        int rc = 0;
        {
            // the group's batches in flight complete first (results into the callers' buffers);
            // vpcsum_ctx_destroy does the same for anything submitted to a context directly
            std::lock_guard<std::mutex> lk(g->mu);
            for (auto& slot : g->slots)
                if (slot.ticket && vpcsum_group_wait_locked(g, slot) != 0) rc = -1;
        }
        const int dev0 = g->ctx.empty() ? 0 : g->ctx[0]->device;   // the contexts are gone below
        for (auto* c : g->ctx)
            if (vpcsum_ctx_destroy(c) != 0) rc = -1;
        if (!g->reg.empty()) {
            DeviceScope on_dev(dev0);
            for (auto& r : g->reg)
                if (hostlock_release(r.key, "vpcsum_group_destroy") != 0) rc = -1;
        }
        delete g;
        return rc;
    } VPC_CATCH("vpcsum_group_destroy")
}

int vpcsum_group_register_arena(vpcsum_group_t* g, void* h_arena, uint64_t len) {
    try {
        if (!g || !h_arena || len == 0) return fail("vpcsum_group_register_arena: bad argument");
        std::lock_guard<std::mutex> lk(g->mu);
        VPC_ON_DEVICE(g->ctx[0]->device);
        // the bookkeeping may throw: make room before anything is pinned or mapped
        g->reg.reserve(g->reg.size() + 1);
        for (auto* c : g->ctx) {
            std::lock_guard<std::mutex> lc(c->mu);
            c->registered.reserve(c->registered.size() + 1);
        }
        for (auto& r : g->reg)
            if (r.host == (uint8_t*)h_arena) return fail("vpcsum_group_register_arena: %p is registered already", h_arena);
        uint8_t* key = nullptr;
        if (hostlock_acquire((uint8_t*)h_arena, len, &key, "vpcsum_group_register_arena") != 0) return -1;
        for (size_t i = 0; i < g->ctx.size(); ++i) {
            vpcsum_ctx* c = g->ctx[i];
            std::lock_guard<std::mutex> lc(c->mu);
            DeviceScope on_dev(c->device);
            void* dev = nullptr;
            hipError_t e = on_dev.err;
            if (e == hipSuccess) e = hipHostGetDevicePointer(&dev, h_arena, 0);
            if (e != hipSuccess) {
                // roll back: no context keeps a mapping of an arena the group failed to register, so
                // a retry starts from scratch
                for (size_t q = 0; q < i; ++q) {
                    std::lock_guard<std::mutex> lq(g->ctx[q]->mu);
                    auto& rq = g->ctx[q]->registered;
                    for (size_t k = rq.size(); k-- > 0;)
                        if (rq[k].host == (uint8_t*)h_arena && !rq[k].key) rq.erase(rq.begin() + k);
                }
                (void)hostlock_release(key, "vpcsum_group_register_arena");
                return hipfail(e, "vpcsum_group_register_arena: device mapping");
            }
            c->registered.push_back({(uint8_t*)h_arena, len, (uint8_t*)dev, nullptr});
        }
        g->reg.push_back({(uint8_t*)h_arena, key});
        return 0;
    } VPC_CATCH("vpcsum_group_register_arena")
}

int vpcsum_group_unregister_arena(vpcsum_group_t* g, void* h_arena) {
    try {
        if (!g || !h_arena) return fail("vpcsum_group_unregister_arena: bad argument");
        std::lock_guard<std::mutex> lk(g->mu);
        auto it = std::find_if(g->reg.begin(), g->reg.end(),
                               [&](const vpcsum_group::Reg& r) { return r.host == (uint8_t*)h_arena; });
        if (it == g->reg.end()) return fail("vpcsum_group_unregister_arena: arena not registered");
        // Two phases, so that a failure leaves the registration whole and a retry can succeed:
        // (1) every context finishes its zero-copy batches -- the only step that can fail, and
        // nothing has been dropped yet; (2) every context forgets the mapping (the contexts do not own
        // the page-lock) and the group unpins the arena.
        for (auto* c : g->ctx) {
            std::lock_guard<std::mutex> lc(c->mu);
            DeviceScope on_dev(c->device);
            if (on_dev.err != hipSuccess) return hipfail(on_dev.err, "hipSetDevice");
            if (ctx_quiesce_zero_copy(c) != 0) return -1;
        }
        for (auto* c : g->ctx) {
            std::lock_guard<std::mutex> lc(c->mu);
            auto& r = c->registered;
            for (size_t k = r.size(); k-- > 0;)
                if (r[k].host == (uint8_t*)h_arena && !r[k].key) r.erase(r.begin() + k);
        }
        uint8_t* key = it->key;
        g->reg.erase(it);
        VPC_ON_DEVICE(g->ctx[0]->device);
        return hostlock_release(key, "vpcsum_group_unregister_arena");
    } VPC_CATCH("vpcsum_group_unregister_arena")
}

}  // extern "C"

// Byte-balanced contiguous cuts of a host batch over the group's contexts (shard_by_bytes in
// vproxy_amd/shard.py); submit(d, a, b, &ticket) hands range [a, b) to context d.  A range a
// context refuses fails the group submit only after the ranges already submitted have finished:
// they write into the caller's buffers, which the caller may free once the error is back.
template <class Submit>
static int group_submit_ranges(vpcsum_group* g, const vpcsum_desc_t* h_desc, uint32_t n, uint64_t* ticket,
                               Submit submit) {
    const uint64_t t = g->next_ticket++;
    auto& slot = g->slots[t & 1];
    if (slot.ticket && vpcsum_group_wait_locked(g, slot) != 0) return -1;
    const size_t k = g->ctx.size();
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) total += h_desc[i].l3_len;
    std::vector<uint32_t> cut(k + 1, n);
    cut[0] = 0;
    uint64_t acc = 0;
    size_t r = 1;
    for (uint32_t i = 0; i < n && r < k; ++i) {
        acc += h_desc[i].l3_len;
        while (r < k && acc * k >= total * r) cut[r++] = i + 1;
    }
    slot.sub.assign(k, 0);
    for (size_t d = 0; d < k; ++d) {
        const uint32_t a = cut[d], b = std::max(cut[d], cut[d + 1]);
        if (submit(d, a, b, &slot.sub[d]) != 0) {
            char e[1024];
            snprintf(e, sizeof(e), "%s", g_err);
            for (size_t q = 0; q < d; ++q) (void)vpcsum_ctx_wait(g->ctx[q], slot.sub[q]);
            slot.sub.clear();
            return fail("%s", e);
        }
    }
    slot.ticket = t;
    *ticket = t;
    return 0;
}

extern "C" {

int vpcsum_group_submit(vpcsum_group_t* g, uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc,
                        uint32_t n, uint32_t* h_out, uint8_t* h_status, uint32_t mode, uint64_t* ticket) {
    try {
        if (!g || !ticket) return fail("vpcsum_group_submit: NULL group or ticket");
        if (n && (!h_arena || !h_desc)) return fail("vpcsum_group_submit: NULL arena or descriptors");
        std::lock_guard<std::mutex> lk(g->mu);
        return group_submit_ranges(g, h_desc, n, ticket, [&](size_t d, uint32_t a, uint32_t b, uint64_t* t) {
            return vpcsum_ctx_submit(g->ctx[d], h_arena, arena_len, h_desc + a, b - a, h_out ? h_out + a : nullptr,
                                     h_status ? h_status + a : nullptr, mode, t);
        });
    } VPC_CATCH("vpcsum_group_submit")
}

int vpcsum_group_nat_submit(vpcsum_group_t* g, uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc,
                            const vpcsum_nat_t* h_rw, uint32_t n, uint8_t* h_status, uint32_t nat_mode,
                            uint64_t* ticket) {
    try {
        if (!g || !ticket) return fail("vpcsum_group_nat_submit: NULL group or ticket");
        if (n && (!h_arena || !h_desc || !h_rw)) return fail("vpcsum_group_nat_submit: NULL arena, descriptors or rewrites");
        std::lock_guard<std::mutex> lk(g->mu);
        return group_submit_ranges(g, h_desc, n, ticket, [&](size_t d, uint32_t a, uint32_t b, uint64_t* t) {
            return vpcsum_ctx_nat_submit(g->ctx[d], h_arena, arena_len, h_desc + a, h_rw + a, b - a,
                                         h_status ? h_status + a : nullptr, nat_mode, t);
        });
    } VPC_CATCH("vpcsum_group_nat_submit")
}

int vpcsum_group_submit_pre(vpcsum_group_t* g, uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc,
                            const void* h_pre, uint32_t pre_fmt, uint32_t n, uint32_t* h_out, uint8_t* h_status,
                            uint32_t mode, uint64_t* ticket) {
    try {
        if (!g || !ticket) return fail("vpcsum_group_submit_pre: NULL group or ticket");
        if (n && (!h_arena || !h_desc || !h_pre)) return fail("vpcsum_group_submit_pre: NULL arena, descriptors or pre-images");
        if (pre_fmt > VPCSUM_PRE_FMT_PRE) return fail("vpcsum_group_submit_pre: bad pre_fmt %u", pre_fmt);
        const size_t esz = pre_fmt == VPCSUM_PRE_FMT_PRE ? sizeof(vpcsum_pre_t) : sizeof(vpcsum_pre4_t);
        std::lock_guard<std::mutex> lk(g->mu);
        return group_submit_ranges(g, h_desc, n, ticket, [&](size_t d, uint32_t a, uint32_t b, uint64_t* t) {
            return vpcsum_ctx_submit_pre(g->ctx[d], h_arena, arena_len, h_desc + a, (const uint8_t*)h_pre + a * esz, pre_fmt,
                                         b - a, h_out ? h_out + a : nullptr, h_status ? h_status + a : nullptr, mode, t);
        });
    } VPC_CATCH("vpcsum_group_submit_pre")
}

int vpcsum_group_wait(vpcsum_group_t* g, uint64_t ticket) {
    try {
        if (!g) return fail("vpcsum_group_wait: NULL group");
        std::lock_guard<std::mutex> lk(g->mu);
        auto& slot = g->slots[ticket & 1];
        if (slot.ticket != ticket) {
            if (ticket == 0 || ticket >= g->next_ticket) return fail("vpcsum_group_wait: unknown ticket %llu", (unsigned long long)ticket);
            return 0;   // already completed
        }
        return vpcsum_group_wait_locked(g, slot);
    } VPC_CATCH("vpcsum_group_wait")
}

// SURVEY.md §8(b)'s entry points over one process-wide device group (vpcsum_init creates it).
// Every call on the group holds a shared lock for its whole duration and vpcsum_init /
// vpcsum_shutdown an exclusive one: a shutdown on one thread waits for the submits and waits in
// flight on others and completes every batch still pending (vpcsum_group_destroy: results into
// the callers' buffers); a call after it fails with "vpcsum_init first" (never a freed group).
// A handle carries the generation of the group that issued it (bits 48..63; each vpcsum_init
// starts a new one), so that a handle from before a shutdown is refused by the next group instead
// of naming one of its tickets.
}  // extern "C"

static std::shared_mutex g_default_rw;
static vpcsum_group* g_default = nullptr;
static uint64_t g_default_gen = 0;   // generation of g_default (written under the exclusive lock)
constexpr int kGenShift = 48;
constexpr uint64_t kTicketMask = (1ull << kGenShift) - 1;

template <class F>
static int with_default_group(const char* what, F f) {
    std::shared_lock<std::shared_mutex> lk(g_default_rw);
    if (!g_default) return fail("%s: vpcsum_init first", what);
    return f(g_default);
}

// a submit's group ticket -> the handle the caller gets
static int default_handle(int rc, uint64_t* handle) {
    if (rc == 0 && handle) *handle = (*handle & kTicketMask) | (g_default_gen << kGenShift);
    return rc;
}

extern "C" {

int vpcsum_init(uint64_t dev_mask, uint64_t max_arena_bytes, uint32_t max_pkts) {
    try {
        std::unique_lock<std::shared_mutex> lk(g_default_rw);
        if (g_default) return fail("vpcsum_init: already initialised (vpcsum_shutdown first)");
        vpcsum_group_t* g = nullptr;
        if (vpcsum_group_create(dev_mask, max_arena_bytes, max_pkts, &g) != 0) return -1;
        g_default = g;
        g_default_gen = (g_default_gen + 1) & 0xffff ? (g_default_gen + 1) & 0xffff : 1;
        return 0;
    } VPC_CATCH("vpcsum_init")
}

int vpcsum_shutdown(void) {
    try {
        std::unique_lock<std::shared_mutex> lk(g_default_rw);
        vpcsum_group_t* g = g_default;
        g_default = nullptr;
        return vpcsum_group_destroy(g);
    } VPC_CATCH("vpcsum_shutdown")
}

int vpcsum_register_arena(void* h_arena, uint64_t len) {
    try {
        return with_default_group("vpcsum_register_arena",
                                  [&](vpcsum_group* g) { return vpcsum_group_register_arena(g, h_arena, len); });
    } VPC_CATCH("vpcsum_register_arena")
}

int vpcsum_batch_submit(uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc, uint32_t n,
                        uint32_t* h_out, uint8_t* h_status, uint32_t mode, uint64_t* handle) {
    try {
        return with_default_group("vpcsum_batch_submit", [&](vpcsum_group* g) {
            return default_handle(vpcsum_group_submit(g, h_arena, arena_len, h_desc, n, h_out, h_status, mode, handle),
                                  handle);
        });
    } VPC_CATCH("vpcsum_batch_submit")
}

int vpcsum_batch_submit_pre(uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc, const void* h_pre,
                            uint32_t pre_fmt, uint32_t n, uint32_t* h_out, uint8_t* h_status, uint32_t mode,
                            uint64_t* handle) {
    try {
        return with_default_group("vpcsum_batch_submit_pre", [&](vpcsum_group* g) {
            return default_handle(vpcsum_group_submit_pre(g, h_arena, arena_len, h_desc, h_pre, pre_fmt, n, h_out, h_status,
                                                          mode, handle),
                                  handle);
        });
    } VPC_CATCH("vpcsum_batch_submit_pre")
}

int vpcsum_nat_submit(uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc, const vpcsum_nat_t* h_rw,
                      uint32_t n, uint8_t* h_status, uint32_t nat_mode, uint64_t* handle) {
    try {
        return with_default_group("vpcsum_nat_submit", [&](vpcsum_group* g) {
            return default_handle(vpcsum_group_nat_submit(g, h_arena, arena_len, h_desc, h_rw, n, h_status, nat_mode, handle),
                                  handle);
        });
    } VPC_CATCH("vpcsum_nat_submit")
}

int vpcsum_batch_wait(uint64_t handle) {
    try {
        return with_default_group("vpcsum_batch_wait", [&](vpcsum_group* g) {
            if ((handle >> kGenShift) != g_default_gen)
                return fail("vpcsum_batch_wait: handle 0x%llx is from before vpcsum_shutdown (its batch was completed "
                            "by the shutdown)",
                            (unsigned long long)handle);
            return vpcsum_group_wait(g, handle & kTicketMask);
        });
    } VPC_CATCH("vpcsum_batch_wait")
}

// ------------------------------------------------------------------------------------------
// PNI entry points
// ------------------------------------------------------------------------------------------
// The exception travels in env->ex as PNIThrowException stores it (pni.h:74-80); errno_ carries
// EINVAL for argument errors, ENOMEM when host memory ran out and EIO for failures of the device
// runtime (PNIStoreErrno's slot, pni.h:86-89), so Java code that inspects it sees a meaningful value.
static int pni_throw(void* env, const char* type) {
    PNIException_vpcsum* ex = (PNIException_vpcsum*)env;
    ex->type = (char*)type;
    strncpy(ex->message, g_err, sizeof(ex->message));
    ex->message[sizeof(ex->message) - 1] = '\0';
    ex->errno_ = strcmp(type, "java.lang.IllegalArgumentException") == 0 ? EINVAL
                 : strcmp(type, "java.lang.OutOfMemoryError") == 0       ? ENOMEM
                                                                         : EIO;
    return -1;
}

int Java_io_vproxy_vpcsum_VPCsum_create(PNIEnv_vpcsum_long* env, int32_t device, int64_t maxArena, int32_t maxPkts) {
    try {
        if (maxArena <= 0 || maxPkts <= 0) {
            fail("maxArena and maxPkts must be positive");
            return pni_throw(env, "java.lang.IllegalArgumentException");
        }
        vpcsum_ctx_t* c = nullptr;
        if (vpcsum_ctx_create(device, (uint64_t)maxArena, (uint32_t)maxPkts, &c) != 0) return pni_throw(env, "java.io.IOException");
        env->return_ = (int64_t)(intptr_t)c;
        return 0;
    } VPC_CATCH_PNI("Java_io_vproxy_vpcsum_VPCsum_create")
}

int Java_io_vproxy_vpcsum_VPCsum_registerArena(PNIEnv_vpcsum_void* env, int64_t ctx, void* arena, int64_t len) {
    try {
        if (len <= 0) {
            fail("len must be positive");
            return pni_throw(env, "java.lang.IllegalArgumentException");
        }
        if (vpcsum_ctx_register_arena((vpcsum_ctx_t*)(intptr_t)ctx, arena, (uint64_t)len) != 0)
            return pni_throw(env, "java.io.IOException");
        return 0;
    } VPC_CATCH_PNI("Java_io_vproxy_vpcsum_VPCsum_registerArena")
}

int Java_io_vproxy_vpcsum_VPCsum_submit(PNIEnv_vpcsum_long* env, int64_t ctx, void* arena, int64_t arenaLen, void* desc,
                                        int32_t n, void* out, void* status, int32_t mode) {
    try {
        if (n < 0 || arenaLen < 0) {
            fail("negative length");
            return pni_throw(env, "java.lang.IllegalArgumentException");
        }
        uint64_t t = 0;
        if (vpcsum_ctx_submit((vpcsum_ctx_t*)(intptr_t)ctx, (uint8_t*)arena, (uint64_t)arenaLen, (const vpcsum_desc_t*)desc,
                              (uint32_t)n, (uint32_t*)out, (uint8_t*)status, (uint32_t)mode, &t) != 0)
            return pni_throw(env, "java.io.IOException");
        env->return_ = (int64_t)t;
        return 0;
    } VPC_CATCH_PNI("Java_io_vproxy_vpcsum_VPCsum_submit")
}

int Java_io_vproxy_vpcsum_VPCsum_waitFor(PNIEnv_vpcsum_void* env, int64_t ctx, int64_t ticket) {
    try {
        if (vpcsum_ctx_wait((vpcsum_ctx_t*)(intptr_t)ctx, (uint64_t)ticket) != 0) return pni_throw(env, "java.io.IOException");
        return 0;
    } VPC_CATCH_PNI("Java_io_vproxy_vpcsum_VPCsum_waitFor")
}

int Java_io_vproxy_vpcsum_VPCsum_verifyFrames(PNIEnv_vpcsum_long* env, int64_t ctx, void* arena, int64_t arenaLen,
                                              void* frameOff, void* frameLen, int32_t n, void* out, void* status) {
    try {
        if (n < 0 || arenaLen < 0) {
            fail("verifyFrames: negative size");
            return pni_throw(env, "java.lang.IllegalArgumentException");
        }
        uint64_t t = 0;
        if (vpcsum_ctx_verify_frames((vpcsum_ctx_t*)(intptr_t)ctx, (const uint8_t*)arena, (uint64_t)arenaLen,
                                     (const uint64_t*)frameOff, (const uint32_t*)frameLen, (uint32_t)n, (uint32_t*)out,
                                     (uint8_t*)status, &t) != 0)
            return pni_throw(env, "java.io.IOException");
        env->return_ = (int64_t)t;
        return 0;
    } VPC_CATCH_PNI("Java_io_vproxy_vpcsum_VPCsum_verifyFrames")
}

int Java_io_vproxy_vpcsum_VPCsum_verifyFramesHsum(PNIEnv_vpcsum_long* env, int64_t ctx, void* arena, int64_t arenaLen,
                                                  void* frameOff, void* frameLen, int32_t n, void* out, void* status,
                                                  void* hsum) {
    try {
        if (n < 0 || arenaLen < 0) {
            fail("verifyFramesHsum: negative size");
            return pni_throw(env, "java.lang.IllegalArgumentException");
        }
        uint64_t t = 0;
        if (vpcsum_ctx_verify_frames_hsum((vpcsum_ctx_t*)(intptr_t)ctx, (const uint8_t*)arena, (uint64_t)arenaLen,
                                          (const uint64_t*)frameOff, (const uint32_t*)frameLen, (uint32_t)n, (uint32_t*)out,
                                          (uint8_t*)status, (vpcsum_hsum_t*)hsum, &t) != 0)
            return pni_throw(env, "java.io.IOException");
        env->return_ = (int64_t)t;
        return 0;
    } VPC_CATCH_PNI("Java_io_vproxy_vpcsum_VPCsum_verifyFramesHsum")
}

int Java_io_vproxy_vpcsum_VPCsum_egressFrames(PNIEnv_vpcsum_long* env, int64_t ctx, void* arena, int64_t arenaLen,
                                              void* frameOff, void* frameLen, void* frameFlags, int32_t n, void* out,
                                              void* status) {
    try {
        if (n < 0 || arenaLen < 0) {
            fail("egressFrames: negative size");
            return pni_throw(env, "java.lang.IllegalArgumentException");
        }
        uint64_t t = 0;
        if (vpcsum_ctx_egress_frames((vpcsum_ctx_t*)(intptr_t)ctx, (uint8_t*)arena, (uint64_t)arenaLen,
                                     (const uint64_t*)frameOff, (const uint32_t*)frameLen, (const uint8_t*)frameFlags,
                                     (uint32_t)n, (uint32_t*)out, (uint8_t*)status, &t) != 0)
            return pni_throw(env, "java.io.IOException");
        env->return_ = (int64_t)t;
        return 0;
    } VPC_CATCH_PNI("Java_io_vproxy_vpcsum_VPCsum_egressFrames")
}

int Java_io_vproxy_vpcsum_VPCsum_parseFrames(PNIEnv_vpcsum_long* env, int64_t ctx, void* arena, int64_t arenaLen,
                                             void* frameOff, void* frameLen, int32_t n, void* desc, void* status,
                                             void* tuples) {
    try {
        if (n < 0 || arenaLen < 0) {
            fail("parseFrames: negative size");
            return pni_throw(env, "java.lang.IllegalArgumentException");
        }
        uint64_t t = 0;
        if (vpcsum_ctx_parse_frames((vpcsum_ctx_t*)(intptr_t)ctx, (const uint8_t*)arena, (uint64_t)arenaLen,
                                    (const uint64_t*)frameOff, (const uint32_t*)frameLen, (uint32_t)n,
                                    (vpcsum_desc_t*)desc, (uint8_t*)status, (vpcsum_tuple_t*)tuples, &t) != 0)
            return pni_throw(env, "java.io.IOException");
        env->return_ = (int64_t)t;
        return 0;
    } VPC_CATCH_PNI("Java_io_vproxy_vpcsum_VPCsum_parseFrames")
}

int Java_io_vproxy_vpcsum_VPCsum_submitPre(PNIEnv_vpcsum_long* env, int64_t ctx, void* arena, int64_t arenaLen,
                                           void* desc, void* pre, int32_t n, void* out, void* status, int32_t mode) {
    try {
        if (n < 0 || arenaLen < 0) {
            fail("submitPre: negative size");
            return pni_throw(env, "java.lang.IllegalArgumentException");
        }
        uint64_t t = 0;
        if (vpcsum_ctx_submit_pre((vpcsum_ctx_t*)(intptr_t)ctx, (uint8_t*)arena, (uint64_t)arenaLen,
                                  (const vpcsum_desc_t*)desc, pre, VPCSUM_PRE_FMT_PRE, (uint32_t)n, (uint32_t*)out,
                                  (uint8_t*)status, (uint32_t)mode, &t) != 0)
            return pni_throw(env, "java.io.IOException");
        env->return_ = (int64_t)t;
        return 0;
    } VPC_CATCH_PNI("Java_io_vproxy_vpcsum_VPCsum_submitPre")
}

int Java_io_vproxy_vpcsum_VPCsum_natSubmit(PNIEnv_vpcsum_long* env, int64_t ctx, void* arena, int64_t arenaLen,
                                           void* desc, void* rw, int32_t n, void* status, int32_t natMode) {
    try {
        if (n < 0 || arenaLen < 0) {
            fail("natSubmit: negative size");
            return pni_throw(env, "java.lang.IllegalArgumentException");
        }
        uint64_t t = 0;
        if (vpcsum_ctx_nat_submit((vpcsum_ctx_t*)(intptr_t)ctx, (uint8_t*)arena, (uint64_t)arenaLen,
                                  (const vpcsum_desc_t*)desc, (const vpcsum_nat_t*)rw, (uint32_t)n, (uint8_t*)status,
                                  (uint32_t)natMode, &t) != 0)
            return pni_throw(env, "java.io.IOException");
        env->return_ = (int64_t)t;
        return 0;
    } VPC_CATCH_PNI("Java_io_vproxy_vpcsum_VPCsum_natSubmit")
}

int Java_io_vproxy_vpcsum_VPCsum_setService(PNIEnv_vpcsum_void* env, int64_t ctx, int32_t idleUs) {
    try {
        if (idleUs < 0) {
            fail("setService: negative idle time %d", idleUs);
            return pni_throw(env, "java.lang.IllegalArgumentException");
        }
        if (vpcsum_ctx_set_service((vpcsum_ctx_t*)(intptr_t)ctx, (uint32_t)idleUs) != 0) return pni_throw(env, "java.io.IOException");
        return 0;
    } VPC_CATCH_PNI("Java_io_vproxy_vpcsum_VPCsum_setService")
}

int Java_io_vproxy_vpcsum_VPCsum_close(PNIEnv_vpcsum_void* env, int64_t ctx) {
    try {
        (void)env;
        vpcsum_ctx_destroy((vpcsum_ctx_t*)(intptr_t)ctx);
        return 0;
    } VPC_CATCH_PNI("Java_io_vproxy_vpcsum_VPCsum_close")
}

}  // extern "C"
