// bwlab.hip -- HBM read-bandwidth lab for MI355X (tooling, not product).
// Measures what read patterns reach on this chip so the checksum kernel's roofline fraction can
// be judged against a measured ceiling.  Build: hipcc -O3 --offload-arch=gfx950 tools/bwlab.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint4* q) {
    u32x4 v = NT ? __builtin_nontemporal_load((const u32x4*)q) : *(const u32x4*)q;
    return make_uint4(v.x, v.y, v.z, v.w);
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int UNR, bool NT>
__global__ __launch_bounds__(256) void k_gs(const uint4* __restrict__ p, uint64_t n16, uint32_t* sink) {
    uint32_t x = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (UNR - 1) * stride < n16; i += UNR * stride) {
        uint4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = ld16<NT>(p + i + u * stride);
#pragma unroll
        for (int u = 0; u < UNR; ++u) x += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    for (; i < n16; i += stride) { uint4 v = p[i]; x += v.x + v.y + v.z + v.w; }
    if (x == 0x12345678) sink[0] = x;
}

// Each block owns a contiguous slab; lanes sweep it 4 KiB (256 x 16 B) at a time, UNR deep.
template <int UNR, bool NT>
__global__ __launch_bounds__(256) void k_slab(const uint4* __restrict__ p, uint64_t n16, uint32_t* sink) {
    uint32_t x = 0;
    const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per;
    const uint64_t hi = min(lo + per, n16);
    uint64_t i = lo + threadIdx.x;
    for (; i + (UNR - 1) * 256 < hi; i += UNR * 256) {
        uint4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = ld16<NT>(p + i + u * 256);
#pragma unroll
        for (int u = 0; u < UNR; ++u) x += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    for (; i < hi; i += 256) { uint4 v = p[i]; x += v.x + v.y + v.z + v.w; }
    if (x == 0x12345678) sink[0] = x;
}

// Packet pattern: read the first `bytes` of every `stride`-byte frame, TEAM lanes per frame.
template <int TEAM, int UNR, bool NT>
__global__ __launch_bounds__(256) void k_pkt(const uint8_t* __restrict__ a, uint32_t nfr, uint32_t stride, uint32_t bytes, uint32_t* sink) {
    uint32_t x = 0;
    const int tl = threadIdx.x & (TEAM - 1);
    const uint32_t team = (blockIdx.x * 256u + threadIdx.x) / TEAM;
    const uint32_t nteams = gridDim.x * (256u / TEAM);
    const int nch = (bytes + 15) / 16;
    for (uint32_t f = team; f < nfr; f += nteams) {
        const uint4* b = (const uint4*)(a + (uint64_t)f * stride);
        for (int r = 0; r * TEAM < nch; r += UNR) {
            uint4 v[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                int k = (r + u) * TEAM + tl;
                v[u] = k < nch ? ld16<NT>(b + k) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) x += v[u].x + v[u].y + v[u].z + v[u].w;
        }
    }
    if (x == 0x12345678) sink[0] = x;
}

int main(int argc, char** argv) {
    const uint64_t bytes = 2ull << 30;
    uint8_t* buf;
    uint32_t* sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(buf, 1, bytes));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t n16 = bytes / 16;
    auto timeit = [&](const char* name, double nbytes, auto&& launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int r = 0; r < 15; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%-44s best %7.1f GB/s  median %7.1f GB/s  (%.3f ms)\n", name, nbytes / ts[0] / 1e6,
               nbytes / ts[ts.size() / 2] / 1e6, ts[ts.size() / 2]);
    };
    char nm[128];
#define GS(U, NT, BPC)                                                                         \
    snprintf(nm, sizeof nm, "gs unr=%d nt=%d blocks/CU=%d", U, NT, BPC);                       \
    timeit(nm, (double)bytes, [&] { hipLaunchKernelGGL((k_gs<U, NT>), dim3(cus * BPC), dim3(256), 0, 0, (const uint4*)buf, n16, sink); });
    GS(1, false, 8) GS(2, false, 8) GS(4, false, 8) GS(8, false, 8) GS(4, false, 4) GS(4, false, 16) GS(8, false, 16)
    GS(4, true, 8) GS(8, true, 8) GS(4, false, 32)
#define SL(U, NT, BPC)                                                                         \
    snprintf(nm, sizeof nm, "slab unr=%d nt=%d blocks/CU=%d", U, NT, BPC);                     \
    timeit(nm, (double)bytes, [&] { hipLaunchKernelGGL((k_slab<U, NT>), dim3(cus * BPC), dim3(256), 0, 0, (const uint4*)buf, n16, sink); });
    SL(4, false, 8) SL(8, false, 8) SL(4, false, 16) SL(8, true, 8) SL(16, false, 4)
    const uint32_t nfr = 1u << 20, stride = 2048, pb = 1504;
#define PK(T, U, NT, BPC)                                                                      \
    snprintf(nm, sizeof nm, "pkt1504/2048 team=%d unr=%d nt=%d bpc=%d", T, U, NT, BPC);         \
    timeit(nm, (double)nfr * pb, [&] { hipLaunchKernelGGL((k_pkt<T, U, NT>), dim3(cus * BPC), dim3(256), 0, 0, buf, nfr, stride, pb, sink); });
    if (argc > 1) {   // short mode: the packet pattern with nt loads only, strided vs packed
        PK(16, 8, true, 8) PK(16, 8, true, 2) PK(8, 6, true, 2) PK(8, 6, true, 8)
#define PKS(T, U, BPC, STR)                                                                          \
    snprintf(nm, sizeof nm, "pkt1504/%d team=%d unr=%d nt=1 bpc=%d", STR, T, U, BPC);                \
    timeit(nm, (double)nfr * pb, [&] { hipLaunchKernelGGL((k_pkt<T, U, true>), dim3(cus * BPC), dim3(256), 0, 0, buf, nfr, STR, pb, sink); });
        PKS(16, 8, 8, 1504) PKS(16, 8, 2, 1504) PKS(8, 6, 2, 1504) PKS(16, 8, 8, 1536) PKS(16, 8, 2, 1536)
        SL(8, true, 2) SL(8, true, 8)
        return 0;
    }
    PK(16, 8, false, 8) PK(16, 8, true, 8) PK(32, 4, false, 8) PK(64, 2, false, 8) PK(64, 2, false, 16) PK(16, 8, false, 4) PK(8, 12, false, 8)
    PK(16, 8, false, 16) PK(32, 4, false, 16) PK(64, 2, true, 16)
    // contiguous packing (stride == bytes rounded to 16) for comparison
    timeit("pkt1504/1504 team=16 unr=8", (double)nfr * pb, [&] { hipLaunchKernelGGL((k_pkt<16, 8, false>), dim3(cus * 8), dim3(256), 0, 0, buf, nfr, 1504, pb, sink); });
    return 0;
}
