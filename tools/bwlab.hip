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

// NAT-like pattern: per frame, read the first `bytes` (TEAM lanes, 16 B each, UNR frames in
// flight per team) and, with WR, write 32 B back at frame offset 8 (IP header + ports), as the
// NAT rewrite does.  TEAM 1 = a lane per frame (k_natw's layout); TEAM 4 = a 64-B segment per
// 4 lanes, so one load instruction covers 16 frames instead of 64.
template <int TEAM, int UNR, bool WR>
__global__ __launch_bounds__(256) void k_natpat(uint8_t* __restrict__ a, uint32_t nfr, uint32_t stride, uint32_t bytes, uint32_t* sink) {
    uint32_t x = 0;
    const int tl = threadIdx.x & (TEAM - 1);
    const uint32_t team = (blockIdx.x * 256u + threadIdx.x) / TEAM;
    const uint32_t nteams = gridDim.x * (256u / TEAM);
    const int nch = (bytes + 15) / 16;
    constexpr int CPL = TEAM >= 4 ? 1 : 4 / TEAM;   // chunks per lane
    for (uint32_t f0 = team; f0 < nfr; f0 += nteams * UNR) {
        uint4 v[UNR][CPL];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const uint32_t f = f0 + u * nteams;
            const uint4* b = (const uint4*)(a + (uint64_t)f * stride);
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int k = c * TEAM + tl;
                v[u][c] = (f < nfr && k < nch) ? *(const uint4*)(b + k) : make_uint4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const uint32_t f = f0 + u * nteams;
#pragma unroll
            for (int c = 0; c < CPL; ++c) x += v[u][c].x + v[u][c].y + v[u][c].z + v[u][c].w;
            if (WR && f < nfr) {
                uint8_t* b = a + (uint64_t)f * stride;
                if (TEAM == 1) {
                    *(uint4*)(b + 8) = make_uint4(v[u][0].z, v[u][0].w, v[u][1].x ^ x, v[u][1].y);
                    *(uint4*)(b + 24) = make_uint4(v[u][1].z, v[u][1].w, v[u][2].x, v[u][2].y);
                } else if (tl < 2) {
                    *(uint4*)(b + 8 + 16 * tl) = make_uint4(v[u][0].y, v[u][0].z ^ (x & 1), v[u][0].w, v[u][0].x);
                }
            }
        }
    }
    if (x == 0x12345678) sink[0] = x;
}

// The same with aligned write-backs: TEAM lanes read CPL x 16 B each of the frame's first
// TEAM * CPL chunks, and the chunks below WB bytes are written back (modified) in place.
// POL: 0 plain load / plain store, 1 nt load / nt store, 2 plain load / nt store,
// 3 plain load / sc1 (write-through) store, 4 nt load / plain store
template <int TEAM, int CPL, int WB, int POL = 0>
__global__ __launch_bounds__(256) void k_natpat2(uint8_t* __restrict__ a, uint32_t nfr, uint32_t stride, uint32_t* sink) {
    uint32_t x = 0;
    const int tl = threadIdx.x & (TEAM - 1);
    const uint32_t team = (blockIdx.x * 256u + threadIdx.x) / TEAM;
    const uint32_t nteams = gridDim.x * (256u / TEAM);
    constexpr int UNR = 2;
    for (uint32_t f0 = team; f0 < nfr; f0 += nteams * UNR) {
        uint4 v[UNR][CPL];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const uint32_t f = f0 + u * nteams;
            const uint4* b = (const uint4*)(a + (uint64_t)f * stride);
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                if (f >= nfr) { v[u][c] = make_uint4(0, 0, 0, 0); continue; }
                if (POL == 1 || POL == 4) {
                    const u32x4 t = __builtin_nontemporal_load((const u32x4*)(b + c * TEAM + tl));
                    v[u][c] = make_uint4(t.x, t.y, t.z, t.w);
                } else {
                    v[u][c] = b[c * TEAM + tl];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const uint32_t f = f0 + u * nteams;
            uint4* b = (uint4*)(a + (uint64_t)f * stride);
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                x += v[u][c].x + v[u][c].w;
                const int k = c * TEAM + tl;
                if (f < nfr && k * 16 < WB) {
                    const u32x4 t = {v[u][c].y, v[u][c].x ^ (x & 1), v[u][c].w, v[u][c].z};
                    if (POL == 1 || POL == 2) __builtin_nontemporal_store(t, (u32x4*)(b + k));
                    else if (POL == 3) __builtin_amdgcn_raw_buffer_store_b128(t, __builtin_amdgcn_make_buffer_rsrc((void*)b, 0, 0x7fffffff, 0x00020000), k * 16, 0, 16);
                    else *(u32x4*)(b + k) = t;
                }
            }
        }
    }
    if (x == 0x12345678) sink[0] = x;
}

int main(int argc, char** argv) {
    if (argc > 1 && argv[1][0] == 'n') {   // NAT access pattern over a 20.5-GB arena of 2-KB frames
        const uint32_t nfr = 10000000, stride = 2048;
        uint8_t* buf;
        uint32_t* sink;
        CK(hipMalloc(&buf, (uint64_t)nfr * stride));
        CK(hipMalloc(&sink, 4096));
        CK(hipMemset(buf, 1, (uint64_t)nfr * stride));
        int cus = 0;
        CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        auto run = [&](const char* name, auto&& launch) {
            for (int i = 0; i < 3; ++i) launch();
            CK(hipDeviceSynchronize());
            std::vector<float> ts;
            for (int r = 0; r < 9; ++r) {
                CK(hipEventRecord(e0));
                launch();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                ts.push_back(ms);
            }
            std::sort(ts.begin(), ts.end());
            printf("%-48s median %6.2f Gframes/s (%.3f ms)\n", name, nfr / ts[ts.size() / 2] / 1e6, ts[ts.size() / 2]);
        };
        char nm[128];
#define NP(T, U, WR, BPC, BY)                                                                        \
        snprintf(nm, sizeof nm, "natpat team=%d unr=%d wr=%d bpc=%d bytes=%d", T, U, WR, BPC, BY);   \
        run(nm, [&] { hipLaunchKernelGGL((k_natpat<T, U, WR>), dim3(cus * BPC), dim3(256), 0, 0, buf, nfr, stride, BY, sink); });
#define NP2(T, C, WB)                                                                                \
        snprintf(nm, sizeof nm, "natpat2 team=%d chunks/lane=%d write=%dB@0 bpc=24", T, C, WB);      \
        run(nm, [&] { hipLaunchKernelGGL((k_natpat2<T, C, WB>), dim3(cus * 24), dim3(256), 0, 0, buf, nfr, stride, sink); });
#define NP3(T, C, WB, POL)                                                                           \
        snprintf(nm, sizeof nm, "natpat2 team=%d chunks/lane=%d write=%dB@0 pol=%d", T, C, WB, POL);  \
        run(nm, [&] { hipLaunchKernelGGL((k_natpat2<T, C, WB, POL>), dim3(cus * 24), dim3(256), 0, 0, buf, nfr, stride, sink); });
        if (argc > 2) {   // cache policies of the read + write-back
            for (int rep = 0; rep < 2; ++rep) {
                NP3(4, 1, 64, 0) NP3(4, 1, 64, 1) NP3(4, 1, 64, 2) NP3(4, 1, 64, 3) NP3(4, 1, 64, 4)
                NP3(1, 4, 64, 0) NP3(1, 4, 64, 1) NP3(1, 4, 64, 2) NP3(1, 4, 64, 3)
            }
            return 0;
        }
        for (int rep = 0; rep < 2; ++rep) {
            NP(1, 2, false, 24, 48) NP(1, 2, true, 24, 48) NP(4, 2, false, 24, 48) NP(4, 2, true, 24, 48)
            NP2(1, 4, 64) NP2(1, 4, 32) NP2(4, 1, 64) NP2(4, 1, 32) NP2(4, 1, 16) NP2(8, 1, 128) NP2(8, 1, 64) NP2(8, 1, 0)
        }
        return 0;
    }
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
