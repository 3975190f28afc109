// Host <-> GPU ping-pong latency through a mailbox in (a) pinned host memory and (b) fine-grained
// device memory written by the host over the PCIe BAR, if the platform maps it (tooling: decides
// where the service grid's command word and descriptors should live).
// Build: hipcc --offload-arch=gfx950 -O2 tools/bar_probe.cpp -o tools/bar_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <algorithm>
#include <chrono>
#include <vector>

// GPU side: wait for ping == k (system-scope load), answer pong = k, for k = 1..iters.  MODE adds
// one of the service grid's per-batch steps between the two, to price it:
// 1 acquire fence (system), 2 release fence (system), 3 release fence (agent), 4 device atomic
// add (agent, acq_rel), 5 a 16-B load from host memory, 6 steps 1+2+4 together.
__device__ uint32_t g_ctr;
template <int MODE>
__global__ void k_echo(volatile uint32_t* ping, uint32_t* pong, uint32_t iters, const uint4* hsrc) {
    if (threadIdx.x != 0) return;
    if (blockIdx.x != 0) {   // extra pollers of the same line (the service grid has 32)
        uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load((uint32_t*)ping, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != iters) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) return;
            __builtin_amdgcn_s_sleep(1);
        }
        return;
    }
    uint32_t sink = 0;
    for (uint32_t k = 1; k <= iters; ++k) {
        uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load((uint32_t*)ping, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != k) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) return;   // 2 s: give up
            __builtin_amdgcn_s_sleep(1);
        }
        if (MODE == 1 || MODE == 6) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        if (MODE == 5) sink += __builtin_nontemporal_load(&hsrc[k & 63].x);
        if (MODE == 2 || MODE == 6) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        if (MODE == 3) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (MODE == 4 || MODE == 6) sink += __hip_atomic_fetch_add(&g_ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pong, k + (sink & 0u), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double run(const char* name, uint32_t* ping_h, uint32_t* ping_d, uint32_t* pong_h, uint32_t* pong_d, int iters,
                  int mode = 0, const uint4* hsrc = nullptr, int pollers = 1) {
    *(volatile uint32_t*)ping_h = 0;
    *(volatile uint32_t*)pong_h = 0;
    switch (mode) {
        case 0: hipLaunchKernelGGL(k_echo<0>, dim3(pollers), dim3(64), 0, 0, ping_d, pong_d, (uint32_t)iters, hsrc); break;
        case 1: hipLaunchKernelGGL(k_echo<1>, dim3(1), dim3(64), 0, 0, ping_d, pong_d, (uint32_t)iters, hsrc); break;
        case 2: hipLaunchKernelGGL(k_echo<2>, dim3(1), dim3(64), 0, 0, ping_d, pong_d, (uint32_t)iters, hsrc); break;
        case 3: hipLaunchKernelGGL(k_echo<3>, dim3(1), dim3(64), 0, 0, ping_d, pong_d, (uint32_t)iters, hsrc); break;
        case 4: hipLaunchKernelGGL(k_echo<4>, dim3(1), dim3(64), 0, 0, ping_d, pong_d, (uint32_t)iters, hsrc); break;
        case 5: hipLaunchKernelGGL(k_echo<5>, dim3(1), dim3(64), 0, 0, ping_d, pong_d, (uint32_t)iters, hsrc); break;
        default: hipLaunchKernelGGL(k_echo<6>, dim3(1), dim3(64), 0, 0, ping_d, pong_d, (uint32_t)iters, hsrc); break;
    }
    std::vector<double> us;
    for (int k = 1; k <= iters; ++k) {
        auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(ping_h, (uint32_t)k, __ATOMIC_RELEASE);
        while (__atomic_load_n(pong_h, __ATOMIC_ACQUIRE) != (uint32_t)k) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                printf("%s: no answer at %d\n", name, k);
                (void)hipDeviceSynchronize();
                return -1;
            }
        }
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    (void)hipDeviceSynchronize();
    std::sort(us.begin(), us.end());
    const double med = us[us.size() / 2];
    printf("{\"mailbox\": \"%s\", \"round_trip_median_us\": %.2f, \"p99_us\": %.2f}\n", name, med, us[us.size() * 99 / 100]);
    return med;
}

int main() {
    const int iters = 2000;
    uint32_t *h = nullptr, *hd = nullptr;
    if (hipHostMalloc((void**)&h, 4096, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
    (void)hipHostGetDevicePointer((void**)&hd, h, 0);
    // (a) ping and pong both in pinned host memory (what the service grid uses today)
    run("host_pinned", h, hd, h + 16, hd + 16, iters);
    const char* names[] = {"", "+acquire_system", "+release_system", "+release_agent", "+atomic_agent", "+host_load_16B",
                           "+acquire+release+atomic"};
    for (int m = 1; m <= 6; ++m) run(names[m], h, hd, h + 16, hd + 16, iters, m, (const uint4*)(hd + 256));
    run("32_pollers_same_line", h, hd, h + 16, hd + 16, iters, 0, nullptr, 32);
    run("8_pollers_same_line", h, hd, h + 16, hd + 16, iters, 0, nullptr, 8);
    // cost of the host-side runtime calls a service submit makes while the grid runs
    {
        hipStream_t st;
        (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
        *(volatile uint32_t*)h = 0;
        hipLaunchKernelGGL(k_echo<0>, dim3(1), dim3(64), 0, st, hd, hd + 16, 1u, (const uint4*)nullptr);   // waits for ping 1
        const int q = 20000;
        auto t0 = std::chrono::steady_clock::now();
        int busy = 0;
        for (int i = 0; i < q; ++i) busy += hipStreamQuery(st) != hipSuccess;
        auto t1 = std::chrono::steady_clock::now();
        for (int i = 0; i < q; ++i) (void)hipSetDevice(0);
        auto t2 = std::chrono::steady_clock::now();
        __atomic_store_n(h, 1u, __ATOMIC_RELEASE);
        (void)hipStreamSynchronize(st);
        auto t3 = std::chrono::steady_clock::now();
        for (int i = 0; i < q; ++i) (void)hipStreamQuery(st);
        auto t4 = std::chrono::steady_clock::now();
        printf("{\"hipStreamQuery_busy_us\": %.3f, \"busy_fraction\": %.2f, \"hipSetDevice_us\": %.3f, \"hipStreamQuery_idle_us\": %.3f}\n",
               std::chrono::duration<double, std::micro>(t1 - t0).count() / q, busy / (double)q,
               std::chrono::duration<double, std::micro>(t2 - t1).count() / q,
               std::chrono::duration<double, std::micro>(t4 - t3).count() / q);
        (void)hipStreamDestroy(st);
    }
    return 0;
}
