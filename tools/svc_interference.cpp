// svc_interference.cpp -- why an idle service grid slows launched batches beside it (VERDICT r5
// item 3): submit+wait latency of LAUNCHED zero-copy batches of one context while something else is
// resident on the GPU, conditions interleaved round by round on one box:
//   none        nothing else resident
//   svc32       another context's service grid, idle (32 workgroups x 256, polling its mailbox)
//   svc8/svc1   the same grid cut to 8 / 1 workgroups (VPCSUM_SVC_GRID)
//   spin32x256  a grid of the same shape that only sleeps (vpcsum_spin_probe_async): no memory traffic
//   spin1x64    one sleeping wave
//   svc32_acquire  the 32-workgroup grid with round 5's acquire loads in its relay poll
// (argv[2] = "poll": the relay poll modes instead, VPCSUM_SVC_POLL)
// Batches (context B, no service): 1,024 and 8,192 descriptors (MODE_WRITE), 1,024 raw frames
// verified (parse + verify kernels), 1,024 raw egress frames (parse + sum).
// Build: hipcc -O2 -std=c++17 -I include tools/svc_interference.cpp -L vproxy_amd -lvpcsum
//        -Wl,-rpath,'$ORIGIN/../vproxy_amd' -o tools/svc_interference
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "vpcsum.h"

static void frame(uint8_t* l3, uint32_t i) {
    memset(l3, 0, 40);
    l3[0] = 0x45;
    l3[2] = 1500 >> 8;
    l3[3] = 1500 & 0xff;
    l3[8] = 64;
    l3[9] = 6;
    for (int k = 0; k < 4; ++k) l3[12 + k] = (uint8_t)(i >> (8 * k)), l3[16 + k] = (uint8_t)(~i >> (8 * k));
    l3[32] = 0x50;
    for (int k = 40; k < 1500; ++k) l3[k] = (uint8_t)(k * 31 + i * 7);
}

#define CHECK(x)                                                          \
    do {                                                                  \
        if ((x) != 0) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, vpcsum_last_error());         \
            exit(1);                                                      \
        }                                                                 \
    } while (0)

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 400;
    const uint32_t nmax = 8192, stride = 2048;
    std::vector<uint8_t> eth((size_t)nmax * stride + 4096, 0);
    std::vector<uint8_t> l3a((size_t)nmax * stride + 4096, 0);
    std::vector<vpcsum_desc_t> desc(nmax);
    std::vector<uint64_t> foff(nmax);
    std::vector<uint32_t> flen(nmax);
    std::vector<uint8_t> fflags(nmax, VPCSUM_F_IP | VPCSUM_F_L4), st(nmax);
    std::vector<uint32_t> out(nmax);
    for (uint32_t i = 0; i < nmax; ++i) {
        uint8_t* f = eth.data() + (size_t)i * stride;
        f[12] = 0x08;
        frame(f + 14, i);
        foff[i] = (uint64_t)i * stride;
        flen[i] = 1514;
        frame(l3a.data() + (size_t)i * stride, i);
        memset(&desc[i], 0, sizeof(desc[i]));
        desc[i].l3_off = (uint64_t)i * stride;
        desc[i].l3_len = 1500;
        desc[i].l4_off = 20;
        desc[i].l3_ver = 4;
        desc[i].l4_proto = 6;
        desc[i].flags = VPCSUM_F_IP | VPCSUM_F_L4;
    }
    vpcsum_ctx_t* b = nullptr;
    CHECK(vpcsum_ctx_create(0, eth.size(), nmax, &b));
    CHECK(vpcsum_ctx_register_arena(b, eth.data(), eth.size()));
    CHECK(vpcsum_ctx_register_arena(b, l3a.data(), l3a.size()));
    // the other context, whose idle service grid is the suspect; its own small arena
    std::vector<uint8_t> small(64 * stride, 0);
    for (uint32_t i = 0; i < 64; ++i) frame(small.data() + (size_t)i * stride, i);
    vpcsum_ctx_t* a = nullptr;
    CHECK(vpcsum_ctx_create(0, small.size(), 64, &a));
    CHECK(vpcsum_ctx_register_arena(a, small.data(), small.size()));
    hipStream_t spin_stream;
    if (hipStreamCreateWithFlags(&spin_stream, hipStreamNonBlocking) != hipSuccess) return 1;

    struct Cond { const char* name; int svc_grid; uint32_t spin_wgs, spin_threads; int poll; };
    // argv[2] == "poll": the relay poll modes of the 32-workgroup grid instead (VPCSUM_SVC_POLL)
    const bool polls = argc > 2 && strcmp(argv[2], "poll") == 0;
    // poll -1: the library's default relay poll (VPCSUM_SVC_POLL unset)
    const Cond base[] = {{"none", 0, 0, 0, -1},         {"svc32", 32, 0, 0, -1},        {"svc8", 8, 0, 0, -1},
                         {"svc1", 1, 0, 0, -1},         {"spin32x256", 0, 32, 256, -1}, {"spin1x64", 0, 1, 64, -1},
                         {"svc32_acquire", 32, 0, 0, 0}};
    const Cond pollc[] = {{"none", 0, 0, 0, 0},           {"svc32_acquire", 32, 0, 0, 0},  {"svc32_relaxed", 32, 0, 0, 1},
                          {"svc32_backoff", 32, 0, 0, 2}, {"svc32_relaxed_backoff", 32, 0, 0, 3},
                          {"svc32_relaxed_rareclock", 32, 0, 0, 5}, {"svc32_all", 32, 0, 0, 7}};
    const Cond* conds = polls ? pollc : base;
    constexpr int kCond = 7;
    const char* forms[] = {"desc1024", "desc8192", "verify_frames1024", "egress_frames1024"};
    constexpr int kForm = 4;
    std::vector<double> us[kCond][kForm];
    constexpr int kRounds = 5;
    for (int r = 0; r < kRounds; ++r) {
        for (int ci = 0; ci < kCond; ++ci) {
            const Cond& c = conds[ci];
            // the condition: a service grid on context a (idle for the whole block), or a spin probe
            if (c.svc_grid) {
                setenv("VPCSUM_SVC_GRID", std::to_string(c.svc_grid).c_str(), 1);
                if (c.poll < 0) unsetenv("VPCSUM_SVC_POLL");
                else setenv("VPCSUM_SVC_POLL", std::to_string(c.poll).c_str(), 1);
                CHECK(vpcsum_ctx_set_service(a, 2000000));   // 2 s idle: resident through the block
                uint64_t t = 0;
                CHECK(vpcsum_ctx_submit(a, small.data(), small.size(), desc.data(), 3, out.data(), nullptr,
                                        VPCSUM_MODE_COMPUTE, &t));
                CHECK(vpcsum_ctx_wait(a, t));
            }
            if (c.spin_wgs) CHECK(vpcsum_spin_probe_async(c.spin_wgs, c.spin_threads, 300000, spin_stream));
            for (int fi = 0; fi < kForm; ++fi) {
                for (int it = 0; it < iters / kRounds + 10; ++it) {
                    uint64_t t = 0;
                    const auto t0 = std::chrono::steady_clock::now();
                    if (fi == 0 || fi == 1)
                        CHECK(vpcsum_ctx_submit(b, l3a.data(), l3a.size(), desc.data(), fi == 0 ? 1024 : 8192, out.data(),
                                                nullptr, VPCSUM_MODE_WRITE, &t));
                    else if (fi == 2)
                        CHECK(vpcsum_ctx_verify_frames(b, eth.data(), eth.size(), foff.data(), flen.data(), 1024, nullptr,
                                                       st.data(), &t));
                    else
                        CHECK(vpcsum_ctx_egress_frames(b, eth.data(), eth.size(), foff.data(), flen.data(), fflags.data(),
                                                       1024, out.data(), st.data(), &t));
                    CHECK(vpcsum_ctx_wait(b, t));
                    const auto t1 = std::chrono::steady_clock::now();
                    if (it >= 10) us[ci][fi].push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
                }
            }
            if (c.svc_grid) CHECK(vpcsum_ctx_set_service(a, 0));   // stops the grid
            if (c.spin_wgs && hipStreamSynchronize(spin_stream) != hipSuccess) return 1;
        }
        fprintf(stderr, "round %d done\n", r);
    }
    printf("{");
    for (int ci = 0; ci < kCond; ++ci) {
        printf("%s\"%s\": {", ci ? ", " : "", conds[ci].name);
        for (int fi = 0; fi < kForm; ++fi) {
            std::vector<double>& v = us[ci][fi];
            std::sort(v.begin(), v.end());
            printf("%s\"%s\": {\"median_us\": %.1f, \"p10_us\": %.1f, \"p90_us\": %.1f}", fi ? ", " : "", forms[fi],
                   v[v.size() / 2], v[v.size() / 10], v[v.size() * 9 / 10]);
        }
        printf("}");
    }
    printf(", \"iters\": %d}\n", iters);
    vpcsum_ctx_destroy(a);
    vpcsum_ctx_destroy(b);
    return 0;
}
