// flush_latency.cpp -- submit+wait latency of small zero-copy flushes through the C-ABI, the way
// GpuCsumBatch.flush drives it at every Iface.completeTx (tooling; no Python in the timed loop).
// Frames: C2-shaped IPv4/TCP 1500 B at stride 2048 in a registered arena (an AF_XDP umem
// stand-in), MODE_WRITE.  Each size runs with a kernel launch per flush and through the
// low-latency service grid (vpcsum_ctx_set_service).
// Build: g++ -O2 -std=c++17 -I include tools/flush_latency.cpp -L vproxy_amd -lvpcsum
//        -Wl,-rpath,'$ORIGIN/../vproxy_amd' -o tools/flush_latency
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "vpcsum.h"

static void frame(uint8_t* l3, uint32_t i) {
    // IPv4 (ihl 5) + TCP (doff 5) + 1460 payload bytes, deterministic content
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

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    const uint32_t nmax = 8192, stride = 2048;
    std::vector<uint8_t> arena((size_t)nmax * stride + 4096, 0);
    std::vector<vpcsum_desc_t> desc(nmax);
    for (uint32_t i = 0; i < nmax; ++i) {
        frame(arena.data() + (size_t)i * stride, i);
        memset(&desc[i], 0, sizeof(desc[i]));
        desc[i].l3_off = (uint64_t)i * stride;
        desc[i].l3_len = 1500;
        desc[i].l4_off = 20;
        desc[i].l3_ver = 4;
        desc[i].l4_proto = 6;
        desc[i].flags = VPCSUM_F_IP | VPCSUM_F_L4;
    }
    std::vector<uint32_t> out(nmax);
    // NAT'd frames flushed from their pre-images (vpcsum_ctx_submit_pre, 16-B entries naming the
    // addresses and ports): the same frames, every descriptor F_PRE
    std::vector<vpcsum_desc_t> pdesc(desc);
    std::vector<vpcsum_pre4_t> pre(nmax);
    for (uint32_t i = 0; i < nmax; ++i) {
        pdesc[i].flags |= VPCSUM_F_PRE;
        const uint8_t* l3 = arena.data() + (size_t)i * stride;
        memcpy(pre[i].src, l3 + 12, 4);
        memcpy(pre[i].dst, l3 + 16, 4);
        memcpy(pre[i].sport, l3 + 20, 2);
        memcpy(pre[i].dport, l3 + 22, 2);
        pre[i].mask = VPCSUM_NAT_SRC | VPCSUM_NAT_DST | VPCSUM_NAT_SPORT | VPCSUM_NAT_DPORT;
    }
    // the same frames behind a 14-B Ethernet header, for the egress path that parses raw frames on
    // the GPU (vpcsum_ctx_egress_frames: offsets, lengths and per-frame flags only)
    std::vector<uint8_t> eth((size_t)nmax * stride + 4096, 0);
    std::vector<uint64_t> foff(nmax);
    std::vector<uint32_t> flen(nmax);
    std::vector<uint8_t> fflags(nmax, VPCSUM_F_IP | VPCSUM_F_L4);
    std::vector<uint8_t> fst(nmax);
    std::vector<vpcsum_desc_t> pdesc_out(nmax);
    std::vector<vpcsum_tuple_t> tup(nmax);
    for (uint32_t i = 0; i < nmax; ++i) {
        uint8_t* f = eth.data() + (size_t)i * stride;
        f[12] = 0x08;
        frame(f + 14, i);
        foff[i] = (uint64_t)i * stride;
        flen[i] = 1514;
    }
    vpcsum_ctx_t* ctx = nullptr;
    if (vpcsum_ctx_create(0, eth.size(), nmax, &ctx) || vpcsum_ctx_register_arena(ctx, arena.data(), arena.size()) ||
        vpcsum_ctx_register_arena(ctx, eth.data(), eth.size())) {
        fprintf(stderr, "setup: %s\n", vpcsum_last_error());
        return 1;
    }
    // A/B configurations on the same box: 2 = the service with descriptors read from its buffer
    // only (no inline descriptors in the command line); 3 = frame loads clamped to the last chunk
    // (re-loads) instead of predicated; 4 = release semantics on the completion count and `done`.  The configurations run interleaved in kRounds rounds of
    // iters / kRounds flushes per size, so that drift on the box hits all of them alike.
    // 5 = raw frames parsed on the GPU, two launches per flush (vpcsum_ctx_egress_frames).
    // 6 / 7 = NAT'd frames from their pre-images (vpcsum_ctx_submit_pre), launched / service grid.
    // 8 = raw frames through the service grid (parse + sum per frame, no launch).
    // 9 / 10 = ingress verify of received frames, status bytes only (vpcsum_ctx_verify_frames, the
    // GpuCsumBatch.verifyFrames form), launched (parse + verify kernels) / service grid.
    // 11 / 12 = parse of received frames with flow tuples (vpcsum_ctx_parse_frames), launched / service.
    constexpr int kCfg = 13;
    static const char* names[kCfg] = {"launch", "service", "service_no_inline", "service_clamped_loads",
                                      "service_release_done", "egress_frames", "pre_launch", "pre_service",
                                      "egress_frames_service", "verify_frames", "verify_frames_service",
                                      "parse_frames", "parse_frames_service"};
    static const uint32_t sizes[7] = {1u, 3u, 4u, 32u, 128u, 1024u, 8192u};
    constexpr int kRounds = 5;
    std::vector<double> us[kCfg][7];
    for (int r = 0; r < kRounds; ++r) {
        for (int svc = 0; svc < kCfg; ++svc) {
            setenv("VPCSUM_SVC_INLINE", svc == 2 ? "0" : "1", 1);
            setenv("VPCSUM_SVC_CLAMP", svc == 3 ? "1" : "0", 1);
            setenv("VPCSUM_SVC_RELEASE_DONE", svc == 4 ? "1" : "0", 1);
            if (vpcsum_ctx_set_service(ctx, ((svc && svc < 5) || svc == 7 || svc == 8 || svc == 10 || svc == 12) ? 200000 : 0)) {
                fprintf(stderr, "service: %s\n", vpcsum_last_error());
                return 1;
            }
            for (int si = 0; si < 7; ++si) {
                const uint32_t b = sizes[si];
                if (svc >= 2 && svc < 5 && b > 128) break;
                for (int it = 0; it < iters / kRounds + 20; ++it) {
                    uint64_t t = 0;
                    const auto t0 = std::chrono::steady_clock::now();
                    const int rc = svc >= 11
                        ? vpcsum_ctx_parse_frames(ctx, eth.data(), eth.size(), foff.data(), flen.data(), b, pdesc_out.data(),
                                                  fst.data(), tup.data(), &t)
                        : svc >= 9
                        ? vpcsum_ctx_verify_frames(ctx, eth.data(), eth.size(), foff.data(), flen.data(), b, nullptr,
                                                   fst.data(), &t)
                        : (svc == 5 || svc == 8)
                        ? vpcsum_ctx_egress_frames(ctx, eth.data(), eth.size(), foff.data(), flen.data(), fflags.data(),
                                                   b, out.data(), fst.data(), &t)
                        : svc >= 6 ? vpcsum_ctx_submit_pre(ctx, arena.data(), arena.size(), pdesc.data(), pre.data(),
                                                           VPCSUM_PRE_FMT_PRE4, b, out.data(), nullptr, VPCSUM_MODE_WRITE, &t)
                        : vpcsum_ctx_submit(ctx, arena.data(), arena.size(), desc.data(), b, out.data(), nullptr,
                                            VPCSUM_MODE_WRITE, &t);
                    if (rc || vpcsum_ctx_wait(ctx, t)) {
                        fprintf(stderr, "flush: %s\n", vpcsum_last_error());
                        return 1;
                    }
                    const auto t1 = std::chrono::steady_clock::now();
                    if (it >= 20) us[svc][si].push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
                }
            }
        }
    }
    // A small flush right after a large (launched) one, through the service: the large batch stops
    // the resident grid (api.cpp svc_quiesce), so the small one pays a grid launch.  32 frames after
    // 1,024 each time, median / p99 of the small flushes.
    std::vector<double> alt;
    if (vpcsum_ctx_set_service(ctx, 200000)) {
        fprintf(stderr, "service: %s\n", vpcsum_last_error());
        return 1;
    }
    for (int it = 0; it < iters / 2 + 20; ++it) {
        uint64_t t = 0;
        if (vpcsum_ctx_submit(ctx, arena.data(), arena.size(), desc.data(), 1024, out.data(), nullptr, VPCSUM_MODE_WRITE, &t) ||
            vpcsum_ctx_wait(ctx, t)) {
            fprintf(stderr, "flush: %s\n", vpcsum_last_error());
            return 1;
        }
        const auto t0 = std::chrono::steady_clock::now();
        if (vpcsum_ctx_submit(ctx, arena.data(), arena.size(), desc.data(), 32, out.data(), nullptr, VPCSUM_MODE_WRITE, &t) ||
            vpcsum_ctx_wait(ctx, t)) {
            fprintf(stderr, "flush: %s\n", vpcsum_last_error());
            return 1;
        }
        const auto t1 = std::chrono::steady_clock::now();
        if (it >= 20) alt.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::sort(alt.begin(), alt.end());
    printf("{\"service_32_after_1024\": {\"median_us\": %.1f, \"p99_us\": %.1f}, ", alt[alt.size() / 2],
           alt[(size_t)(alt.size() * 0.99)]);
    const char* sep = "";
    for (int svc = 0; svc < kCfg; ++svc) {
        printf("%s\"%s\": {", sep, names[svc]);
        sep = ", ";
        const char* sep2 = "";
        for (int si = 0; si < 7; ++si) {
            std::vector<double>& v = us[svc][si];
            if (v.empty()) continue;
            std::sort(v.begin(), v.end());
            printf("%s\"%u\": {\"median_us\": %.1f, \"p99_us\": %.1f}", sep2, sizes[si], v[v.size() / 2],
                   v[(size_t)(v.size() * 0.99)]);
            sep2 = ", ";
        }
        printf("}");
    }
    uint64_t sb = 0, sl = 0;
    vpcsum_ctx_stats(ctx, &sb, &sl);
    printf(", \"service_batches\": %llu, \"service_launches\": %llu, \"iters\": %d}\n", (unsigned long long)sb,
           (unsigned long long)sl, iters);
    vpcsum_ctx_destroy(ctx);
    return 0;
}
