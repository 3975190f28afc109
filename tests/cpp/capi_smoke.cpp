// C-ABI consumer in plain C++ (no torch, no Python): what a JNI/Panama-side native or any other
// host binds.  Builds the reference's udpIpv4Example / tcpIpv4SynExample frames
// (TestPacket.java:459-494, 329-378), checksums them through vpcsum_ctx_* and through the PNI
// entry points, and checks the values the reference test pins (0x7f41/0xdf0d, 0x87e4/0xf3ff);
// then NAT-rewrites them through the PNI entry (zero-copy and staged) and verifies the result.
// Build: g++ -std=c++17 -I include tests/cpp/capi_smoke.cpp -L vproxy_amd -lvpcsum -o capi_smoke
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>

#include "vpcsum.h"

static std::vector<uint8_t> hex(const char* h) {
    std::vector<uint8_t> b;
    for (size_t i = 0; h[i] && h[i + 1]; i += 2) b.push_back((uint8_t)strtoul(std::string(h + i, 2).c_str(), nullptr, 16));
    return b;
}

#define CHECK(c, ...) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); fprintf(stderr, __VA_ARGS__); fprintf(stderr, "\n"); return 1; } } while (0)

int main() {
    // udpIpv4Example (Ethernet + IPv4 + UDP DNS answer)
    std::vector<uint8_t> udp = hex(
        "f8ffc207896ed66292eecebf08004500005937bd400040117f41c0a80101c0a801440035c9140045df0d"
        "15bb8000000100010000000003313237013001300131077370656369616c067670726f78790263630000010001c00c0001000100000bef00047f000001");
    // tcpIpv4SynExample
    std::vector<uint8_t> syn = hex(
        "cc70edc4e4f9f8ffc207896e08004500004000004000400687e40af2c270b465310cf56801bbeac8fcf500000000b002"
        "fffff3ff0000020405b4010303060101080a16ac9a990000000004020000");

    std::vector<uint8_t> arena(4096, 0);
    memcpy(arena.data() + 0, udp.data(), udp.size());
    memcpy(arena.data() + 2048, syn.data(), syn.size());
    vpcsum_desc_t d[2];
    memset(d, 0, sizeof(d));
    d[0].l3_off = 14; d[0].l3_len = 0x59; d[0].l4_off = 20; d[0].l3_ver = 4; d[0].l4_proto = 17; d[0].flags = VPCSUM_F_IP | VPCSUM_F_L4;
    d[1].l3_off = 2048 + 14; d[1].l3_len = 0x40; d[1].l4_off = 20; d[1].l3_ver = 4; d[1].l4_proto = 6; d[1].flags = VPCSUM_F_IP | VPCSUM_F_L4;

    CHECK(vpcsum_abi_version() == VPCSUM_ABI_VERSION, "abi");
    vpcsum_ctx_t* ctx = nullptr;
    CHECK(vpcsum_ctx_create(0, 1 << 20, 64, &ctx) == 0, "ctx_create: %s", vpcsum_last_error());
    uint32_t out[2] = {0, 0};
    uint8_t st[2] = {0, 0};
    uint64_t t = 0;
    CHECK(vpcsum_ctx_submit(ctx, arena.data(), arena.size(), d, 2, out, st, VPCSUM_MODE_VERIFY, &t) == 0, "submit: %s", vpcsum_last_error());
    CHECK(vpcsum_ctx_wait(ctx, t) == 0, "wait: %s", vpcsum_last_error());
    CHECK((out[0] & 0xffff) == 0x7f41 && (out[0] >> 16) == 0xdf0d, "udp %08x", out[0]);
    CHECK((out[1] & 0xffff) == 0x87e4 && (out[1] >> 16) == 0xf3ff, "syn %08x", out[1]);
    CHECK(st[0] == (VPCSUM_S_DONE | VPCSUM_S_IP_OK | VPCSUM_S_L4_OK), "status0 %02x", st[0]);
    CHECK(st[1] == (VPCSUM_S_DONE | VPCSUM_S_IP_OK | VPCSUM_S_L4_OK), "status1 %02x", st[1]);

    // error path: capacity exceeded -> -1 + message
    CHECK(vpcsum_ctx_submit(ctx, arena.data(), arena.size(), d, 1000, out, st, 0, &t) < 0, "expected failure");
    CHECK(strstr(vpcsum_last_error(), "capacity") != nullptr, "msg %s", vpcsum_last_error());
    vpcsum_ctx_destroy(ctx);

    // PNI entry points (what io.vproxy.vpcsum.VPCsum downcalls)
    PNIEnv_vpcsum_long envl;
    memset(&envl, 0, sizeof(envl));
    CHECK(Java_io_vproxy_vpcsum_VPCsum_create(&envl, 0, 1 << 20, 64) == 0, "pni create");
    int64_t h = envl.return_;
    memset(arena.data() + 14 + 10, 0, 2);       // dirty the IP checksum; write mode recomputes it
    memset(&envl, 0, sizeof(envl));
    CHECK(Java_io_vproxy_vpcsum_VPCsum_submit(&envl, h, arena.data(), (int64_t)arena.size(), d, 2, out, st, VPCSUM_MODE_WRITE) == 0, "pni submit");
    PNIEnv_vpcsum_void envv;
    memset(&envv, 0, sizeof(envv));
    CHECK(Java_io_vproxy_vpcsum_VPCsum_waitFor(&envv, h, envl.return_) == 0, "pni wait");
    CHECK(arena[14 + 10] == 0x7f && arena[14 + 11] == 0x41, "in-place IP checksum %02x%02x", arena[24], arena[25]);
    // registered umem + low-latency service grid (what GpuCsumBatch sets up)
    memset(&envv, 0, sizeof(envv));
    CHECK(Java_io_vproxy_vpcsum_VPCsum_registerArena(&envv, h, arena.data(), (int64_t)arena.size()) == 0, "pni register");
    CHECK(Java_io_vproxy_vpcsum_VPCsum_setService(&envv, h, 5000) == 0, "pni setService");
    for (int rep = 0; rep < 3; ++rep) {
        memset(arena.data() + 14 + 10, 0, 2);
        memset(arena.data() + 2048 + 14 + 20 + 16, 0, 2);
        memset(&envl, 0, sizeof(envl));
        CHECK(Java_io_vproxy_vpcsum_VPCsum_submit(&envl, h, arena.data(), (int64_t)arena.size(), d, 2, out, st, VPCSUM_MODE_WRITE) == 0, "svc submit");
        CHECK(Java_io_vproxy_vpcsum_VPCsum_waitFor(&envv, h, envl.return_) == 0, "svc wait");
        CHECK(arena[24] == 0x7f && arena[25] == 0x41, "svc IP checksum %02x%02x", arena[24], arena[25]);
        CHECK(arena[2048 + 14 + 36] == 0xf3 && arena[2048 + 14 + 37] == 0xff, "svc TCP checksum");
    }
    uint64_t sb = 0;
    CHECK(vpcsum_ctx_stats((vpcsum_ctx_t*)(intptr_t)h, &sb, nullptr) == 0 && sb == 3, "service batches %llu", (unsigned long long)sb);
    CHECK(Java_io_vproxy_vpcsum_VPCsum_setService(&envv, h, -1) == -1, "negative idle must throw");
    CHECK(Java_io_vproxy_vpcsum_VPCsum_setService(&envv, h, 0) == 0, "pni service off");
    // NAT through the PNI entry (SwitchUtils.applyNat for a batch): setSrcPort(121) + setDst on
    // both frames, zero-copy on the registered arena and staged from a pageable copy; the frames
    // must verify afterwards (sums updated as Java's recompute leaves them)
    vpcsum_nat_t rw[2];
    memset(rw, 0, sizeof(rw));
    for (int i = 0; i < 2; ++i) {
        rw[i].sport[1] = 121;
        rw[i].dst[0] = 1; rw[i].dst[1] = 2; rw[i].dst[2] = 3; rw[i].dst[3] = 4;
        rw[i].mask = VPCSUM_NAT_SPORT | VPCSUM_NAT_DST;
    }
    std::vector<uint8_t> copy(arena);
    for (int mode = 0; mode < 2; ++mode) {
        for (int staged = 0; staged < 2; ++staged) {
            uint8_t* a = staged ? copy.data() : arena.data();
            memset(&envl, 0, sizeof(envl));
            CHECK(Java_io_vproxy_vpcsum_VPCsum_natSubmit(&envl, h, a, (int64_t)arena.size(), d, rw, 2, st, mode) == 0, "pni natSubmit");
            CHECK(Java_io_vproxy_vpcsum_VPCsum_waitFor(&envv, h, envl.return_) == 0, "nat wait");
            CHECK(st[0] == VPCSUM_S_DONE && st[1] == VPCSUM_S_DONE, "nat status %02x %02x", st[0], st[1]);
            CHECK(a[14 + 20 + 1] == 121 && a[2048 + 14 + 20 + 1] == 121 && a[14 + 16] == 1, "nat bytes");
            memset(&envl, 0, sizeof(envl));
            CHECK(Java_io_vproxy_vpcsum_VPCsum_submit(&envl, h, a, (int64_t)arena.size(), d, 2, out, st, VPCSUM_MODE_VERIFY) == 0, "verify");
            CHECK(Java_io_vproxy_vpcsum_VPCsum_waitFor(&envv, h, envl.return_) == 0, "verify wait");
            CHECK(st[0] == (VPCSUM_S_DONE | VPCSUM_S_IP_OK | VPCSUM_S_L4_OK) && st[1] == st[0], "after nat %02x %02x", st[0], st[1]);
        }
    }
    // RX parse with flow tuples through the PNI entry (TcpInput / UdpInput's conntrack key) on the
    // NAT'ed frames of the registered arena: dst 1.2.3.4 and source port 121 on both, SYN on the TCP one
    uint64_t foff[2] = {0, 2048};
    uint32_t flen[2] = {(uint32_t)udp.size(), (uint32_t)syn.size()};
    vpcsum_desc_t pd[2];
    vpcsum_tuple_t tu[2];
    memset(&envl, 0, sizeof(envl));
    CHECK(Java_io_vproxy_vpcsum_VPCsum_parseFrames(&envl, h, arena.data(), (int64_t)arena.size(), foff, flen, 2, pd, st, tu) == 0,
          "pni parseFrames");
    CHECK(Java_io_vproxy_vpcsum_VPCsum_waitFor(&envv, h, envl.return_) == 0, "parse wait");
    CHECK(st[0] == 0 && st[1] == 0, "parse status %02x %02x", st[0], st[1]);
    CHECK(pd[0].l3_off == 14 && pd[0].l3_len == 0x59 && pd[0].l4_proto == 17 && pd[1].l3_off == 2048 + 14 && pd[1].l4_proto == 6,
          "parsed descriptors");
    for (int i = 0; i < 2; ++i) {
        CHECK(tu[i].l3_ver == 4 && tu[i].dst[0] == 1 && tu[i].dst[3] == 4 && tu[i].sport[0] == 0 && tu[i].sport[1] == 121,
              "tuple %d", i);
    }
    CHECK(tu[0].src[0] == 0xc0 && tu[0].dport[0] == 0xc9 && tu[0].dport[1] == 0x14 && tu[0].tcp_flags == 0, "udp tuple");
    CHECK(tu[1].src[0] == 0x0a && tu[1].dport[0] == 0x01 && tu[1].dport[1] == 0xbb && tu[1].tcp_flags == 0x02, "syn tuple");
    memset(&envl, 0, sizeof(envl));
    CHECK(Java_io_vproxy_vpcsum_VPCsum_create(&envl, 0, -1, 64) == -1, "pni bad args");
    CHECK(envl.ex.type && strcmp(envl.ex.type, "java.lang.IllegalArgumentException") == 0, "ex type");
    Java_io_vproxy_vpcsum_VPCsum_close(&envv, h);
    printf("capi ok\n");
    return 0;
}
