// A host allocation that fails inside a C-ABI entry point returns -1 with a message instead of
// unwinding a C++ exception into the (C / JVM) caller (tests/test_lib_cpu.py; no GPU needed: the
// group's bookkeeping is allocated before any device call).  This program replaces the global
// operator new, which libvpcsum.so's allocations resolve to, and makes it fail on demand.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

#include "vpcsum.h"

static bool g_fail_new = false;

void* operator new(std::size_t n) {
    if (g_fail_new) throw std::bad_alloc();
    void* p = std::malloc(n ? n : 1);
    if (!p) throw std::bad_alloc();
    return p;
}
void operator delete(void* p) noexcept { std::free(p); }
void operator delete(void* p, std::size_t) noexcept { std::free(p); }

int main() {
    const int devices[1] = {0};
    vpcsum_group_t* g = nullptr;
    g_fail_new = true;
    const int rc = vpcsum_group_create_list(devices, 1, 1 << 20, 1024, &g);
    g_fail_new = false;
    if (rc != -1 || g != nullptr) {
        std::printf("expected -1 and no group, got %d\n", rc);
        return 1;
    }
    if (!std::strstr(vpcsum_last_error(), "out of host memory")) {
        std::printf("unexpected message: %s\n", vpcsum_last_error());
        return 1;
    }
    std::printf("alloc failure returned -1: %s\n", vpcsum_last_error());
    return 0;
}
