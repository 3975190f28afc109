/* PNIEnv layout of include/vpcsum.h against the PNI runtime's (base/src/main/c-generated/pni.h:15-73
 * in vproxy): PNIException {char* type; char message[4096]; int32_t errno_}, then a 16-byte return
 * union.  The generated Java side hands the runtime's PNIEnv memory straight to these entry points,
 * so every offset must match.  Compiled with gcc by tests/test_lib_cpu.py; the run checks that a
 * throw through the PNI entry points fills type, message and errno_ (argument errors only: no GPU). */
#include <errno.h>
#include <stddef.h>
#include <stdio.h>
#include <string.h>
#include "vpcsum.h"

_Static_assert(offsetof(PNIException_vpcsum, type) == 0, "ex.type");
_Static_assert(offsetof(PNIException_vpcsum, message) == 8, "ex.message");
_Static_assert(offsetof(PNIException_vpcsum, errno_) == 8 + 4096, "ex.errno_");
_Static_assert(sizeof(PNIException_vpcsum) == 4112, "PNIException size (errno_ + 4 B padding)");
_Static_assert(offsetof(PNIEnv_vpcsum_long, return_) == 4112 && sizeof(PNIEnv_vpcsum_long) == 4128, "PNIEnv_long");
_Static_assert(offsetof(PNIEnv_vpcsum_int, return_) == 4112 && sizeof(PNIEnv_vpcsum_int) == 4128, "PNIEnv_int");
_Static_assert(sizeof(PNIEnv_vpcsum_void) == 4128, "PNIEnv_void");
_Static_assert(sizeof(vpcsum_desc_t) == 16 && sizeof(vpcsum_nat4_t) == 16 && sizeof(vpcsum_nat_t) == 48, "entries");
_Static_assert(offsetof(vpcsum_nat_t, mask) == 36 && offsetof(vpcsum_nat_t, ttl) == 37, "vpcsum_nat_t");

int main(void) {
    PNIEnv_vpcsum_long env;
    memset(&env, 0, sizeof(env));
    if (Java_io_vproxy_vpcsum_VPCsum_create(&env, 0, -1, 64) != -1) return 1;
    if (!env.ex.type || strcmp(env.ex.type, "java.lang.IllegalArgumentException") != 0) return 2;
    if (env.ex.errno_ != EINVAL || strstr(env.ex.message, "positive") == NULL) return 3;
    memset(&env, 0, sizeof(env));
    if (Java_io_vproxy_vpcsum_VPCsum_natSubmit(&env, 0, NULL, 0, NULL, NULL, -1, NULL, 0) != -1) return 4;
    if (env.ex.errno_ != EINVAL) return 5;
    printf("pni layout ok\n");
    return 0;
}
