// Library-level C-ABI entry points: error string, version, device query, RNG.
#include <stdarg.h>

#include "common.cuh"

namespace tagan {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace tagan

extern "C" {

const char* tagan_last_error(void) { return tagan::g_err; }

int tagan_version(void) { return 1; }

int tagan_device_arch(char* buf, int len) {
    TAGAN_REQUIRE(buf != nullptr && len > 0, TAGAN_ERR_ARG, "tagan_device_arch: null buffer");
    int dev = 0;
    TAGAN_CHECK_HIP(hipGetDevice(&dev), "hipGetDevice");
    hipDeviceProp_t p;
    TAGAN_CHECK_HIP(hipGetDeviceProperties(&p, dev), "hipGetDeviceProperties");
    snprintf(buf, (size_t)len, "%s", p.gcnArchName);
    return TAGAN_OK;
}

float tagan_uniform(uint64_t seed, uint64_t stream, uint32_t counter) {
    return tagan::drop_u(tagan::drop_key(seed, stream), counter);
}

}  // extern "C"
