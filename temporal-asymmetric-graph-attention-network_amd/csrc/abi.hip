// Library-level C-ABI entry points: error string, version, device query, RNG.
#include <stdarg.h>

#include "common.cuh"

namespace tagan {
static thread_local char g_err[512] = "";
static const uint64_t* g_seed_ctr = nullptr;

const uint64_t* seed_counter() { return g_seed_ctr; }

namespace {
__global__ void k_counter_step(uint64_t* c) {
    if (threadIdx.x == 0) c[0] = c[0] + 1;
}
}  // namespace

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

int tagan_debug_build(void) {
#ifdef TAGAN_DEBUG
    return 1;
#else
    return 0;
#endif
}

int tagan_device_arch(char* buf, int len) {
    TAGAN_REQUIRE(buf != nullptr && len > 0, TAGAN_ERR_ARG, "tagan_device_arch: null buffer");
    int dev = 0;
    TAGAN_CHECK_HIP(hipGetDevice(&dev), "hipGetDevice");
    hipDeviceProp_t p;
    TAGAN_CHECK_HIP(hipGetDeviceProperties(&p, dev), "hipGetDeviceProperties");
    snprintf(buf, (size_t)len, "%s", p.gcnArchName);
    return TAGAN_OK;
}

void tagan_set_seed_counter(const uint64_t* counter) { tagan::g_seed_ctr = counter; }

int tagan_seed_counter_step(uint64_t* counter, void* stream) {
    TAGAN_REQUIRE(counter != nullptr, TAGAN_ERR_ARG, "seed_counter_step: null counter");
    tagan::k_counter_step<<<1, 64, 0, tagan::as_stream(stream)>>>(counter);
    TAGAN_CHECK_LAUNCH("seed_counter_step");
    return TAGAN_OK;
}

float tagan_uniform(uint64_t seed, uint64_t stream, uint32_t counter) {
    return tagan::drop_u(tagan::drop_key(seed, stream), counter);
}

}  // extern "C"
