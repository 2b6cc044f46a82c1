// hfv_test_kernels.hip -- kernels only the test build of the library (lib/libscionhfv_test.so,
// -DHFV_TEST_HOOKS) links: the product library exports none of them.
#include <hip/hip_runtime.h>

#include "hfv_internal.h"

namespace hfv {

// hfv_debug_publish_delay: hold a stream for `us` microseconds, bounded by the 100 MHz
// s_memrealtime, so a test can queue a key-table publish behind it deterministically.
__global__ void k_debug_spin(uint32_t us)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * us) __builtin_amdgcn_s_sleep(8);
}

int launch_debug_spin(void *stream, uint32_t us)
{
    if (us > 1000000u) us = 1000000u;
    hipLaunchKernelGGL(k_debug_spin, dim3(1), dim3(64), 0, (hipStream_t)stream, us);
    return (int)hipGetLastError();
}

}  // namespace hfv
