// Can the host CPU store into fine-grained device memory (large-BAR mapping), and how fast
// does a GPU wave see it?  Probe for the resident service's descriptor ring placement.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <chrono>

__global__ void k_echo(volatile uint64_t *ring, uint64_t *out, int iters)
{
    // wait for the host to store i into ring[0], then answer i into out[0] (host memory)
    for (int i = 1; i <= iters; ++i) {
        uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load((uint64_t *)ring, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != (uint64_t)i) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) return;   // 2 s
            __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(out, (uint64_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

int main()
{
    for (int mode = 0; mode < 2; ++mode) {
        uint64_t *ring = nullptr;
        hipError_t e;
        if (mode == 0) e = hipExtMallocWithFlags((void **)&ring, 4096, hipDeviceMallocFinegrained);
        else e = hipHostMalloc((void **)&ring, 4096, hipHostMallocMapped | hipHostMallocCoherent);
        printf("mode %d (%s) alloc: %s\n", mode, mode ? "host pinned" : "VRAM fine-grained", hipGetErrorString(e));
        if (e != hipSuccess) continue;
        hipPointerAttribute_t attr;
        if (hipPointerGetAttributes(&attr, ring) == hipSuccess)
            printf("  hostPointer %p devicePointer %p\n", attr.hostPointer, attr.devicePointer);
        if (mode == 0) {
            // the host touches it only if the runtime mapped it into the host address space
            if (!attr.hostPointer) { printf("  not host-mapped\n"); continue; }
        }
        volatile uint64_t *h = (volatile uint64_t *)(mode == 0 ? attr.hostPointer : ring);
        h[0] = 0;
        uint64_t *out = nullptr;
        hipHostMalloc((void **)&out, 64, hipHostMallocMapped | hipHostMallocCoherent);
        *(volatile uint64_t *)out = 0;
        const int iters = 2000;
        hipLaunchKernelGGL(k_echo, dim3(1), dim3(64), 0, 0, (volatile uint64_t *)ring, out, iters);
        auto t0 = std::chrono::steady_clock::now();
        int ok = 1;
        for (int i = 1; i <= iters && ok; ++i) {
            h[0] = i;
            auto w0 = std::chrono::steady_clock::now();
            while (*(volatile uint64_t *)out != (uint64_t)i) {
                if (std::chrono::steady_clock::now() - w0 > std::chrono::seconds(3)) { ok = 0; break; }
            }
        }
        double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        hipDeviceSynchronize();
        printf("  round trips ok=%d: %.2f us per host-store -> GPU-see -> GPU-store -> host-see\n", ok, us / iters);
    }
    return 0;
}
