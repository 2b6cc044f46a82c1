// atomic_claim.hip -- cost of claiming work through a device-scope global atomic counter, the
// building block of cross-block work stealing for the resident service's tail: one lane per
// wave of every block does ITERS fetch-and-adds (with return, each one waiting for the previous,
// as a tile claim would) on counter (block % C); reports ns per claim per wave and claims per
// second over the chip, for C = 1 (one counter), 8 (per XCD) and 256 (per block).
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ITERS = 256;

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void kclaim(uint32_t *ctr, uint32_t nctr, uint32_t *out)
{
    uint32_t acc = 0;
    if ((threadIdx.x & 63) == 0) {
        uint32_t *c = ctr + (blockIdx.x % nctr) * 32;   // one counter per 128-byte line
        for (int i = 0; i < ITERS; ++i)
            acc += __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (acc == 0xdeadbeef) out[0] = acc;
}

template <int WAVES>
static void run(int ncu, uint32_t nctr, uint32_t *ctr, uint32_t *out)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kclaim<WAVES>, dim3(ncu), dim3(WAVES * 64), 0, 0, ctr, nctr, out);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(kclaim<WAVES>, dim3(ncu), dim3(WAVES * 64), 0, 0, ctr, nctr, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double claims = (double)ncu * WAVES * ITERS;
    printf("counters %3u, waves/block %2d: %8.1f us, %7.1f ns per claim per wave, %7.1f M claims/s chip-wide\n", nctr,
           WAVES, best * 1e3, best * 1e6 / ITERS, claims / (best * 1e-3) / 1e6);
}

int main()
{
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int ncu = p.multiProcessorCount;
    printf("%s, %d CUs\n", p.gcnArchName, ncu);
    uint32_t *ctr, *out;
    (void)hipMalloc(&ctr, 1024 * 128);
    (void)hipMalloc(&out, 64);
    (void)hipMemset(ctr, 0, 1024 * 128);
    for (uint32_t c : {1u, 8u, 256u}) {
        run<1>(ncu, c, ctr, out);
        run<16>(ncu, c, ctr, out);
    }
    (void)hipFree(ctr);
    (void)hipFree(out);
    return 0;
}
