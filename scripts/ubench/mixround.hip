// mixround.hip -- does moving the last AES rounds' table lookups from LDS to the vector-memory
// path (L1-resident global T-tables) raise the per-CU packet rate of the verify loop?
// Every lane runs the verify kernel's round structure on a private state: rounds on the 4-table
// LDS layout (128 KiB, 32 lane copies, v_perm address, conflict-free), and the last G rounds
// (G = 0..3) from four 1 KiB global T-tables (global_load_dword, L1/L2 resident).  One 1024-thread
// block per CU, as the service grid.  Reports packets per CU-clock and per second.
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int TILES = 256;   // chains per lane

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

__shared__ uint32_t s_tab[32768];

template <int K>
__device__ __forceinline__ uint32_t lu(uint32_t w, uint32_t base, uint32_t sel)
{
    const uint32_t a = __builtin_amdgcn_perm(w, base, sel);
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(s_tab) + a);
}

typedef const __attribute__((address_space(1))) uint32_t *G1;
template <int K>
__device__ __forceinline__ uint32_t glu(uint32_t w, G1 t)
{
    return t[K * 256 + ((w >> (8 * K)) & 0xff)];
}

template <int G>
__global__ __launch_bounds__(1024) void kmix(uint32_t *out, const uint32_t *__restrict__ gtab, uint32_t seed, uint64_t *clk)
{
    for (int i = threadIdx.x; i < 32768; i += 1024) s_tab[i] = (i * 2654435761u) ^ (i >> 5);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t b0 = (lane & 31) << 2, b1 = b0 | 0x80u, b2 = b0 | 0x10000u, b3 = b1 | 0x10000u;
    uint32_t s0, s1, s2, s3;
    asm volatile("v_mov_b32 %0, 0x0c020400" : "=v"(s0));
    asm volatile("v_mov_b32 %0, 0x0c020500" : "=v"(s1));
    asm volatile("v_mov_b32 %0, 0x0c020600" : "=v"(s2));
    asm volatile("v_mov_b32 %0, 0x0c020700" : "=v"(s3));
    G1 gt = (G1)gtab;
    uint32_t acc = 0;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int t = 0; t < TILES; ++t) {
        uint32_t s[4] = {seed ^ threadIdx.x ^ t, seed * 3 + t, blockIdx.x + t * 7, acc};
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            uint32_t n[4];
            if (r < 10 - G) {
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    n[c] = xor3(xor3(lu<0>(s[c], b0, s0), lu<1>(s[(c + 1) & 3], b1, s1), lu<2>(s[(c + 2) & 3], b2, s2)),
                                lu<3>(s[(c + 3) & 3], b3, s3), seed + r);
            } else {
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    n[c] = xor3(xor3(glu<0>(s[c], gt), glu<1>(s[(c + 1) & 3], gt), glu<2>(s[(c + 2) & 3], gt)),
                                glu<3>(s[(c + 3) & 3], gt), seed + r);
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) s[c] = n[c];
        }
        acc ^= s[0] ^ s[1];
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 1024 + threadIdx.x] = acc;
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <int G>
void run(int ncu, const uint32_t *gtab)
{
    uint32_t *out;
    uint64_t *clk;
    (void)hipMalloc(&out, ncu * 1024 * 4);
    (void)hipMalloc(&clk, ncu * 8);
    hipLaunchKernelGGL(kmix<G>, dim3(ncu), dim3(1024), 0, 0, out, gtab, 3u, clk);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    uint64_t hc[1024];
    double cyc = 0;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(kmix<G>, dim3(ncu), dim3(1024), 0, 0, out, gtab, 5u + rep, clk);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) {
            best = ms;
            (void)hipMemcpy(hc, clk, ncu * 8, hipMemcpyDeviceToHost);
            cyc = 0;
            for (int i = 0; i < ncu; ++i) cyc += (double)hc[i];
            cyc /= ncu;
        }
    }
    double pk = (double)TILES * 1024 * ncu;
    // s_memtime counts at the shader clock on gfx950? report both: per s_memtime tick and per second
    printf("G=%d (LDS rounds %2d, global rounds %d): %.1f us, %.2f Gpkt/s, %.3f pkt per CU per memtime-tick (%.0f ticks)\n",
           G, 10 - G, G, best * 1e3, pk / (best * 1e-3) / 1e9, (double)TILES * 1024 / cyc, cyc);
    (void)hipFree(out);
    (void)hipFree(clk);
}

int main()
{
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    int ncu = p.multiProcessorCount;
    printf("%s, %d CUs\n", p.gcnArchName, ncu);
    uint32_t *gtab;
    (void)hipMalloc(&gtab, 4096);
    uint32_t h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = (i * 2654435761u) ^ 0x5a5a;
    (void)hipMemcpy(gtab, h, sizeof h, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; ++rep) {
        run<0>(ncu, gtab);
        run<1>(ncu, gtab);
        run<2>(ncu, gtab);
        run<3>(ncu, gtab);
    }
    (void)hipFree(gtab);
    return 0;
}
