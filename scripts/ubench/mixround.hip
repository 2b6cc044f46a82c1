// mixround.hip -- does moving the last AES rounds' table lookups from LDS to the vector-memory
// path (L1-resident global T-tables) raise the per-CU packet rate of the verify loop?
// Every lane runs the verify kernel's round structure on a private state: rounds on the 4-table
// LDS layout (128 KiB, 32 lane copies, v_perm address, conflict-free), and the last G rounds
// (G = 0..3) from four 1 KiB global T-tables (global_load_dword, L1/L2 resident).  One 1024-thread
// block per CU, as the service grid.  Reports packets per CU-clock and per second.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

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

// MEM = 1 / 2: every tile also streams the verify kernel's record words (8 B at +40, 8 B at +48,
// 4 B at +56 of a 64 B record, one record per lane, consecutive records per wave) from a buffer
// far larger than the Infinity Cache, loaded MEM tiles ahead of their use and folded into the
// state: what the HBM stream costs the LDS-bound round loop, and whether a deeper prefetch helps.
template <int G, int MEM = 0>
__global__ __launch_bounds__(1024) void kmix(uint32_t *out, const uint32_t *__restrict__ gtab, uint32_t seed, uint64_t *clk,
                                             const uint8_t *__restrict__ recs = nullptr, uint64_t nrec = 0)
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
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    typedef const __attribute__((address_space(1))) u2 *P2;
    typedef const __attribute__((address_space(1))) uint32_t *P1;
    const uint64_t nw = (uint64_t)gridDim.x * 16, w = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
    auto ld = [&](int t, uint32_t r[5]) {
        const uint64_t i = ((w + (uint64_t)t * nw) * 64 + lane) & (nrec - 1);
        const __attribute__((address_space(1))) uint8_t *p = (const __attribute__((address_space(1))) uint8_t *)recs + i * 64;
        const u2 a = *reinterpret_cast<P2>(p + 40), b = *reinterpret_cast<P2>(p + 48);
        r[0] = a.x; r[1] = a.y; r[2] = b.x; r[3] = b.y; r[4] = *reinterpret_cast<P1>(p + 56);
    };
    uint32_t q0[5] = {0, 0, 0, 0, 0}, q1[5] = {0, 0, 0, 0, 0};
    if constexpr (MEM >= 1) ld(0, q0);
    if constexpr (MEM >= 2) ld(1, q1);
    uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int t = 0; t < TILES; ++t) {
        uint32_t s[4] = {seed ^ threadIdx.x ^ t, seed * 3 + t, blockIdx.x + t * 7, acc};
        if constexpr (MEM >= 1) {
            s[0] ^= q0[0] ^ q0[4]; s[1] ^= q0[1]; s[2] ^= q0[2]; s[3] ^= q0[3];
            if constexpr (MEM == 1) {
                ld(t + 1, q0);
            } else {
#pragma unroll
                for (int j = 0; j < 5; ++j) q0[j] = q1[j];
                ld(t + 2, q1);
            }
        }
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

template <int G, int MEM = 0>
void run(int ncu, const uint32_t *gtab, const uint8_t *recs = nullptr, uint64_t nrec = 0)
{
    uint32_t *out;
    uint64_t *clk;
    (void)hipMalloc(&out, ncu * 1024 * 4);
    (void)hipMalloc(&clk, ncu * 8);
    hipLaunchKernelGGL((kmix<G, MEM>), dim3(ncu), dim3(1024), 0, 0, out, gtab, 3u, clk, recs, nrec);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    uint64_t hc[1024];
    double cyc = 0;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((kmix<G, MEM>), dim3(ncu), dim3(1024), 0, 0, out, gtab, 5u + rep, clk, recs, nrec);
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
    printf("MEM=%d G=%d (LDS rounds %2d, global rounds %d): %.1f us, %.2f Gpkt/s, %.3f pkt per CU per memtime-tick (%.0f ticks)\n",
           MEM, G, 10 - G, G, best * 1e3, pk / (best * 1e-3) / 1e9, (double)TILES * 1024 / cyc, cyc);
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
    uint8_t *recs;
    const uint64_t nrec = 1ull << 24;   // 1 GiB of 64 B records
    (void)hipMalloc(&recs, nrec * 64);
    (void)hipMemset(recs, 0x5a, nrec * 64);
    const bool memonly = getenv("MIX_MEM") != nullptr;
    for (int rep = 0; rep < 2; ++rep) {
        if (!memonly) {
            run<0>(ncu, gtab);
            run<1>(ncu, gtab);
            run<2>(ncu, gtab);
            run<3>(ncu, gtab);
        }
        run<0, 0>(ncu, gtab, recs, nrec);
        run<0, 1>(ncu, gtab, recs, nrec);
        run<0, 2>(ncu, gtab, recs, nrec);
    }
    (void)hipFree(recs);
    (void)hipFree(gtab);
    return 0;
}
