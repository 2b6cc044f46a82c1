// valu_rate.hip -- issue rate of the VALU ops the verify kernels use (v_bitop3_b32, v_xor_b32,
// v_perm_b32, v_alignbit_b32, v_fma_f32 for reference) and of ds_read_b32, on gfx950.
// Each lane runs 8 independent chains; every CU is filled with 8 waves per SIMD.  Cycles per
// wave-instruction per SIMD = (s_memtime delta) / (instructions per wave * waves per SIMD).
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ITERS = 2048;
constexpr int TABW = 4096;   // 16 KiB: up to 8 blocks per CU

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t *out, uint64_t *clk, uint32_t seed)
{
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + 1) + i;
    uint32_t b = seed ^ threadIdx.x, c = seed + 7;
    float f[8];
    for (int i = 0; i < 8; ++i) f[i] = (float)a[i];
    __shared__ uint32_t tab[TABW];
    for (int i = threadIdx.x; i < TABW; i += 256) tab[i] = (i * 2654435761u) & 0x3fff;
    __syncthreads();
    uint32_t lanebase = (threadIdx.x & 31) << 2;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if constexpr (OP == 0) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(c));
                if constexpr (OP == 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
                if constexpr (OP == 2) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
                if constexpr (OP == 3) asm volatile("v_alignbit_b32 %0, %0, %1, 16" : "+v"(a[i]) : "v"(b));
                if constexpr (OP == 4) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[i]) : "v"(b), "v"(c));
                if constexpr (OP == 6) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                if constexpr (OP == 7) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
                if constexpr (OP == 8) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(a[i]) : "v"(b));
                if constexpr (OP == 9) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a[i]));
                if constexpr (OP == 10) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
                if constexpr (OP == 12) asm volatile("v_alignbyte_b32 %0, %0, %1, 2" : "+v"(a[i]) : "v"(b));
                if constexpr (OP == 13) asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(a[i]));
                if constexpr (OP == 14) asm volatile("v_and_b32 %0, 0xff00, %0" : "+v"(a[i]));
            }
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= a[i] ^ __float_as_uint(f[i]);
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) clk[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}


// T-table-like lookups: 8 independent chains; each step builds an LDS byte address from byte 1
// of the chain value (OP 0: v_perm_b32; OP 1: v_mov_b32_sdwa into a register whose byte 0
// holds the lane bits) and XORs the looked-up word into the chain.
template <int OP>
__global__ __launch_bounds__(256) void kl(uint32_t *out, uint64_t *clk, uint32_t seed)
{
    __shared__ uint32_t tab[4096];   // 16 KiB, bank-replicated pattern: dword (x << 5) | (lane & 31) for x < 128
    for (int i = threadIdx.x; i < 4096; i += 256) tab[i] = (i * 2654435761u) & 0x7f7f7f7fu;
    __syncthreads();
    uint32_t a[8], ad[8];
    const uint32_t lanebits = (threadIdx.x & 31) << 2;
    const uint32_t sel = 0x0c0c0500u;   // byte0 <- lanebits byte0, byte1 <- a byte1
    for (int i = 0; i < 8; ++i) { a[i] = (seed * (threadIdx.x + 1) + i * 77) & 0x7f7f7f7fu; ad[i] = lanebits; }
    uint32_t vsel = sel;
    asm volatile("" : "+v"(vsel));
    uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                uint32_t addr;
                if constexpr (OP == 0) addr = __builtin_amdgcn_perm(a[i], lanebits, vsel);
                else {
                    asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1" : "+v"(ad[i]) : "v"(a[i]));
                    addr = ad[i];
                }
                uint32_t v = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(tab) + addr);
                a[i] = a[i] ^ v;
            }
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= a[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) clk[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int OP, bool LDS = false>
void run(const char *name, int blocks_per_cu, int ncu)
{
    int nb = ncu * blocks_per_cu;
    uint32_t *out;
    uint64_t *clk;
    (void)hipMalloc(&out, nb * 256 * 4);
    (void)hipMalloc(&clk, nb * 4 * 8);
    if (LDS) hipLaunchKernelGGL(kl<OP>, dim3(nb), dim3(256), 0, 0, out, clk, 3u); else hipLaunchKernelGGL(k<OP>, dim3(nb), dim3(256), 0, 0, out, clk, 3u);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    if (LDS) hipLaunchKernelGGL(kl<OP>, dim3(nb), dim3(256), 0, 0, out, clk, 5u); else hipLaunchKernelGGL(k<OP>, dim3(nb), dim3(256), 0, 0, out, clk, 5u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    uint64_t *h = new uint64_t[nb * 4];
    (void)hipMemcpy(h, clk, nb * 4 * 8, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < nb * 4; ++i) avg += h[i];
    avg /= nb * 4;
    double instr_per_wave = (double)ITERS * 32;
    int waves_per_simd = blocks_per_cu;   // 256 threads = 4 waves = 1 per SIMD per block
    double cyc = avg / (instr_per_wave * waves_per_simd);
    double rate = instr_per_wave * nb * 4 * 64 / (ms * 1e-3) / 1e12;   // (LDS kernels: lookups)
    printf("%-10s waves/SIMD %d: %.2f cycles per wave-instr per SIMD (s_memtime), %.1f T lane-ops/s, %.1f us\n", name,
           waves_per_simd, cyc, rate, ms * 1e3);
    delete[] h;
    hipFree(out);
    hipFree(clk);
}

int main()
{
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    int ncu = p.multiProcessorCount;
    printf("%s, %d CUs, clock %d kHz\n", p.gcnArchName, ncu, p.clockRate);
    for (int w : {4, 8}) {
        run<0>("bitop3", w, ncu);
        run<1>("xor", w, ncu);
        run<2>("perm", w, ncu);
        run<3>("alignbit", w, ncu);
        run<12>("alignbyte", w, ncu);
        run<4>("fma_f32", w, ncu);
        run<6>("mov_sdwa", w, ncu);
        run<7>("and_or", w, ncu);
        run<8>("lshl_or", w, ncu);
        run<9>("bfe_u32", w, ncu);
        run<10>("bfi", w, ncu);
        run<13>("lshrrev", w, ncu);
        run<14>("and_lit", w, ncu);
        run<0, true>("lds_perm", w, ncu);
        run<1, true>("lds_sdwa", w, ncu);
    }
    return 0;
}
