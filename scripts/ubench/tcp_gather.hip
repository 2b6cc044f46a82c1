// tcp_gather.hip -- can the vector-memory path (TA/TCP, the per-CU L1) serve table lookups
// beside LDS?  The verify kernels are LDS-issue bound; if L1-resident
// gathers run concurrently with ds_read_b32, moving part of the lookups to global loads of a
// small L1-resident table raises the per-CU lookup rate.
// Each lane runs 8 independent chains; every step forms a table address from byte 1 of the
// chain value and XORs the looked-up word back in (the T-table access pattern).
// OP 0: all 8 chains from LDS (bank-replicated table, conflict-free);
// OP 1: all 8 chains global_load_dword from a 1 KiB table (8 x 128 B lines);
// OP 2: all 8 chains global_load_ubyte from a 256 B table;
// OP 3: 6 LDS + 2 global dword chains;  OP 4: 4 LDS + 4 global dword;  OP 5: 7 LDS + 1 global.
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ITERS = 1024;

template <int OP>
__global__ __launch_bounds__(256) void kg(uint32_t *out, const uint32_t *__restrict__ gtab, uint32_t seed)
{
    __shared__ uint32_t tab[4096];   // 16 KiB: dword (x << 5) | (lane & 31), x < 128
    for (int i = threadIdx.x; i < 4096; i += 256) tab[i] = (i * 2654435761u) & 0x7f7f7f7fu;
    __syncthreads();
    constexpr int NG = OP == 0 ? 0 : OP == 3 ? 2 : OP == 4 ? 4 : OP == 5 ? 1 : 8;
    uint32_t a[8];
    const uint32_t lanebits = (threadIdx.x & 31) << 2;
    uint32_t vsel = 0x0c0c0500u;
    asm volatile("" : "+v"(vsel));
    for (int i = 0; i < 8; ++i) a[i] = (seed * (threadIdx.x + 1) + i * 77) & 0x7f7f7f7fu;
    const uint8_t *gb = reinterpret_cast<const uint8_t *>(gtab);
#pragma unroll 1
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                uint32_t v;
                if (i < 8 - NG) {
                    uint32_t addr = __builtin_amdgcn_perm(a[i], lanebits, vsel);
                    v = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(tab) + addr);
                } else if constexpr (OP == 2) {
                    v = gb[(a[i] >> 8) & 0xff];
                } else {
                    v = *reinterpret_cast<const uint32_t *>(gb + ((a[i] >> 6) & 0x3fc));
                }
                a[i] = a[i] ^ v;
            }
        }
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= a[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
void run(const char *name, int blocks_per_cu, int ncu, const uint32_t *gtab)
{
    int nb = ncu * blocks_per_cu;
    uint32_t *out;
    (void)hipMalloc(&out, nb * 256 * 4);
    hipLaunchKernelGGL(kg<OP>, dim3(nb), dim3(256), 0, 0, out, gtab, 3u);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(kg<OP>, dim3(nb), dim3(256), 0, 0, out, gtab, 5u + rep);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    double lookups = (double)ITERS * 32 * nb * 256;
    printf("%-14s waves/SIMD %d: %.2f T lookups/s (%.1f per CU-clock at 2.4 GHz), %.1f us\n", name, blocks_per_cu,
           lookups / (best * 1e-3) / 1e12, lookups / (best * 1e-3) / ncu / 2.4e9, best * 1e3);
    (void)hipDeviceSynchronize();
    hipFree(out);
}

int main()
{
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    int ncu = p.multiProcessorCount;
    printf("%s, %d CUs\n", p.gcnArchName, ncu);
    uint32_t *gtab;
    (void)hipMalloc(&gtab, 4096);
    uint32_t h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = (i * 2654435761u) & 0x7f7f7f7fu;
    (void)hipMemcpy(gtab, h, sizeof h, hipMemcpyHostToDevice);
    for (int w : {4, 8}) {
        run<0>("lds8", w, ncu, gtab);
        run<1>("glob_dword8", w, ncu, gtab);
        run<2>("glob_ubyte8", w, ncu, gtab);
        run<5>("lds7+glob1", w, ncu, gtab);
        run<3>("lds6+glob2", w, ncu, gtab);
        run<4>("lds4+glob4", w, ncu, gtab);
    }
    hipFree(gtab);
    return 0;
}
