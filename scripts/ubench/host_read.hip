// PCIe ceiling for the zero-copy host path (hfv_verify_records_host on a registered ring):
// how fast can a kernel read 2^20 64-byte records that lie in registered host memory, for
// the access shapes the verify kernel could use?
//   pattern 0: one lane per record, 8 B at +40 and 12 B at +48 (what k_verify_records does)
//   pattern 1: two lanes per record, 16 B each over bytes 32..63 (one 32 B sector per record)
//   pattern 2: four lanes per record, 16 B each over the whole 64 B record
//   dma:       hipMemcpyAsync of the whole ring to device memory (the staged alternative)
// Prints records/s and PCIe payload GB/s for each.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int PAT>
__global__ __launch_bounds__(1024) void k_host_read(const uint8_t *__restrict__ recs, size_t n, uint32_t *out)
{
    uint32_t acc = 0;
    constexpr int LPR = PAT == 0 ? 1 : PAT == 1 ? 2 : 4;   // lanes per record
    const size_t total = n * LPR;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / LPR, c = i % LPR;
        const uint8_t *p = recs + r * 64;
        if constexpr (PAT == 0) {
            u32x2 a = __builtin_nontemporal_load((const u32x2 *)(p + 40));
            u32x3 b = __builtin_nontemporal_load((const u32x3 *)(p + 48));
            acc ^= a.x ^ a.y ^ b.x ^ b.y ^ b.z;
        } else if constexpr (PAT == 1) {
            u32x4 v = __builtin_nontemporal_load((const u32x4 *)(p + 32 + 16 * c));
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        } else {
            u32x4 v = __builtin_nontemporal_load((const u32x4 *)(p + 16 * c));
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

template <int PAT>
static void run(const char *mem, const uint8_t *d, size_t n, uint32_t *out, int grid)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    k_host_read<PAT><<<grid, 1024>>>(d, n, out);
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0;
    const int reps = 10;
    for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(e0));
        k_host_read<PAT><<<grid, 1024>>>(d, n, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        sum += ms;
    }
    const double payload = PAT == 0 ? 20.0 : PAT == 1 ? 32.0 : 64.0;
    printf("{\"mem\": \"%s\", \"pattern\": %d, \"grid\": %d, \"ms_best\": %.4f, \"ms_mean\": %.4f, \"mrec_s\": %.1f, "
           "\"payload_GBs\": %.2f}\n",
           mem, PAT, grid, best, sum / reps, n / (best * 1e-3) / 1e6, n * payload / (best * 1e-3) / 1e9);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main()
{
    const size_t n = (size_t)1 << 20, bytes = n * 64;
    int dev, cus;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    uint32_t *out;
    CK(hipMalloc(&out, 4));
    void *dbuf;
    CK(hipMalloc(&dbuf, bytes));
    // registered pageable allocation (what hfv_host_register does) and hipHostMalloc
    uint8_t *reg = (uint8_t *)aligned_alloc(4096, bytes);
    memset(reg, 1, bytes);
    CK(hipHostRegister(reg, bytes, hipHostRegisterMapped));
    uint8_t *dreg;
    CK(hipHostGetDevicePointer((void **)&dreg, reg, 0));
    uint8_t *pin;
    CK(hipHostMalloc((void **)&pin, bytes, hipHostMallocMapped));
    memset(pin, 1, bytes);
    uint8_t *dpin;
    CK(hipHostGetDevicePointer((void **)&dpin, pin, 0));
    for (int g : {cus, 4 * cus}) {
        run<0>("registered", dreg, n, out, g);
        run<1>("registered", dreg, n, out, g);
        run<2>("registered", dreg, n, out, g);
        run<0>("hostmalloc", dpin, n, out, g);
        run<1>("hostmalloc", dpin, n, out, g);
        run<2>("hostmalloc", dpin, n, out, g);
    }
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 4; ++i) {
        CK(hipEventRecord(e0, s));
        CK(hipMemcpyAsync(dbuf, reg, bytes, hipMemcpyHostToDevice, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"mem\": \"registered\", \"dma_h2d_ms\": %.4f, \"mrec_s\": %.1f, \"GBs\": %.2f}\n", ms,
               n / (ms * 1e-3) / 1e6, bytes / (ms * 1e-3) / 1e9);
    }
    CK(hipHostUnregister(reg));
    free(reg);
    CK(hipHostFree(pin));
    CK(hipFree(dbuf));
    CK(hipFree(out));
    return 0;
}
