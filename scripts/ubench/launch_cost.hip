// launch_cost.hip -- host cost of one kernel launch and launch->sync round trip on gfx950 for
// the shapes the service uses (256 x 1024 threads, ~147 KiB static LDS, 9 arguments), with and
// without the dispatch timing events of hipExtLaunchKernel, against a 1-block empty kernel.
// Prints median microseconds over 200 launches each (after 20 untimed).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

__global__ void k_empty(int *p) { if (p && threadIdx.x == 9999) p[0] = 1; }

__global__ __launch_bounds__(1024) void k_lds(int *p, const int *q, void *a, void *b, unsigned c, unsigned d,
                                                unsigned long e, unsigned long f)
{
    __shared__ unsigned big[36864];   // 144 KiB
    big[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (p && big[(threadIdx.x + 1) & 1023] == 99999u) p[0] = 1;
}

// the same kernel with a by-value argument struct of N bytes (the service's SvcArgs carries up
// to kSvcInline = 64 inline descriptors: ~2.3 KiB)
template <int N>
struct BigArg {
    unsigned long w[N / 8];
};
template <int N>
__global__ __launch_bounds__(1024) void k_lds_arg(const BigArg<N> a)
{
    __shared__ unsigned big[36864];   // 144 KiB
    big[threadIdx.x] = (unsigned)a.w[threadIdx.x % (N / 8)];
    __syncthreads();
    if (big[(threadIdx.x + 1) & 1023] == 99999u) big[0] = 1;
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

template <class F>
static void measure(const char *name, F launch, hipStream_t s)
{
    for (int i = 0; i < 20; ++i) { launch(); (void)hipStreamSynchronize(s); }
    std::vector<double> call, rt;
    for (int i = 0; i < 200; ++i) {
        (void)hipDeviceSynchronize();
        auto t0 = clk::now();
        launch();
        auto t1 = clk::now();
        (void)hipDeviceSynchronize();
        auto t2 = clk::now();
        call.push_back(us(t0, t1));
        rt.push_back(us(t0, t2));
    }
    std::sort(call.begin(), call.end());
    std::sort(rt.begin(), rt.end());
    printf("%-44s call median %6.1f us (p10 %5.1f p90 %5.1f)   launch->sync median %6.1f us (p10 %5.1f p90 %5.1f)\n",
           name, call[100], call[20], call[180], rt[100], rt[20], rt[180]);
}

int main()
{
    (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    int *p = nullptr;
    (void)hipMalloc(&p, 4096);
    measure("empty 1x64", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr); }, s);
    measure("empty 256x1024", [&] { hipLaunchKernelGGL(k_empty, dim3(256), dim3(1024), 0, s, nullptr); }, s);
    measure("lds144K 256x1024", [&] {
        hipLaunchKernelGGL(k_lds, dim3(256), dim3(1024), 0, s, nullptr, p, p, p, 1u, 2u, 3ul, 4ul);
    }, s);
    measure("lds144K 256x1024 hipExtLaunchKernel+events", [&] {
        hipExtLaunchKernelGGL(k_lds, dim3(256), dim3(1024), 0, s, e0, e1, 0u, nullptr, p, p, p, 1u, 2u, 3ul, 4ul);
    }, s);
    measure("lds144K 256x1024 hipExtLaunchKernel no ev", [&] {
        hipExtLaunchKernelGGL(k_lds, dim3(256), dim3(1024), 0, s, nullptr, nullptr, 0u, nullptr, p, p, p, 1u, 2u, 3ul, 4ul);
    }, s);
    BigArg<128> a128 = {};
    BigArg<1024> a1k = {};
    BigArg<2304> a2k = {};
    measure("lds144K struct arg 128 B, no ev", [&] {
        hipExtLaunchKernelGGL(k_lds_arg<128>, dim3(256), dim3(1024), 0, s, nullptr, nullptr, 0u, a128);
    }, s);
    measure("lds144K struct arg 1 KiB, no ev", [&] {
        hipExtLaunchKernelGGL(k_lds_arg<1024>, dim3(256), dim3(1024), 0, s, nullptr, nullptr, 0u, a1k);
    }, s);
    measure("lds144K struct arg 2.25 KiB, no ev", [&] {
        hipExtLaunchKernelGGL(k_lds_arg<2304>, dim3(256), dim3(1024), 0, s, nullptr, nullptr, 0u, a2k);
    }, s);
    measure("lds144K + hipEventRecord around", [&] {
        (void)hipEventRecord(e0, s);
        hipLaunchKernelGGL(k_lds, dim3(256), dim3(1024), 0, s, nullptr, p, p, p, 1u, 2u, 3ul, 4ul);
        (void)hipEventRecord(e1, s);
    }, s);
    return 0;
}
