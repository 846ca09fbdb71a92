/*
 * barbench.hip — cost of a workgroup barrier step in the detection kernels'
 * shape: one 1024-thread workgroup per CU (150 KB of dynamic LDS), 1024
 * workgroups, K steps of [an LDS write, barrier, an LDS read of another
 * wave's slot].  Prints cycles per step per workgroup (s_memtime of thread 0)
 * and the kernel time, for K = 0 and K = 64.
 *   hipcc --offload-arch=gfx950 -O3 tools/barbench.hip -o tools/barbench
 */
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(1024) void k_bar(int K, int work, unsigned long long *cyc, int *sink) {
    extern __shared__ int lds[];
    const int tid = threadIdx.x;
    int acc = tid;
    lds[tid] = tid;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < K; ++k) {
        for (int w = 0; w < work; ++w) acc = acc * 1664525 + 1013904223;   /* dependent VALU between barriers */
        lds[tid] = acc;
        __syncthreads();
        acc += lds[(tid + 64 * (k + 1)) & 1023];
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
    if (acc == 0x7fffffff) sink[0] = acc;
}

int main() {
    const int F = 1024;
    unsigned long long *cyc;
    int *sink;
    CK(hipMalloc(&cyc, F * 8));
    CK(hipMalloc(&sink, 4));
    const size_t lds = 150 * 1024;
    CK(hipFuncSetAttribute((const void *)k_bar, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<unsigned long long> h(F);
    for (int work : {0, 16, 64}) {
        for (int K : {0, 64}) {
            for (int rep = 0; rep < 2; ++rep) {
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(k_bar, dim3(F), dim3(1024), lds, 0, K, work, cyc, sink);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
            }
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            CK(hipMemcpy(h.data(), cyc, F * 8, hipMemcpyDeviceToHost));
            double m = 0;
            for (auto v : h) m += (double)v / F;
            printf("work %2d K %2d: kernel %.4f ms, %.0f cycles per workgroup, %.0f per step (two barriers)\n", work, K,
                   ms, m, K ? m / K : 0.0);
        }
    }
    return 0;
}
