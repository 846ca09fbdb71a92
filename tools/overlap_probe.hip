/*
 * overlap_probe.hip — do kernels on two HIP streams run at the same time on
 * this box?  A "chain" kernel (16 one-wave workgroups spinning for T_A, like
 * reference mode's sequential passes) on stream A beside a "wide" kernel
 * (1024 workgroups of 1024 threads with 150 KB of LDS each, spinning T_B per
 * workgroup, like the detection kernels) on stream B; total wall time against
 * the two alone.  Variants: no CU masks, and stream A / B on disjoint CU masks.
 *   hipcc --offload-arch=gfx950 -O3 tools/overlap_probe.hip -o tools/overlap_probe
 */
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_spin(long long ticks, int *sink) {
    const long long t0 = wall_clock64();
    int acc = 0;
    while (wall_clock64() - t0 < ticks) acc += threadIdx.x;
    if (acc == 0x7fffffff) sink[0] = acc;
}

__global__ __launch_bounds__(1024) void k_wide(long long ticks, int *sink) {
    extern __shared__ int lds[];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const long long t0 = wall_clock64();
    int acc = lds[(threadIdx.x + 1) & 1023];
    while (wall_clock64() - t0 < ticks) acc += 1;
    if (acc == 0x7fffffff) sink[0] = acc;
}

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
    int *sink;
    CK(hipMalloc(&sink, 4));
    const long long tA = 100 * 2000;    /* wall_clock64 at 100 MHz: 2 ms */
    const long long tB = 100 * 50;      /* 50 us per wide workgroup: 4 rounds over 256 CUs ~ 0.2 ms */
    const size_t lds = 150 * 1024;
    CK(hipFuncSetAttribute((const void *)k_wide, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    for (int variant = 0; variant < 3; ++variant) {
        hipStream_t sa, sb;
        if (variant == 0) {
            CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
            CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
        } else {
            /* A: CUs 0..15 or 0..31 (bit c -> XCD c mod 8), B: the rest */
            const int na = variant == 1 ? 16 : 32;
            std::vector<uint32_t> ma(8, 0u), mb(8, 0u);
            for (int c = 0; c < 256; ++c) ((c < na) ? ma : mb)[c / 32] |= 1u << (c % 32);
            CK(hipExtStreamCreateWithCUMask(&sa, 8, ma.data()));
            CK(hipExtStreamCreateWithCUMask(&sb, 8, mb.data()));
        }
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipDeviceSynchronize());
            auto t0 = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(k_spin, dim3(16), dim3(64), 0, sa, tA, sink);
            CK(hipStreamSynchronize(sa));
            const double a = ms_since(t0);
            t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < 8; ++i) hipLaunchKernelGGL(k_wide, dim3(1024), dim3(1024), lds, sb, tB, sink);
            CK(hipStreamSynchronize(sb));
            const double b = ms_since(t0);
            t0 = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(k_spin, dim3(16), dim3(64), 0, sa, tA, sink);
            for (int i = 0; i < 8; ++i) hipLaunchKernelGGL(k_wide, dim3(1024), dim3(1024), lds, sb, tB, sink);
            CK(hipStreamSynchronize(sa));
            CK(hipStreamSynchronize(sb));
            const double ab = ms_since(t0);
            printf("variant %s: chain alone %.3f ms, 8 wide alone %.3f ms, both %.3f ms (%s)\n",
                   variant == 0 ? "no mask" : variant == 1 ? "mask 16/240" : "mask 32/224", a, b, ab,
                   ab < 0.8 * (a + b) ? "overlapped" : "serialised");
        }
        CK(hipStreamDestroy(sa));
        CK(hipStreamDestroy(sb));
    }
    return 0;
}
