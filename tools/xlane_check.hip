/*
 * xlane_check.hip — checks bpm_analysis_amd/csrc/bpmx_xlane.h's register
 * shifts against __shfl_up / __shfl_down for every shift the tile epilogue
 * uses, on doubles with distinct bit patterns per lane.
 *   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/xlane_check.hip -o tools/xlane_check
 */
#include "../bpm_analysis_amd/csrc/bpmx_xlane.h"

#include <cstdio>

using namespace bpmx;

template <int D>
__device__ void one(double v, int k, int *bad) {
    const int lane = threadIdx.x;
    const double u = xl_up<D>(v), ru = __shfl_up(v, D);
    const double d = xl_down<D>(v), rd = __shfl_down(v, D);
    if (lane >= D && __double_as_longlong(u) != __double_as_longlong(ru)) atomicAdd(&bad[2 * k], 1);
    if (lane + D < 64 && __double_as_longlong(d) != __double_as_longlong(rd)) atomicAdd(&bad[2 * k + 1], 1);
}

__global__ void k(int *bad) {
    const double v = 1.0 + threadIdx.x * 0.123456789 + 1e-300 * threadIdx.x;
    one<1>(v, 0, bad);
    one<2>(v, 1, bad);
    one<4>(v, 2, bad);
    one<8>(v, 3, bad);
    one<16>(v, 4, bad);
    one<32>(v, 5, bad);
}

int main() {
    int *d, h[12];
    (void)hipMalloc(&d, sizeof h);
    (void)hipMemset(d, 0, sizeof h);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    int tot = 0;
    for (int i = 0; i < 6; ++i) {
        printf("shift %2d: up %d bad, down %d bad\n", 1 << i, h[2 * i], h[2 * i + 1]);
        tot += h[2 * i] + h[2 * i + 1];
    }
    printf(tot ? "XLANE FAIL\n" : "XLANE OK\n");
    return tot != 0;
}
