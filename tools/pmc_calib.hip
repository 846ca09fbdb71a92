/*
 * pmc_calib.hip — calibrate rocprofv3's FETCH_SIZE / WRITE_SIZE against known
 * byte counts for the access widths the bpmx kernels use (4, 8 and 16 bytes
 * per lane, coalesced).  MI355X_MICROARCH.md calibrates only the 16-byte
 * streaming read (FETCH_SIZE = half the bytes) and says other widths are
 * uncalibrated; tools/pmc_traffic.py applies the factors measured here.
 *
 *   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pmc_calib.hip -o tools/pmc_calib
 *   rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -o run -- ./tools/pmc_calib
 *   rocprofv3 --pmc WRITE_SIZE --output-format csv -d <dir> -o run -- ./tools/pmc_calib
 *
 * Every kernel streams a 768 MiB buffer once (three times the 256 MiB
 * Infinity Cache, so re-use cannot hide bytes), reading with one load width or
 * writing with one store width; it prints the bytes each kernel moves so the
 * counter's ratio can be read off the CSV (kernel names carry the width).
 */
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <typename T>
__global__ __launch_bounds__(256) void calib_read(const T *__restrict__ p, size_t n, double *sink) {
    double acc = 0.0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const T v = p[i];
        acc += (double)((const unsigned char *)&v)[0];
    }
    if (acc == -1.0) *sink = acc;                            /* never true: keeps the loads */
}

template <typename T>
__global__ __launch_bounds__(256) void calib_write(T *__restrict__ p, size_t n) {
    T v;
    __builtin_memset(&v, 0, sizeof v);
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = v;
}

struct alignas(16) B16 { unsigned long long a, b; };

int main() {
    const size_t bytes = (size_t)768 << 20;
    unsigned char *buf;
    double *sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(buf, 1, bytes));
    const dim3 g(2048), b(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(calib_read<unsigned int>, g, b, 0, 0, (const unsigned int *)buf, bytes / 4, sink);
        hipLaunchKernelGGL(calib_read<double>, g, b, 0, 0, (const double *)buf, bytes / 8, sink);
        hipLaunchKernelGGL(calib_read<B16>, g, b, 0, 0, (const B16 *)buf, bytes / 16, sink);
        hipLaunchKernelGGL(calib_write<unsigned int>, g, b, 0, 0, (unsigned int *)buf, bytes / 4);
        hipLaunchKernelGGL(calib_write<double>, g, b, 0, 0, (double *)buf, bytes / 8);
        hipLaunchKernelGGL(calib_write<B16>, g, b, 0, 0, (B16 *)buf, bytes / 16);
    }
    CK(hipDeviceSynchronize());
    printf("bytes per kernel %zu (read u32 / f64 / 16 B, write u32 / f64 / 16 B, twice)\n", bytes);
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
