/*
 * rdbench.hip — practical HBM read rate on this box: a 5.42 GB buffer (the
 * metric batch's PCM) streamed once by (a) coalesced global_load_dwordx4 into
 * registers, (b) LDS-DMA (global_load_lds_dwordx4) into per-wave LDS slots.
 *   hipcc --offload-arch=gfx950 -O3 tools/rdbench.hip -o tools/rdbench
 */
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_read(const u4 *__restrict__ p, size_t n16, unsigned *out) {
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * 256 * 4;
    for (size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x; i < n16; i += stride) {
        u4 a = p[i], b = i + 256 < n16 ? p[i + 256] : u4{0,0,0,0};
        u4 c = i + 512 < n16 ? p[i + 512] : u4{0,0,0,0}, d = i + 768 < n16 ? p[i + 768] : u4{0,0,0,0};
        acc += a.x ^ b.y ^ c.z ^ d.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int SLOTS>
__global__ __launch_bounds__(256) void k_dma(const u4 *__restrict__ p, size_t ntiles, unsigned *out) {
    __shared__ u4 slot[4][SLOTS][1152];        /* 18 KB per slot, 4 waves */
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * 4;
    size_t t = (size_t)blockIdx.x * 4 + w;
    auto issue = [&](size_t tt, u4 *s) {
        for (int r = 0; r < 18; ++r) {
            const u4 *src = p + tt * 1152 + r * 64 + lane;
            const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) void *)(s + r * 64));
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" :: "v"(src), "s"(m0) : "memory");
        }
    };
    int k = 0;
    for (int j = 0; j < SLOTS; ++j) if (t + j * stride < ntiles) issue(t + j * stride, slot[w][j]);
    for (; t < ntiles; t += stride, ++k) {
        if (SLOTS == 2 && t + stride < ntiles) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        u4 *s = slot[w][SLOTS == 2 ? (k & 1) : 0];
        acc += s[lane].x ^ s[1100 + (lane & 31)].y;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (t + SLOTS * stride < ntiles) issue(t + SLOTS * stride, s);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const size_t bytes = 1024ull * 2646000 * 2;
    const size_t n16 = bytes / 16, ntiles = n16 / 1152;
    u4 *p; unsigned *o;
    CK(hipMalloc(&p, bytes)); CK(hipMalloc(&o, 4));
    CK(hipMemset(p, 1, bytes));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < 10; ++i) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-28s %.3f ms  %.2f TB/s\n", name, ms / 10, bytes / (ms / 10 * 1e-3) / 1e12);
    };
    for (int g : {1024, 2048, 4096, 8192})
        run((std::string("dwordx4 grid ") + std::to_string(g)).c_str(), [&] { hipLaunchKernelGGL(k_read, dim3(g), dim3(256), 0, 0, p, n16, o); });
    run("lds-dma 1 slot, 1 WG/CU x4", [&] { hipLaunchKernelGGL(k_dma<1>, dim3(512), dim3(256), 0, 0, p, ntiles, o); });
    run("lds-dma 2 slots, 1 WG/CU", [&] { hipLaunchKernelGGL(k_dma<2>, dim3(256), dim3(256), 0, 0, p, ntiles, o); });
    return 0;
}
