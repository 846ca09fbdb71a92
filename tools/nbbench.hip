/*
 * nbbench.hip — variant timing for the native-mode block dot-product kernel
 * (u_j = sum F_i x[c_j+i], v_j = sum G_i x[c_j+i], 8 f64 outputs per block of
 * ds+1 int16 samples).  Not product code: the winner moves into
 * bpm_analysis_amd/csrc/k_envelope_native.hip.
 *   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/nbbench.hip -o tools/nbbench
 *   ./tools/nbbench [files] [secs]
 */
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

struct Acc8 {
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    __device__ __forceinline__ void add(double x, const double *__restrict__ c) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = __builtin_fma(c[k], x, a[k]);
    }
};

__device__ __forceinline__ double lo16(uint32_t w) { return (double)(int)(int16_t)(w & 0xFFFFu); }
__device__ __forceinline__ double hi16(uint32_t w) { return (double)((int)w >> 16); }

/* ---- V_B<R,BS>: lane = R blocks, BS-sample bursts straight from global ---- */
template <int R, int BS>
__global__ __launch_bounds__(256) void vb(const int16_t *pcm, int64_t n, int64_t nb, int ds,
                                          const double *__restrict__ coef, double *uv) {
    constexpr int NW = BS / 2;
    const int f = blockIdx.y;
    const int64_t H = (nb + R - 1) / R;
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= H) return;
    Acc8 acc[R];
    const uint32_t *wp[R];
    uint32_t sh[R];
    bool ok[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t j = g + r * H;
        ok[r] = j < nb;
        const int16_t *xb = pcm + (int64_t)f * n + (ok[r] ? j : g) * ds;
        wp[r] = (const uint32_t *)((uintptr_t)xb & ~(uintptr_t)3);
        sh[r] = ((uintptr_t)xb & 2) ? 16u : 0u;
    }
    const int L = ds + 1;
    int i = 0;
    for (; i + BS <= L; i += BS) {
        const double *cr = coef + (int64_t)i * 8;
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        uint32_t w[R][NW + 1];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t *p = wp[r] + i / 2;
#pragma unroll
            for (int q = 0; q < NW / 4; ++q) {
                u4 t;
                __builtin_memcpy(&t, p + 4 * q, 16);
                w[r][4 * q] = t.x; w[r][4 * q + 1] = t.y; w[r][4 * q + 2] = t.z; w[r][4 * q + 3] = t.w;
            }
            w[r][NW] = sh[r] ? p[NW] : 0u;
        }
#pragma unroll
        for (int m = 0; m < NW; ++m) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t d = __builtin_amdgcn_alignbit(w[r][m + 1], w[r][m], sh[r]);
                acc[r].add(lo16(d), cr + (2 * m) * 8);
                acc[r].add(hi16(d), cr + (2 * m + 1) * 8);
            }
        }
    }
    for (; i < L; ++i) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int16_t *xb = (const int16_t *)((const char *)wp[r] + (sh[r] >> 3));
            acc[r].add((double)xb[i], coef + (int64_t)i * 8);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!ok[r]) continue;
        const int64_t j = g + r * H;
        double2 *o = (double2 *)(uv + ((int64_t)f * nb + j) * 8);
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = make_double2(acc[r].a[2 * k], acc[r].a[2 * k + 1]);
    }
}

/* ---- V_A: one wave per workgroup, persistent; 64-block tile staged through LDS,
 * next tile prefetched into registers while the current one is computed ---- */
template <int RCH, int UN = 1>
__global__ __launch_bounds__(64) void va(const int16_t *pcm, int64_t n, int64_t nb, int ds, int nfiles,
                                         const double *__restrict__ coef, double *uv) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    __shared__ u4 tile[RCH * 64 + 1];
    const int lane = threadIdx.x;
    const int64_t tpf = (nb + 63) / 64;
    const int64_t ntiles = tpf * nfiles;
    const int64_t total = n * nfiles;
    auto issue = [&](int64_t t, u4 *reg, int &off) {
        const int64_t f = t / tpf, j0 = (t % tpf) * 64;
        const int64_t s0 = f * n + j0 * ds;                      /* first sample */
        const int64_t a0 = s0 & ~(int64_t)7;
        off = (int)(s0 - a0);
#pragma unroll
        for (int r = 0; r < RCH; ++r) {
            const int64_t c = a0 + (int64_t)(r * 64 + lane) * 8;
            if (c + 8 <= total) __builtin_memcpy(&reg[r], pcm + c, 16);
            else reg[r] = u4{0, 0, 0, 0};
        }
    };
    u4 reg[RCH];
    int off = 0;
    int64_t t = blockIdx.x;
    if (t < ntiles) issue(t, reg, off);
    while (t < ntiles) {
        const int64_t f = t / tpf, j0 = (t % tpf) * 64;
#pragma unroll
        for (int r = 0; r < RCH; ++r) tile[r * 64 + lane] = reg[r];
        const int coff = off;
        __syncthreads();
        const int64_t tn = t + gridDim.x;
        if (tn < ntiles) issue(tn, reg, off);
        const int64_t j = j0 + lane;
        if (j < nb) {
            const uint16_t *tl = (const uint16_t *)tile;
            const int base = coff + lane * ds;                 /* halfword index */
            const uint32_t *wp = (const uint32_t *)tile + (base >> 1);
            const uint32_t sh = (base & 1) ? 16u : 0u;
            Acc8 acc;
            const int L = ds + 1;
            int i = 0;
#pragma unroll UN
            for (; i + 8 <= L; i += 8) {
                const uint32_t *p = wp + i / 2;
                const uint32_t w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3], w4 = p[4];
                const uint32_t d0 = __builtin_amdgcn_alignbit(w1, w0, sh);
                const uint32_t d1 = __builtin_amdgcn_alignbit(w2, w1, sh);
                const uint32_t d2 = __builtin_amdgcn_alignbit(w3, w2, sh);
                const uint32_t d3 = __builtin_amdgcn_alignbit(w4, w3, sh);
                const double *cr = coef + (int64_t)i * 8;
                acc.add(lo16(d0), cr + 0);  acc.add(hi16(d0), cr + 8);
                acc.add(lo16(d1), cr + 16); acc.add(hi16(d1), cr + 24);
                acc.add(lo16(d2), cr + 32); acc.add(hi16(d2), cr + 40);
                acc.add(lo16(d3), cr + 48); acc.add(hi16(d3), cr + 56);
            }
            for (; i < L; ++i) acc.add((double)(int16_t)tl[base + i], coef + (int64_t)i * 8);
            double2 *o = (double2 *)(uv + (f * nb + j) * 8);
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] = make_double2(acc.a[2 * k], acc.a[2 * k + 1]);
        }
        __syncthreads();
        t = tn;
    }
}

/* ---- V_C: one wave per workgroup, persistent; 32-block tile in LDS, lane =
 * (block, half): lanes 0-31 sum samples [0, sp), lanes 32-63 [sp, ds], halves
 * combined with v_permlane32_swap; next tile prefetched into registers ---- */
__device__ __forceinline__ double swap_half(double x) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return __builtin_bit_cast(double, ((uint64_t)rh[1] << 32) | rl[1]);
}

template <int RCH>
__global__ __launch_bounds__(128) void vc(const int16_t *pcm, int64_t n, int64_t nb, int ds, int nfiles,
                                          const double *__restrict__ coef, double *uv) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    __shared__ u4 tile[RCH * 128 + 1];
    __shared__ double comb[8][64];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t tpf = (nb + 63) / 64;
    const int64_t ntiles = tpf * nfiles;
    const int64_t total = n * nfiles;
    const int L = ds + 1;
    const int sp = (L / 16) * 8;
    auto issue = [&](int64_t t, u4 *reg, int &off) {
        const int64_t f = t / tpf, j0 = (t % tpf) * 64;
        const int64_t s0 = f * n + j0 * ds;
        const int64_t a0 = s0 & ~(int64_t)7;
        off = (int)(s0 - a0);
#pragma unroll
        for (int r = 0; r < RCH; ++r) {
            const int64_t c = a0 + (int64_t)(r * 128 + tid) * 8;
            if (c + 8 <= total) __builtin_memcpy(&reg[r], pcm + c, 16);
            else reg[r] = u4{0, 0, 0, 0};
        }
    };
    u4 reg[RCH];
    int off = 0;
    int64_t t = blockIdx.x;
    if (t < ntiles) issue(t, reg, off);
    const int i0 = w ? sp : 0, cnt = w ? L - sp : sp;
    const double *cb = coef + (int64_t)i0 * 8;
    while (t < ntiles) {
        const int64_t f = t / tpf, j0 = (t % tpf) * 64;
#pragma unroll
        for (int r = 0; r < RCH; ++r) tile[r * 128 + tid] = reg[r];
        const int coff = off;
        __syncthreads();
        const int64_t tn = t + gridDim.x;
        if (tn < ntiles) issue(tn, reg, off);
        const int64_t j = j0 + lane;
        const uint16_t *tl = (const uint16_t *)tile;
        const int base = coff + lane * ds + i0;
        const uint32_t *wp = (const uint32_t *)tile + (base >> 1);
        const uint32_t sh = (base & 1) ? 16u : 0u;
        Acc8 acc;
        int i = 0;
        for (; i + 8 <= cnt; i += 8) {
            const uint32_t *p = wp + i / 2;
            const uint32_t w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3], w4 = p[4];
            const uint32_t d0 = __builtin_amdgcn_alignbit(w1, w0, sh);
            const uint32_t d1 = __builtin_amdgcn_alignbit(w2, w1, sh);
            const uint32_t d2 = __builtin_amdgcn_alignbit(w3, w2, sh);
            const uint32_t d3 = __builtin_amdgcn_alignbit(w4, w3, sh);
            const double *cr = cb + (int64_t)i * 8;
            acc.add(lo16(d0), cr + 0);  acc.add(hi16(d0), cr + 8);
            acc.add(lo16(d1), cr + 16); acc.add(hi16(d1), cr + 24);
            acc.add(lo16(d2), cr + 32); acc.add(hi16(d2), cr + 40);
            acc.add(lo16(d3), cr + 48); acc.add(hi16(d3), cr + 56);
        }
        for (; i < cnt; ++i) acc.add((double)(int16_t)tl[base + i], cb + (int64_t)i * 8);
        if (w == 1) {
#pragma unroll
            for (int k = 0; k < 8; ++k) comb[k][lane] = acc.a[k];
        }
        __syncthreads();
        if (w == 0 && j < nb) {
            double o8[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) o8[k] = acc.a[k] + comb[k][lane];
            double2 *o = (double2 *)(uv + (f * nb + j) * 8);
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] = make_double2(o8[2 * k], o8[2 * k + 1]);
        }
        t = tn;
    }
}

/* data-path only: sum of samples per block (no coefficient traffic) */
__global__ __launch_bounds__(256) void vdata(const int16_t *pcm, int64_t n, int64_t nb, int ds, double *uv) {
    const int f = blockIdx.y;
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= nb) return;
    const int16_t *xb = pcm + (int64_t)f * n + j * ds;
    const uint32_t *wp = (const uint32_t *)((uintptr_t)xb & ~(uintptr_t)3);
    const uint32_t sh = ((uintptr_t)xb & 2) ? 16u : 0u;
    double s0 = 0, s1 = 0;
    const int L = ds + 1;
    int i = 0;
    for (; i + 64 <= L; i += 64) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        uint32_t w[33];
        const uint32_t *p = wp + i / 2;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            u4 t;
            __builtin_memcpy(&t, p + 4 * q, 16);
            w[4 * q] = t.x; w[4 * q + 1] = t.y; w[4 * q + 2] = t.z; w[4 * q + 3] = t.w;
        }
        w[32] = sh ? p[32] : 0u;
#pragma unroll
        for (int m = 0; m < 32; ++m) {
            const uint32_t d = __builtin_amdgcn_alignbit(w[m + 1], w[m], sh);
            s0 += lo16(d);
            s1 += hi16(d);
        }
    }
    uv[(int64_t)f * nb + j] = s0 + s1;
}

int main(int argc, char **argv) {
    const int F = argc > 1 ? atoi(argv[1]) : 1024;
    const double secs = argc > 2 ? atof(argv[2]) : 60.0;
    const int ds = argc > 3 ? atoi(argv[3]) : 146;
    const int64_t n = (int64_t)(secs * 44100);
    const int64_t nd = (n + ds - 1) / ds, nb = nd - 1;
    printf("F=%d n=%lld ds=%d nb=%lld\n", F, (long long)n, ds, (long long)nb);
    int16_t *pcm;
    double *coef, *uv, *uv2;
    CK(hipMalloc(&pcm, (size_t)F * n * 2 + 64));
    CK(hipMalloc(&coef, (size_t)(ds + 1) * 8 * 8));
    CK(hipMalloc(&uv, (size_t)F * nb * 64));
    CK(hipMalloc(&uv2, (size_t)F * nb * 64));
    {
        std::vector<int16_t> h((size_t)n);
        uint64_t s = 1;
        for (auto &v : h) { s = s * 6364136223846793005ull + 1442695040888963407ull; v = (int16_t)(s >> 48); }
        for (int f = 0; f < F; ++f) CK(hipMemcpy(pcm + (size_t)f * n, h.data(), n * 2, hipMemcpyHostToDevice));
        std::vector<double> c((size_t)(ds + 1) * 8);
        for (size_t i = 0; i < c.size(); ++i) c[i] = 1.0 / (1.0 + (double)i);
        CK(hipMemcpy(coef, c.data(), c.size() * 8, hipMemcpyHostToDevice));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double gb = (double)F * n * 2 / 1e9;
    const char *only = argc > 4 ? argv[4] : nullptr;
    auto timeit = [&](const char *name, auto launch) {
        if (only && !strstr(name, only)) return;
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        const int reps = 10;
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-16s %8.3f ms  %7.1f GB/s\n", name, ms, gb / ms * 1e3);
    };
    auto cmp = [&](const char *name) {
        if (only && !strstr(name, only)) return;
        std::vector<double> a((size_t)F * nb * 8), b((size_t)F * nb * 8);
        CK(hipMemcpy(a.data(), uv, a.size() * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), uv2, b.size() * 8, hipMemcpyDeviceToHost));
        printf("  %s vs vb<1>: %s\n", name, memcmp(a.data(), b.data(), a.size() * 8) == 0 ? "identical" : "DIFFER");
    };
    timeit("vdata", [&] { vdata<<<dim3((nb + 255) / 256, F), 256>>>(pcm, n, nb, ds, uv2); });
    timeit("vb<1,64>", [&] { vb<1, 64><<<dim3((nb + 255) / 256, F), 256>>>(pcm, n, nb, ds, coef, uv); });
    timeit("vb<1,32>", [&] { vb<1, 32><<<dim3((nb + 255) / 256, F), 256>>>(pcm, n, nb, ds, coef, uv2); });
    cmp("vb<1,32>");
    timeit("vb<2,32>", [&] { vb<2, 32><<<dim3((nb + 511) / 512, F), 256>>>(pcm, n, nb, ds, coef, uv2); });
    cmp("vb<2,32>");
    timeit("vb<2,64>", [&] { vb<2, 64><<<dim3((nb + 511) / 512, F), 256>>>(pcm, n, nb, ds, coef, uv2); });
    cmp("vb<2,64>");
    timeit("vb<4,32>", [&] { vb<4, 32><<<dim3((nb + 1023) / 1024, F), 256>>>(pcm, n, nb, ds, coef, uv2); });
    cmp("vb<4,32>");
    int ncu = 256;
    for (int per : {4, 8}) {
        char nm[32];
        snprintf(nm, sizeof nm, "va<19> x%d", per);
        CK(hipMemset(uv2, 0, (size_t)F * nb * 64));
        timeit(nm, [&] { va<19><<<ncu * per, 64>>>(pcm, n, nb, ds, F, coef, uv2); });
        cmp(nm);
    }
    for (int per : {8}) {
        char nm[32];
        snprintf(nm, sizeof nm, "va<19,2> x%d", per);
        CK(hipMemset(uv2, 0, (size_t)F * nb * 64));
        timeit(nm, [&] { va<19, 2><<<ncu * per, 64>>>(pcm, n, nb, ds, F, coef, uv2); });
        cmp(nm);
        snprintf(nm, sizeof nm, "va<19,4> x%d", per);
        CK(hipMemset(uv2, 0, (size_t)F * nb * 64));
        timeit(nm, [&] { va<19, 4><<<ncu * per, 64>>>(pcm, n, nb, ds, F, coef, uv2); });
        cmp(nm);
    }
    auto cmpt = [&](const char *name) {
        if (only && !strstr(name, only)) return;
        std::vector<double> a((size_t)F * nb * 8), b((size_t)F * nb * 8);
        CK(hipMemcpy(a.data(), uv, a.size() * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), uv2, b.size() * 8, hipMemcpyDeviceToHost));
        double mx = 0;
        for (size_t i = 0; i < a.size(); ++i) { double d = fabs(a[i] - b[i]) / (fabs(a[i]) + 1e-300); if (d > mx) mx = d; }
        printf("  %s vs vb<1>: max rel diff %.3g\n", name, mx);
    };
    for (int per : {4, 6, 8}) {
        char nm[32];
        snprintf(nm, sizeof nm, "vc<10> x%d", per);
        CK(hipMemset(uv2, 0, (size_t)F * nb * 64));
        timeit(nm, [&] { vc<10><<<ncu * per, 128>>>(pcm, n, nb, ds, F, coef, uv2); });
        cmpt(nm);
    }
    return 0;
}
