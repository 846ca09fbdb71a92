/*
 * lanebench.hip — does a wave64 f64 recursion with only L lanes active issue
 * faster than with 64?  (tools only; reference-mode envelope design question:
 * 1024 recordings fill 16 waves on 16 of 1024 SIMDs, so if a VALU op with few
 * active lanes takes fewer cycles, spreading recordings over more waves pays.)
 * The DF2T step of k_envelope_ref.hip on a register-resident input, timed per
 * step with s_memtime, for L = 64, 32, 16, 8, 4, 1 active lanes; and the Kahan
 * remove+add chain.
 *   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/lanebench.hip -o tools/lanebench
 */
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

struct D4 {
    double b0, b1, b2, b3, b4, a1, a2, a3, a4, z0, z1, z2, z3;
    __device__ __forceinline__ double step(double xn) {
        const double bx0 = b0 * xn, bx1 = xn * b1, bx2 = xn * b2, bx3 = xn * b3, bx4 = xn * b4;
        const double p1 = z1 + bx1, p2 = z2 + bx2, p3 = z3 + bx3;
        const double yn = z0 + bx0;
        z0 = p1 - yn * a1;
        z1 = p2 - yn * a2;
        z2 = p3 - yn * a3;
        z3 = bx4 - yn * a4;
        return yn;
    }
};

/* the Kahan pass with its memory streams, rows [step][file] as k_envelope_ref
 * lays them out: MODE 0: two loads (add, remove) + one store per step; 1: one
 * load (the remove value from registers, w = 30 steps back) + one store; 2:
 * one load + one 16-B store per two steps ([step/2][file][2] rows) */
template <int MODE>
__global__ __launch_bounds__(64) void k_kahan_mem(const double *y, double *sums, long S, long n, double *out,
                                                 unsigned long long *t) {
    constexpr int PF = 32, W = 30;
    const int lane = threadIdx.x;
    const long f = blockIdx.x * 64 + lane;
    double sum = 0, cad = 0, crm = 0;
    double ca[PF], cp[PF], na[PF], cr[PF], nr[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) { ca[u] = fabs(y[(PF + u) * S + f]); cp[u] = fabs(y[u * S + f]); cr[u] = cp[u]; }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (long i0 = PF; i0 + 2 * PF < n; i0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            na[u] = fabs(y[(i0 + PF + u) * S + f]);
            if (MODE == 0) nr[u] = fabs(y[(i0 + PF + u - W) * S + f]);
        }
        double sv[PF];
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const double rv = MODE == 0 ? cr[u] : (u >= W ? ca[u - W] : cp[u - W + PF]);
            const double yr = -rv - crm, tr = sum + yr;
            crm = (tr - sum) - yr;
            sum = tr;
            const double ya = ca[u] - cad, ta = sum + ya;
            cad = (ta - sum) - ya;
            sum = ta;
            sv[u] = sum;
            if (MODE != 2) sums[(i0 + u) * S + f] = sum;
        }
        if (MODE == 2) {
            typedef double dv2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int u = 0; u < PF; u += 2) *(dv2 *)(sums + (((i0 + u) >> 1) * S + f) * 2) = dv2{sv[u], sv[u + 1]};
        }
#pragma unroll
        for (int u = 0; u < PF; ++u) { cp[u] = ca[u]; ca[u] = na[u]; if (MODE == 0) cr[u] = nr[u]; }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[f] = sum;
    if (lane == 0) t[blockIdx.x] = t1 - t0;
}

template <int KAHAN>
__global__ __launch_bounds__(64) void k_lanes(int L, long n, double *out, unsigned long long *t) {
    const int lane = threadIdx.x;
    D4 d{0.02, 0.0, -0.04, 0.0, 0.02, -3.5, 4.6, -2.7, 0.6, 0, 0, 0, 0};
    double x = 1.0 + lane, acc = 0, sum = 0, cad = 0, crm = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (lane < L) {
        for (long i = 0; i < n; i += 16) {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const double xs = x + u;
                if (KAHAN) {
                    const double yr = -xs - crm, tr = sum + yr;
                    crm = (tr - sum) - yr;
                    sum = tr;
                    const double ya = xs - cad, ta = sum + ya;
                    cad = (ta - sum) - ya;
                    sum = ta;
                } else {
                    acc += d.step(xs);
                }
            }
            x += 1.0;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + lane] = acc + sum;
    if (lane == 0) t[blockIdx.x] = t1 - t0;
}

int main() {
    const long n = 1 << 15;
    const int G = 16;
    double *out;
    unsigned long long *t, th[G];
    CK(hipMalloc(&out, G * 64 * 8));
    CK(hipMalloc(&t, G * 8));
    const int Ls[] = {64, 32, 17, 16, 8, 4, 1};
    for (int k = 0; k < 2; ++k)
        for (int L : Ls) {
            for (int r = 0; r < 2; ++r) {
                if (k == 0) hipLaunchKernelGGL(k_lanes<0>, dim3(G), dim3(64), 0, 0, L, n, out, t);
                else hipLaunchKernelGGL(k_lanes<1>, dim3(G), dim3(64), 0, 0, L, n, out, t);
                CK(hipDeviceSynchronize());
            }
            CK(hipMemcpy(th, t, sizeof th, hipMemcpyDeviceToHost));
            double avg = 0;
            for (int g = 0; g < G; ++g) avg += (double)th[g];
            avg /= G;
            /* s_memtime runs at the shader clock on gfx9 (100 MHz constant clock is s_memrealtime) */
            printf("%-6s L=%2d  %.1f memtime ticks/step\n", k ? "kahan" : "filter", L, avg / n);
        }
    /* the Kahan pass with memory streams: 16 waves (1024 recordings) over rows of 18154 steps */
    const long S = 1024, nr = 18154;
    double *y, *sums;
    CK(hipMalloc(&y, (size_t)(nr + 64) * S * 8));
    CK(hipMalloc(&sums, (size_t)(nr + 64) * S * 8));
    CK(hipMemset(y, 0, (size_t)(nr + 64) * S * 8));
    const char *nm[3] = {"2 loads + 1 store / step", "1 load (remove from regs) + 1 store", "1 load + 16-B store / 2 steps"};
    for (int m = 0; m < 3; ++m) {
        for (int r = 0; r < 2; ++r) {
            if (m == 0) hipLaunchKernelGGL(k_kahan_mem<0>, dim3(16), dim3(64), 0, 0, y, sums, S, nr, out, t);
            if (m == 1) hipLaunchKernelGGL(k_kahan_mem<1>, dim3(16), dim3(64), 0, 0, y, sums, S, nr, out, t);
            if (m == 2) hipLaunchKernelGGL(k_kahan_mem<2>, dim3(16), dim3(64), 0, 0, y, sums, S, nr, out, t);
            CK(hipDeviceSynchronize());
        }
        CK(hipMemcpy(th, t, sizeof th, hipMemcpyDeviceToHost));
        double avg = 0;
        for (int g = 0; g < G; ++g) avg += (double)th[g];
        printf("kahan mem: %-40s %.1f ticks/step\n", nm[m], avg / G / (nr - 96));
    }
    return 0;
}
