/*
 * chainbench.hip — cycles per step of the reference-mode recursions on one
 * wave (tools only): the DF2T filter step (k_envelope_ref.hip Df2t::step),
 * with and without a strided scratch store per step, and the Kahan
 * remove+add chain of the rolling mean.  s_memtime counts shader clocks.
 *   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/chainbench.hip -o tools/chainbench
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

/* mode 0: filter chain only; 1: + store per step (stride S doubles);
 * 2: + load per step (same block); 3: Kahan remove+add; 4: two filter chains per lane;
 * 5: load (one block ahead) + store per step, interleaved rows [step][file] (the kernel's layout);
 * 6: the same in 4-step groups [step/4][file][4] (two 16-B loads / stores per 4 steps);
 * 7: the forward pass as the kernel runs it: int16 PCM gathered at stride ds (one recording
 *    per lane, 2646000 frames apart), one block ahead, + row store */
template <int MODE>
__global__ __launch_bounds__(64) void k_chain(double *scr, long S, long n, double *out, unsigned long long *t) {
    const int lane = threadIdx.x;
    D4 d{0.02, 0.0, -0.04, 0.0, 0.02, -3.5, 4.6, -2.7, 0.6, 0, 0, 0, 0};
    D4 e = d;
    double x = 1.0 + lane, acc = 0, sum = 0, cad = 0, crm = 0;
    double *p = scr + blockIdx.x * 64 + lane;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (MODE == 7) {
        const short *pcm = (const short *)(scr + (size_t)(n + 32) * S * 2) + (size_t)(blockIdx.x * 64 + lane) * 2646000;
        double *q = scr + (size_t)(n + 16) * S;
        double cur[16], nxt[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) cur[u] = (double)pcm[(long)u * 146];
        for (long i = 0; i < n; i += 16) {
#pragma unroll
            for (int u = 0; u < 16; ++u) nxt[u] = (double)pcm[((i + 16 + u) % 18000) * 146];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const double y = d.step(cur[u]);
                q[(i + u) * S + blockIdx.x * 64 + lane] = y;
                acc += y;
                cur[u] = nxt[u];
            }
        }
    } else if (MODE == 5 || MODE == 6) {
        typedef double dv2 __attribute__((ext_vector_type(2)));
        double *q = scr + (size_t)(n + 16) * S;                  /* output region */
        double cur[16], nxt[16];
        auto ld = [&](long i, double *v) {
            if (MODE == 5) {
#pragma unroll
                for (int u = 0; u < 16; ++u) v[u] = p[(i + u) * S];
            } else {
                const dv2 *g = (const dv2 *)(scr + ((i >> 2) * S + blockIdx.x * 64 + lane) * 4);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const dv2 a = g[u * S * 2], b = g[u * S * 2 + 1];
                    v[4 * u] = a.x; v[4 * u + 1] = a.y; v[4 * u + 2] = b.x; v[4 * u + 3] = b.y;
                }
            }
        };
        ld(0, cur);
        for (long i = 0; i < n; i += 16) {
            ld(i + 16, nxt);
            double ys[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) ys[u] = d.step(cur[u]);
            if (MODE == 5) {
#pragma unroll
                for (int u = 0; u < 16; ++u) q[(i + u) * S + blockIdx.x * 64 + lane] = ys[u];
            } else {
                dv2 *g = (dv2 *)(q + ((i >> 2) * S + blockIdx.x * 64 + lane) * 4);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    g[u * S * 2] = dv2{ys[4 * u], ys[4 * u + 1]};
                    g[u * S * 2 + 1] = dv2{ys[4 * u + 2], ys[4 * u + 3]};
                }
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) { acc += ys[u]; cur[u] = nxt[u]; }
        }
    } else
    for (long i = 0; i < n; i += 16) {
        double xs[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) xs[u] = MODE == 2 ? p[(i + u) * S] : x + u;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            if (MODE == 3) {
                const double yr = -xs[u] - crm, tr = sum + yr;
                crm = (tr - sum) - yr;
                sum = tr;
                const double ya = xs[u] - cad, ta = sum + ya;
                cad = (ta - sum) - ya;
                sum = ta;
            } else {
                const double y = d.step(xs[u]);
                if (MODE == 4) acc += e.step(xs[u] * 0.5);
                if (MODE == 1) p[(i + u) * S] = y;
                acc += y;
            }
        }
        x += 1.0;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + lane] = acc + sum;
    if (lane == 0) t[blockIdx.x] = t1 - t0;
}

int main() {
    const long n = 1 << 16, S = 1024;
    const int G = 16;
    double *scr, *out;
    unsigned long long *t;
    const size_t pcm_b = (size_t)1024 * 2646000 * 2;
    CK(hipMalloc(&scr, (size_t)(n + 32) * S * 8 * 2 + pcm_b));
    CK(hipMemset(scr, 0, (size_t)(n + 32) * S * 8 * 2 + pcm_b));
    CK(hipMalloc(&out, G * 64 * 8));
    CK(hipMalloc(&t, G * 8));
    const char *nm[8] = {"filter chain", "filter + store", "filter + load", "kahan remove+add", "two filter chains",
                         "ld+st rows", "ld+st 4-step groups", "fwd: gather + row st"};
    for (int m = 0; m < 8; ++m) {
        hipEvent_t a, b;
        CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        for (int r = 0; r < 2; ++r) {
            CK(hipEventRecord(a));
            switch (m) {
            case 0: hipLaunchKernelGGL(k_chain<0>, dim3(G), dim3(64), 0, 0, scr, S, n, out, t); break;
            case 1: hipLaunchKernelGGL(k_chain<1>, dim3(G), dim3(64), 0, 0, scr, S, n, out, t); break;
            case 2: hipLaunchKernelGGL(k_chain<2>, dim3(G), dim3(64), 0, 0, scr, S, n, out, t); break;
            case 3: hipLaunchKernelGGL(k_chain<3>, dim3(G), dim3(64), 0, 0, scr, S, n, out, t); break;
            case 4: hipLaunchKernelGGL(k_chain<4>, dim3(G), dim3(64), 0, 0, scr, S, n, out, t); break;
            case 5: hipLaunchKernelGGL(k_chain<5>, dim3(G), dim3(64), 0, 0, scr, S, n, out, t); break;
            case 6: hipLaunchKernelGGL(k_chain<6>, dim3(G), dim3(64), 0, 0, scr, S, n, out, t); break;
            default: hipLaunchKernelGGL(k_chain<7>, dim3(G), dim3(64), 0, 0, scr, S, n, out, t); break;
            }
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
        }
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        unsigned long long th[G];
        CK(hipMemcpy(th, t, sizeof th, hipMemcpyDeviceToHost));
        printf("%-20s %.2f ns/step (event), %.2f memtime ticks/step\n", nm[m], ms * 1e6 / n, (double)th[0] / n);
    }
    return 0;
}
