// VALU issue cost of single instructions on gfx950 (tools/valu_rate.hip):
// each kernel issues ITERS x 8 independent copies of one instruction (inline
// asm, so the compiler cannot rewrite it) on 4 waves per SIMD over all CUs;
// prints ns and cycles (at 2.4 GHz) per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 2048
#define OP8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)
template <int OP>
__global__ __launch_bounds__(256) void k_rate(double *out, double seed) {
    double x0 = seed + threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    const double a = seed * 0.5;
    float f0 = (float)x0, f1 = f0 + 1, f2 = f0 + 2, f3 = f0 + 3, f4 = f0 + 4, f5 = f0 + 5, f6 = f0 + 6, f7 = f0 + 7;
    const float fa = (float)a;
    for (int i = 0; i < ITERS; ++i) {
#define D(c) if (OP == 0) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x##c) : "v"(a));
#define M(c) if (OP == 1) asm volatile("v_max_f64 %0, %0, %1" : "+v"(x##c) : "v"(a));
#define C(c) if (OP == 2) asm volatile("v_cmp_lt_f64 vcc, %0, %1" : : "v"(x##c), "v"(a) : "vcc");
#define F(c) if (OP == 3) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f##c) : "v"(fa));
#define G(c) if (OP == 4) asm volatile("v_cmp_lt_f32 vcc, %0, %1" : : "v"(f##c), "v"(fa) : "vcc");
#define U(c) if (OP == 5) asm volatile("v_cmp_lt_u64 vcc, %0, %1" : : "v"(x##c), "v"(a) : "vcc");
#define A(c) if (OP == 6) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x##c) : "v"(a));
#define CM(c) if (OP == 7) asm volatile("v_cmp_lt_f64_e64 s[0:1], %0, %1" : : "v"(x##c), "v"(a) : "s0", "s1");
#define CS(c) if (OP == 8) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(f##c) : "v"(fa) : "vcc");
#define MN(c) if (OP == 9) asm volatile("v_min_f32 %0, %0, %1" : "+v"(f##c) : "v"(fa));
        OP8(D) OP8(M) OP8(C) OP8(F) OP8(G) OP8(U) OP8(A) OP8(CM) OP8(CS) OP8(MN)
    }
    out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7 + f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7;
}
int main() {
    const int G = 256 * 4;   // 1024 WGs of 4 waves: 4 waves per SIMD on 256 CUs
    double *o;
    if (hipMalloc(&o, (size_t)G * 256 * 8) != hipSuccess) return 1;
    const char *names[] = {"fma_f64", "max_f64", "cmp_f64", "fma_f32", "cmp_f32", "cmp_u64", "add_f64", "cmp_f64_e64", "cndmask", "min_f32"};
    void (*ks[])(double *, double) = {k_rate<0>, k_rate<1>, k_rate<2>, k_rate<3>, k_rate<4>, k_rate<5>, k_rate<6>, k_rate<7>, k_rate<8>, k_rate<9>};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int k = 0; k < 10; ++k) {
        ks[k]<<<G, 256>>>(o, 1.0001);
        (void)hipEventRecord(e0);
        ks[k]<<<G, 256>>>(o, 1.0001);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double winst = (double)G * 4 * ITERS * 8 / 1024.0;   /* wave-instructions per SIMD */
        printf("%-12s %8.3f ms  %.3f ns = %.2f cycles at 2.4 GHz per wave-instruction per SIMD\n", names[k], ms,
               ms * 1e6 / winst, ms * 1e6 / winst * 2.4);
    }
    return 0;
}
