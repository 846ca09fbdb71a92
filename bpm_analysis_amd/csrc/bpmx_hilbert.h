/*
 * bpmx_hilbert.h — fused in-LDS Hilbert magnitude + rolling mean (k_hilbert.hip).
 */
#ifndef BPMX_HILBERT_H
#define BPMX_HILBERT_H

#include <hip/hip_runtime.h>

#include "bpmx_kernels.h"

#include <cstdint>
#include <cstring>
#include <vector>

namespace bpmx {

constexpr int HB_T = 1024;                 /* threads per recording */
constexpr int HB_KB = 3;                   /* frequencies per butterfly task (odd prime radices) */
constexpr int HB_MAXT = 2;                 /* tasks (HB_KB register-held output pairs each) per thread per stage */
constexpr int HB_RMPER = 20;               /* rolling-mean outputs per thread: Nd <= HB_T * HB_RMPER */
constexpr int HB_MAXS = 16;                /* radix stages */
constexpr int HB_PMAX = 401;               /* largest prime radix (direct DFT cost ~ M p / 2 FMA per stage) */
constexpr size_t HB_LDS_MAX = 160 * 1024;  /* one workgroup per CU */
constexpr int HB_MF_PMIN = 31;             /* odd-prime stages from here on run on the matrix cores (23: slower) */
constexpr int HB_MF_UNITS = 2;             /* 16 x 16 output tiles per wave in such a stage */

/* x / d for 0 <= x, x d < 2^32 by one 32x64-bit multiply: m = floor((2^32 - 1) / d) + 1
 * exceeds 2^32 / d by at most 1, so x m / 2^32 = x / d + eps with eps < 1 / d
 * (exact floor).  The plan's divisors times the kernel's dividends stay
 * below 2^32 (hilbert_plan checks M). */
__host__ __device__ inline uint64_t hb_magic(uint32_t d) { return 0xFFFFFFFFull / d + 1ull; }
__device__ __forceinline__ int hb_div(int x, uint64_t m) { return (int)(((uint64_t)(uint32_t)x * m) >> 32); }

struct HilbPlan {
    int32_t M, N, ns, ntwh, nptab, window;
    int32_t rad[HB_MAXS], B[HB_MAXS], L[HB_MAXS], ptab[HB_MAXS];
    int32_t mf[HB_MAXS];           /* stage runs as an f64 MFMA GEMM (hb_radixp_mfma) */
    /* magic multipliers (hb_magic) of the stage's divisors: L, radix p,
     * h = (p - 1) / 2, k groups (h + HB_KB) / HB_KB, MFMA column tiles (h + 16) / 16 */
    uint64_t dL[HB_MAXS], dP[HB_MAXS], dH[HB_MAXS], dG[HB_MAXS], dT[HB_MAXS];
    int32_t rd[HB_MAXS];           /* stage runs as Rader's 197-point DFT (hb_rader197) */
    int32_t nrtab;                 /* Rader tables after the prime tables: FFT_196(b) / 196 | W_196^e */
    int32_t per;                   /* rolling-mean outputs per thread, ceil(N / HB_T) */
    int32_t cp[HB_MAXS];           /* > 0: small odd prime from exact constants (hb_radixp_const), cp groups */
    int32_t cpo[HB_MAXS];          /* ... its rows' offset in HB_CP (bpmx_dft_consts.h) */
};
constexpr int HB_RD_P = 197;               /* Rader: 197 - 1 = 14 x 14, the 14-point DFTs as 2 x 7 prime-factor */

struct HilbArgs {
    const double *yd;              /* [sumNd] decimated filtered signal */
    const int64_t *doff;
    const int32_t *active;
    int32_t f_begin, f_end;        /* a run of recordings with this plan's Nd */
    const double2 *tabs;           /* twiddle hi [ntwh] | lo [128] | prime cos/sin tables */
    double *env;
    unsigned long long *stamps;    /* tools/hbench phase timing only (nullptr) */
    QuantArgs q;                   /* q.n_levels > 0: also the recording's quantiles (qr_select) into q.qv */
    /* fy != 0: yd of the full decimation tiles (bt blocks each) made here from
     * k_native_blocks' gamma rows and k_native_carry's tile carries, with
     * k_native_yd's arithmetic (yd_j = alpha_b . Qe_t + beta_b . S0_t +
     * gamma_j), straight into the FFT buffer and into ys for the magnitude
     * pass's second read; the rest of yd (partial tile, tail) comes from
     * k_native_carry's writes to yd */
    int32_t fy;
    int32_t bt, gstr;              /* blocks per tile (even, <= 64); gamma row stride */
    const double *gam;             /* [tile][gstr] */
    const double *car;             /* [tile][8]: S0_t | Qe_t */
    const double *al, *be;         /* [64][4] each: alpha_b, beta_b */
    const int64_t *toff;           /* [F] first tile of recording f */
    double *ys;                    /* recording f's full-tile yd at hb_ys_off(doff[f], f): 128-byte aligned,
                                    * no cache line shared with another recording */
};
__host__ __device__ inline int64_t hb_ys_off(int64_t d0, int64_t f) { return ((d0 + 15) & ~(int64_t)15) + 16 * f; }

__global__ void k_hilbert_env(HilbArgs A, HilbPlan P);

/* 1 and the plan, its tables and LDS size when Nd takes the fused kernel; 0 otherwise */
int hilbert_plan(int64_t nd, int window, HilbPlan *P, std::vector<double2> *tabs, size_t *lds_bytes,
                 bool mfma = true, bool rader = true, bool cprime = true);

}  // namespace bpmx

#endif
