/*
 * bpmx_hilbert.h — fused in-LDS Hilbert magnitude + rolling mean (k_hilbert.hip).
 */
#ifndef BPMX_HILBERT_H
#define BPMX_HILBERT_H

#include <hip/hip_runtime.h>

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

struct HilbPlan {
    int32_t M, N, ns, ntwh, nptab, window;
    int32_t rad[HB_MAXS], B[HB_MAXS], L[HB_MAXS], ptab[HB_MAXS];
    int32_t mf[HB_MAXS];           /* stage runs as an f64 MFMA GEMM (hb_radixp_mfma) */
};

struct HilbArgs {
    const double *yd;              /* [sumNd] decimated filtered signal */
    const int64_t *doff;
    const int32_t *active;
    int32_t f_begin, f_end;        /* a run of recordings with this plan's Nd */
    const double2 *tabs;           /* twiddle hi [ntwh] | lo [128] | prime cos/sin tables */
    double *env;
    unsigned long long *stamps;    /* tools/hbench phase timing only (nullptr) */
};

__global__ void k_hilbert_env(HilbArgs A, HilbPlan P);

/* 1 and the plan, its tables and LDS size when Nd takes the fused kernel; 0 otherwise */
int hilbert_plan(int64_t nd, int window, HilbPlan *P, std::vector<double2> *tabs, size_t *lds_bytes,
                 bool mfma = true);

}  // namespace bpmx

#endif
