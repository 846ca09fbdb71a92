/*
 * k_envelope_native.hip — native mode envelope (north_star ordering):
 *   sosfiltfilt(butter(2,[20,150],'band',fs,'sos'), x) at the native rate
 *   -> y[::ds] -> |hilbert| -> centred rolling mean (window sr//10)
 * oracle: scipy/signal/_signaltools.py:4718-4829 (sosfiltfilt), :2318 (hilbert),
 * composed as SURVEY.md §8(a) A13 defines; tolerance 1e-9 relative on env.
 *
 * sosfiltfilt is linear and time-invariant, so over one decimation block of
 * ds samples the per-sample recursion collapses to 8 dot products (the
 * block's forward-state increment u_j and backward-state increment v_j), and
 * over a tile of T blocks the two block recursions collapse again to tile
 * carries (bpm_analysis_amd/native_tables.py: tables, model_tiled):
 *
 *   k_native_blocks  every PCM sample read once from HBM (coalesced tile
 *                    loads, LDS staging), 8 f64 FMA per sample; then, per
 *                    tile, two Kogge-Stone scans over the 64 lanes (forward
 *                    local states, backward suffix sums) leave ONE f64 per
 *                    block (gamma_j) and 64 B per tile of carry inputs.
 *   k_native_carry   one wave per recording: the 15-sample head pad, the
 *                    tile-to-tile carries S0_t (forward) and Qe_t (backward),
 *                    the partial last tile and the <= ds+15-sample tail by
 *                    exact recursion.
 *   k_native_yd      yd_j = alpha_b . Qe_t + beta_b . S0_t + gamma_j.
 *   rocFFT           R2C + C2R (Hilbert transform), one plan pair per (Nd, batch).
 *   k_hilbert_rotate   -i on the half spectrum (C2R of it = N x Hilbert transform).
 *   k_native_env     |z| = sqrt(y^2 + H^2) and the centred rolling mean, LDS-tiled.
 */
#include <rocfft/rocfft.h>

#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include <complex>

#include "bpmx_common.h"
#include "bpmx_kernels.h"
#include "bpmx_native.h"
#include "bpmx_hilbert.h"
#ifndef BPMX_NM_POLICY
#define BPMX_NM_POLICY " nt"   /* cache policy of the metric block kernel's PCM stream: non-temporal (r05 A/B: the kernel -1.8 %, k_native_yd +0.006 ms; "" = default) */
#endif
#include "bpmx_qsel.h"
#include "bpmx_xlane.h"

namespace bpmx {

/* table layout (native_tables.pack).  Every block/tile table is in MODAL
 * coordinates S' = V^-1 S, in which the cascade's state matrix is two 2x2
 * rotation-scaling blocks (its two conjugate pole pairs); TB_V holds V (the
 * original-coordinate slot TB_A is not needed on the device). */
enum { TB_A = 0, TB_V = 0, TB_B = 16, TB_C = 20, TB_D = 24, TB_M = 25, TB_P = 41, TB_ZI = 57, TB_COEF = 64 };

/* tile tables, after the coefficient rows (native_tables.tile_tables):
 * TT_KPOW holds M'^(2^k), k = 0..5, as (a1, b1, a2, b2) per power — the
 * blocks [[a, b], [-b, a]] — in its first 24 doubles; TT_VI = V^-1 */
enum { TT_KPOW = 0, TT_MT = 96, TT_G0 = 112, TT_ALPHA = 128, TT_BETA = 384, TT_VI = 640, TT_SIZE = 656 };
constexpr int NAT_PART = 16;          /* doubles per partial-tile block record: u4 v4 x pad3 S4 */
constexpr int NAT_DSMAX = 1280;       /* decimation factors up to fs/300 - 1 at 384 kHz (tail buffers) */

struct NatTile {
    int64_t s0;                         /* first frame of the tile (index into pcm frames) */
    int64_t gbase;                      /* tile index * gstr: the tile's gamma row (128-byte aligned) */
    int64_t ybase;                      /* doff[f] + j0: yd index of the tile's first block */
    int32_t j0, nb;                     /* first block, blocks of the file */
    int32_t f, pad;
};

/* tile headers through the scalar cache (constant address space): a vector
 * load would wait in vmcnt order behind the in-flight prefetch */
__device__ __forceinline__ NatTile nat_tile_ld(const NatTile *p, int64_t t) {
    typedef const __attribute__((address_space(4))) int64_t c64;
    c64 *q = (c64 *)(p + __builtin_amdgcn_readfirstlane((int)t));   /* t is wave-uniform by contract */
    NatTile r;
    r.s0 = q[0]; r.gbase = q[1]; r.ybase = q[2];
    const int64_t a = q[3], b = q[4];
    r.j0 = (int32_t)a; r.nb = (int32_t)(a >> 32); r.f = (int32_t)b; r.pad = (int32_t)(b >> 32);
    return r;
}

struct NatBlockArgs {
    const void *pcm;
    const NatTile *tiles;
    int64_t n_tiles, total;       /* tiles; samples in pcm (int16 path) */
    int32_t bt, channels, ds;     /* blocks per (full) tile */
    const double *tab, *tt;       /* block tables; tile tables */
    double *gam;                  /* [n_tiles][gstr]: one aligned row per tile */
    double *agg;                  /* [n_tiles][8]: forward tile sum, backward R_0 */
    double *part;                 /* [F][64][NAT_PART]: raw blocks of each file's partial last tile */
};

struct NatCarryArgs {
    const void *pcm;
    const int64_t *foff, *doff, *boff, *toff;
    const int32_t *active;
    int32_t n_files, dtype, channels, ds, bt;
    const double *tab, *tt, *agg;
    double *part;                  /* partial-tile blocks; k_native_carry adds their states */
    double *carry;                 /* [n_tiles][8]: S0_t, Qe_t */
    double *yd;
    InitOutArgs io;                /* io.flags non-null: reset recording f's outputs first */
    const double *ttab;            /* tail tables (NAT_TT_ROWS rows of 16): C A^m | A^m B | A^m zi | h_m */
};
/* k_native_carry's tail recursion, lane-parallel: the exact per-sample
 * recursion z' = A z + B u, y = C z + D u (SosStep, original basis) over the
 * nt <= NAT_TT_PAR tail samples as its impulse response, row m of the tail
 * table holding C A^m, A^m B, A^m zi and h_m (h_0 = D, h_m = C A^(m-1) B),
 * built on the host in long double from the same coefficients */
constexpr int NAT_TT_ROWS = NAT_DSMAX + 20, NAT_TT_PAR = 320;

struct NatYdArgs {
    const NatTile *tiles;
    const int32_t *skip;            /* [F] optional: recordings whose yd k_hilbert_env makes */
    int32_t bt;
    const double *tt, *carry, *gam;
    double *yd;
};

struct NatEnvArgs {
    const double *y;               /* [sumNd] decimated filtered signal (real part) */
    const double *h;               /* [sumNd] N x Hilbert transform (unnormalised C2R) */
    const int64_t *doff;
    const int32_t *active;
    int32_t n_files, window;
    double *env;
    const int32_t *skip;           /* [F] 1: envelope already written by k_hilbert_env */
};

/* ---------------------------------------------------------------------- */
/* ---------------------------------------------------------------------- */
/* 4x4 affine-map helpers (row-major matrices in registers) */
struct V4 { double a, b, c, d; };
struct M4 { double m[16]; };

__device__ __forceinline__ V4 mv(const M4 &M, const V4 &x) {
    V4 r;
    r.a = __builtin_fma(M.m[0], x.a, __builtin_fma(M.m[1], x.b, __builtin_fma(M.m[2], x.c, M.m[3] * x.d)));
    r.b = __builtin_fma(M.m[4], x.a, __builtin_fma(M.m[5], x.b, __builtin_fma(M.m[6], x.c, M.m[7] * x.d)));
    r.c = __builtin_fma(M.m[8], x.a, __builtin_fma(M.m[9], x.b, __builtin_fma(M.m[10], x.c, M.m[11] * x.d)));
    r.d = __builtin_fma(M.m[12], x.a, __builtin_fma(M.m[13], x.b, __builtin_fma(M.m[14], x.c, M.m[15] * x.d)));
    return r;
}
/* block-diagonal rotation form: r = (a1, b1, a2, b2), M = diag([[a1, b1], [-b1, a1]], [[a2, b2], [-b2, a2]]) */
__device__ __forceinline__ V4 mv_rot(const double *r, const V4 &x) {
    const double a1 = r[0], b1 = r[1], a2 = r[2], b2 = r[3];
    return V4{__builtin_fma(a1, x.a, b1 * x.b), __builtin_fma(a1, x.b, -b1 * x.a), __builtin_fma(a2, x.c, b2 * x.d),
              __builtin_fma(a2, x.d, -b2 * x.c)};
}
__device__ __forceinline__ V4 add4(const V4 &x, const V4 &y) { return V4{x.a + y.a, x.b + y.b, x.c + y.c, x.d + y.d}; }
/* acc + rot(r) x with the sum folded into the rotation's FMAs (two per component) */
__device__ __forceinline__ V4 acc_rot(const V4 &acc, const double *r, const V4 &x) {
    const double a1 = r[0], b1 = r[1], a2 = r[2], b2 = r[3];
    return V4{__builtin_fma(a1, x.a, __builtin_fma(b1, x.b, acc.a)), __builtin_fma(a1, x.b, __builtin_fma(-b1, x.a, acc.b)),
              __builtin_fma(a2, x.c, __builtin_fma(b2, x.d, acc.c)), __builtin_fma(a2, x.d, __builtin_fma(-b2, x.c, acc.d))};
}
__device__ __forceinline__ M4 mm(const M4 &X, const M4 &Y) {
    M4 R;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            R.m[i * 4 + j] = __builtin_fma(X.m[i * 4 + 0], Y.m[0 * 4 + j],
                             __builtin_fma(X.m[i * 4 + 1], Y.m[1 * 4 + j],
                             __builtin_fma(X.m[i * 4 + 2], Y.m[2 * 4 + j], X.m[i * 4 + 3] * Y.m[3 * 4 + j])));
    return R;
}
__device__ __forceinline__ M4 eye4() {
    M4 R;
#pragma unroll
    for (int i = 0; i < 16; ++i) R.m[i] = (i % 5 == 0) ? 1.0 : 0.0;
    return R;
}
__device__ __forceinline__ M4 shfl_up_m(const M4 &X, int d) {
    M4 R;
#pragma unroll
    for (int i = 0; i < 16; ++i) R.m[i] = __shfl_up(X.m[i], d);
    return R;
}
__device__ __forceinline__ M4 shfl_down_m(const M4 &X, int d) {
    M4 R;
#pragma unroll
    for (int i = 0; i < 16; ++i) R.m[i] = __shfl_down(X.m[i], d);
    return R;
}
__device__ __forceinline__ V4 shfl_v(const V4 &x, int src) {
    return V4{__shfl(x.a, src), __shfl(x.b, src), __shfl(x.c, src), __shfl(x.d, src)};
}
__device__ __forceinline__ V4 shfl_up_v(const V4 &x, int d) {
    return V4{__shfl_up(x.a, d), __shfl_up(x.b, d), __shfl_up(x.c, d), __shfl_up(x.d, d)};
}
__device__ __forceinline__ V4 shfl_down_v(const V4 &x, int d) {
    return V4{__shfl_down(x.a, d), __shfl_down(x.b, d), __shfl_down(x.c, d), __shfl_down(x.d, d)};
}
/* register-only V4 shifts (bpmx_xlane.h), for the tile epilogue's scans */
template <int D>
__device__ __forceinline__ V4 xl_up_v(const V4 &x) {
    return V4{xl_up<D>(x.a), xl_up<D>(x.b), xl_up<D>(x.c), xl_up<D>(x.d)};
}
template <int D>
__device__ __forceinline__ V4 xl_down_v(const V4 &x) {
    return V4{xl_down<D>(x.a), xl_down<D>(x.b), xl_down<D>(x.c), xl_down<D>(x.d)};
}
__device__ __forceinline__ M4 mpow(const M4 &X, int64_t e) {
    M4 R = eye4(), P = X;
    while (e > 0) {
        if (e & 1) R = mm(P, R);
        P = mm(P, P);
        e >>= 1;
    }
    return R;
}

/* exact per-sample cascade step in scipy _sosfilt operation order */
struct SosStep {
    double s[12];
    __device__ __forceinline__ double step(V4 &z, double u) const {
        const double x1 = s[0] * u + z.a;
        const double z00 = s[1] * u - s[4] * x1 + z.b;
        const double z01 = s[2] * u - s[5] * x1;
        const double y = s[6] * x1 + z.c;
        const double z10 = s[7] * x1 - s[10] * y + z.d;
        const double z11 = s[8] * x1 - s[11] * y;
        z = V4{z00, z01, z10, z11};
        return y;
    }
};

/* k_native_blocks: per decimation block j of every file
 *   u_j = sum_{i<ds} F_i x[j*ds+i],  v_j = sum_{i<=ds} G_i x[j*ds+i]          */

template <int DT, bool MULTI>
__device__ __forceinline__ double nat_frame(const void *__restrict__ pcm, int ch, int64_t frame) {
    if (!MULTI) {
        switch (DT) {
        case BPMX_DT_U8: return (double)((const uint8_t *)pcm)[frame];
        case BPMX_DT_I16: return (double)((const int16_t *)pcm)[frame];
        case BPMX_DT_I32: return (double)((const int32_t *)pcm)[frame];
        case BPMX_DT_F32: return (double)((const float *)pcm)[frame];
        default: return ((const double *)pcm)[frame];
        }
    }
    return frame_value(pcm, DT, ch, frame);
}

/* Per-tile epilogue shared by the block kernels (all 64 lanes call it; lane b
 * holds block j0+b's u, v and first sample x).  A full tile (bt blocks) is
 * reduced to gamma_b = C R_b + D C loc_b + D^2 x_b per block plus its carry
 * inputs (forward tile sum, backward R_0); the file's partial last tile keeps
 * its raw blocks for k_native_carry's exact recursion. */
__device__ __forceinline__ V4 nat_ld4(const double *p) { return V4{p[0], p[1], p[2], p[3]}; }
__device__ __forceinline__ M4 nat_ld16(const double *p) {
    M4 r;
#pragma unroll
    for (int i = 0; i < 16; ++i) r.m[i] = p[i];
    return r;
}
__device__ __forceinline__ double dot4(const V4 &a, const V4 &b) {
    return __builtin_fma(a.a, b.a, __builtin_fma(a.b, b.b, __builtin_fma(a.c, b.c, a.d * b.d)));
}

/* The epilogue's constants, staged in LDS once per workgroup: a vector load
 * here would sit behind the next tile's prefetch in vmcnt order and stall the
 * wave until the whole prefetch landed. */
enum { ET_KPOW = 0, ET_P = 24, ET_C = 40, ET_D = 44, ET_SIZE = 45 };
__device__ __forceinline__ void nat_stage_epilogue_tables(const NatBlockArgs &A, double *et) {
    for (int i = threadIdx.x; i < ET_SIZE; i += blockDim.x) {
        double v;
        if (i < ET_P) v = A.tt[TT_KPOW + i];
        else if (i < ET_C) v = A.tab[TB_P + i - ET_P];
        else if (i < ET_D) v = A.tab[TB_C + i - ET_C];
        else v = A.tab[TB_D];
        et[i] = v;
    }
}

__device__ __forceinline__ void nat_tile_epilogue(const NatBlockArgs &A, const double *et, const NatTile &tl,
                                                  int64_t t, int lane, bool valid, V4 u, V4 v, double x) {
    const int bt = A.bt;
    const int Lt = tl.nb - tl.j0 < bt ? tl.nb - tl.j0 : bt;
    if (Lt < bt) {                                        /* partial last tile: raw blocks */
        if (valid) {
            double *pp = A.part + ((int64_t)tl.f * 64 + lane) * NAT_PART;
            pp[0] = u.a; pp[1] = u.b; pp[2] = u.c; pp[3] = u.d;
            pp[4] = v.a; pp[5] = v.b; pp[6] = v.c; pp[7] = v.d;
            pp[8] = x;
        }
        return;
    }
    if (!valid) { u = V4{0, 0, 0, 0}; v = V4{0, 0, 0, 0}; x = 0; }
    /* incl_b = sum_{c<=b} M^(b-c) u_c  (modal: M^d is two 2x2 rotation blocks) */
    V4 incl = u;
    /* Kogge-Stone steps; the one-lane shifts are DPP (wave_shr/shl:1), the
     * longer ones ds_bpermute (measured: the DPP + permlane composites of
     * bpmx_xlane.h cost more VALU than they save in LDS latency here) */
#define NAT_UP(K)                                                            \
    {                                                                        \
        const V4 y = K == 0 ? xl_up_v<1>(incl) : shfl_up_v(incl, 1 << K);   \
        if (lane >= (1 << K)) incl = acc_rot(incl, et + ET_KPOW + 4 * K, y);   \
    }
    NAT_UP(0) NAT_UP(1) NAT_UP(2) NAT_UP(3) NAT_UP(4) NAT_UP(5)
#undef NAT_UP
    V4 loc = xl_up_v<1>(incl);
    if (lane == 0) loc = V4{0, 0, 0, 0};
    /* R_b = sum_{c>=b} M^(c-b) (P loc_c + v_c) */
    V4 R = valid ? add4(mv(nat_ld16(et + ET_P), loc), v) : V4{0, 0, 0, 0};
#define NAT_DOWN(K)                                                          \
    {                                                                        \
        const V4 y = K == 0 ? xl_down_v<1>(R) : shfl_down_v(R, 1 << K);      \
        if (lane + (1 << K) < 64) R = acc_rot(R, et + ET_KPOW + 4 * K, y);     \
    }
    NAT_DOWN(0) NAT_DOWN(1) NAT_DOWN(2) NAT_DOWN(3) NAT_DOWN(4) NAT_DOWN(5)
#undef NAT_DOWN
    const V4 C = nat_ld4(et + ET_C);
    const double D = et[ET_D];
    if (valid) A.gam[tl.gbase + lane] = dot4(C, R) + D * dot4(C, loc) + D * D * x;
    double *ag = A.agg + t * 8;
    if (lane == bt - 1) { ag[0] = incl.a; ag[1] = incl.b; ag[2] = incl.c; ag[3] = incl.d; }
    if (lane == 0) { ag[4] = R.a; ag[5] = R.b; ag[6] = R.c; ag[7] = R.d; }
}

/* int16 mono fast path.  Persistent single-wave workgroups walk the tile
 * list (bt consecutive blocks of one file per tile).  A tile's samples arrive
 * with coalesced 16-byte loads into registers — issued one tile AHEAD, so
 * HBM latency hides behind the current tile's FMAs — then go through LDS,
 * where lane b reads block b's ds+1 samples (lane stride ds/2 dwords: odd for
 * the usual ds, conflict-free).  The 8 coefficients of each sample are
 * wave-uniform scalar loads. */
constexpr int NB_RCH = 20;              /* 16-byte chunks per lane per tile: <= 10240 samples */

__device__ __forceinline__ double nat_lo16(uint32_t w) { return (double)(int)(int16_t)(w & 0xFFFFu); }
__device__ __forceinline__ double nat_hi16(uint32_t w) { return (double)((int)w >> 16); }

typedef uint32_t nat_u4 __attribute__((ext_vector_type(4)));

/* `coef` is passed separately as __restrict__ so its loads become scalar
 * (wave-uniform) loads: the compiler must know the stores cannot alias it */
__global__ __launch_bounds__(64) void k_native_blocks_i16(NatBlockArgs A, const double *__restrict__ coef) {
    typedef nat_u4 u4;
    __shared__ u4 tile[NB_RCH * 64];
    __shared__ double s_et[ET_SIZE];
    nat_stage_epilogue_tables(A, s_et);
    const int lane = threadIdx.x;
    const int16_t *pcm = (const int16_t *)A.pcm;
    const int64_t total = A.total;
    const int ds = A.ds, bt = A.bt;
    const int nch = (7 + bt * ds + 1 + 7) >> 3;           /* chunks a tile may touch */
    auto issue = [&](int64_t t, u4 *reg, int &off) {
        const int64_t s0 = nat_tile_ld(A.tiles, t).s0;
        const int64_t a0 = s0 & ~(int64_t)7;
        off = (int)(s0 - a0);
#pragma unroll
        for (int r = 0; r < NB_RCH; ++r) {
            const int q = r * 64 + lane;
            const int64_t c = a0 + (int64_t)q * 8;
            if (q < nch && c + 8 <= total) __builtin_memcpy(&reg[r], pcm + c, 16);
            else reg[r] = u4{0, 0, 0, 0};      /* a partial last chunk is patched in LDS */
        }
    };
    u4 reg[NB_RCH];
    int off = 0;
    int64_t t = blockIdx.x;
    if (t < A.n_tiles) issue(t, reg, off);
    while (t < A.n_tiles) {
        const NatTile tl = nat_tile_ld(A.tiles, t);
#pragma unroll
        for (int r = 0; r < NB_RCH; ++r) tile[r * 64 + lane] = reg[r];
        const int coff = off;
        {
            const int64_t a0 = tl.s0 - coff, tail0 = total & ~(int64_t)7;
            if ((total & 7) && a0 + (int64_t)nch * 8 > tail0 && lane < (int)(total & 7))
                ((int16_t *)tile)[tail0 - a0 + lane] = pcm[tail0 + lane];
        }
        __syncthreads();
        const int64_t tn = t + gridDim.x;
        if (tn < A.n_tiles) issue(tn, reg, off);
        const int j = tl.j0 + lane;
        const bool valid = lane < bt && j < tl.nb;
        double u0 = 0, u1 = 0, u2 = 0, u3 = 0, v0 = 0, v1 = 0, v2 = 0, v3 = 0, x0 = 0;
        if (valid) {
            const int base = coff + lane * ds;                        /* halfword index in the tile */
            const uint32_t *wp = (const uint32_t *)tile + (base >> 1);
            const uint32_t sh = (base & 1) ? 16u : 0u;
            auto acc = [&](double xv, const double *c) {
                u0 = __builtin_fma(c[0], xv, u0); u1 = __builtin_fma(c[1], xv, u1);
                u2 = __builtin_fma(c[2], xv, u2); u3 = __builtin_fma(c[3], xv, u3);
                v0 = __builtin_fma(c[4], xv, v0); v1 = __builtin_fma(c[5], xv, v1);
                v2 = __builtin_fma(c[6], xv, v2); v3 = __builtin_fma(c[7], xv, v3);
            };
            const int L = ds + 1;                                    /* row ds has F = 0 */
            int i = 0;
            for (; i + 8 <= L; i += 8) {
                const uint32_t *p = wp + i / 2;
                const uint32_t w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3], w4 = p[4];
                const uint32_t d0 = __builtin_amdgcn_alignbit(w1, w0, sh);
                const uint32_t d1 = __builtin_amdgcn_alignbit(w2, w1, sh);
                const uint32_t d2 = __builtin_amdgcn_alignbit(w3, w2, sh);
                const uint32_t d3 = __builtin_amdgcn_alignbit(w4, w3, sh);
                const double *cr = coef + (int64_t)i * 8;
                acc(nat_lo16(d0), cr + 0);  acc(nat_hi16(d0), cr + 8);
                acc(nat_lo16(d1), cr + 16); acc(nat_hi16(d1), cr + 24);
                acc(nat_lo16(d2), cr + 32); acc(nat_hi16(d2), cr + 40);
                acc(nat_lo16(d3), cr + 48); acc(nat_hi16(d3), cr + 56);
            }
            const int16_t *th = (const int16_t *)tile;
            for (; i < L; ++i) acc((double)th[base + i], coef + (int64_t)i * 8);
            x0 = (double)th[base];
        }
        nat_tile_epilogue(A, s_et, tl, t, lane, valid, V4{u0, u1, u2, u3}, V4{v0, v1, v2, v3}, x0);
        __syncthreads();
        t = tn;
    }
}

/* generic path (other sample formats, multi-channel): one wave per tile, each
 * lane reads its block straight from global memory */
template <int DT, bool MULTI>
__global__ __launch_bounds__(64) void k_native_blocks_gen(NatBlockArgs A) {
    const int64_t t = blockIdx.x;
    if (t >= A.n_tiles) return;
    __shared__ double s_et[ET_SIZE];
    nat_stage_epilogue_tables(A, s_et);
    __syncthreads();
    const NatTile tl = nat_tile_ld(A.tiles, t);
    const int lane = threadIdx.x, ds = A.ds;
    const int j = tl.j0 + lane;
    const bool valid = lane < A.bt && j < tl.nb;
    double u0 = 0, u1 = 0, u2 = 0, u3 = 0, v0 = 0, v1 = 0, v2 = 0, v3 = 0, x0 = 0;
    if constexpr (DT == BPMX_DT_I16 && MULTI) {
        /* int16 stereo: lane = block strides ds frames through global memory
         * (64 cache lines per load instruction), so the tile's frames are
         * first staged in LDS with coalesced dword loads (one stereo frame
         * each); same frames, same arithmetic as frame_value */
        if (A.channels == 2 && ((uintptr_t)A.pcm & 3) == 0) {
            __shared__ uint32_t s_fr[NB_RCH * 512 + 1];
            const int nvalid = (int)min((int64_t)A.bt, (int64_t)tl.nb - tl.j0);
            const int nfr = nvalid * ds + 1;                 /* frames [s0, s0 + nvalid ds] */
            const uint32_t *src = (const uint32_t *)A.pcm + tl.s0;
            for (int k = lane; k < nfr; k += 64) s_fr[k] = src[k];
            __syncthreads();
            if (valid) {
                const double *__restrict__ coef = A.tab + TB_COEF;
                const uint32_t *fr = s_fr + lane * ds;
                for (int i = 0; i <= ds; ++i) {
                    const uint32_t w = fr[i];
                    const double xv = ((double)(int16_t)(w & 0xFFFFu) + (double)(int16_t)(w >> 16)) / 2.0;
                    const double *c = coef + i * 8;
                    u0 = __builtin_fma(c[0], xv, u0); u1 = __builtin_fma(c[1], xv, u1);
                    u2 = __builtin_fma(c[2], xv, u2); u3 = __builtin_fma(c[3], xv, u3);
                    v0 = __builtin_fma(c[4], xv, v0); v1 = __builtin_fma(c[5], xv, v1);
                    v2 = __builtin_fma(c[6], xv, v2); v3 = __builtin_fma(c[7], xv, v3);
                    if (i == 0) x0 = xv;
                }
            }
            nat_tile_epilogue(A, s_et, tl, t, lane, valid, V4{u0, u1, u2, u3}, V4{v0, v1, v2, v3}, x0);
            return;
        }
    }
    if (valid) {
        const double *__restrict__ coef = A.tab + TB_COEF;
        const int64_t fb = tl.s0 + (int64_t)lane * ds;
        for (int i = 0; i <= ds; ++i) {
            const double xv = nat_frame<DT, MULTI>(A.pcm, A.channels, fb + i);
            const double *c = coef + i * 8;                      /* row ds has F = 0 */
            u0 = __builtin_fma(c[0], xv, u0); u1 = __builtin_fma(c[1], xv, u1);
            u2 = __builtin_fma(c[2], xv, u2); u3 = __builtin_fma(c[3], xv, u3);
            v0 = __builtin_fma(c[4], xv, v0); v1 = __builtin_fma(c[5], xv, v1);
            v2 = __builtin_fma(c[6], xv, v2); v3 = __builtin_fma(c[7], xv, v3);
            if (i == 0) x0 = xv;
        }
    }
    nat_tile_epilogue(A, s_et, tl, t, lane, valid, V4{u0, u1, u2, u3}, V4{v0, v1, v2, v3}, x0);
}

/* ---------------------------------------------------------------------- */
/* int16 mono, exact-integer path on the matrix cores.
 *
 * The 8 block projections are a GEMM: [64 blocks x K samples] x [K x 8
 * coefficients], K = ds + 1 padded to 32 * KS.  The f64 VALU form above is
 * bound by 8 f64 FMAs per sample (~2x the HBM time of reading the PCM), so the
 * coefficients are quantised instead: q_c,i = round(coef_c,i * 2^(P - e_c))
 * with 2^e_c >= max_i |coef_c,i| (|q| <= 2^54, i.e. 2^-55 of the column's
 * largest coefficient — below f64 rounding of the coefficient itself) and
 * split into 7 balanced base-256 digits d_r.  A sample splits exactly into
 * x = 256 h + (l - 128) + 128 with h = x >> 8 and l - 128 = (x & 255) ^ 0x80,
 * both int8, so
 *     sum_i q_i x_i = sum_r 256^r [ sum_i d_r,i (l_i - 128) + sum_i d_(r-1),i h_i ] + 128 sum_i q_i
 * and each bracket is one int32 accumulator row of v_mfma_i32_32x32x32_i8
 * (the 128 sum q term enters as the accumulators' initial value, digit by
 * digit).  8 digit rows x 8 coefficients = two 32-row M tiles; per 32-block N
 * tile and K step four MFMAs.  Every sum is exact in int32; the 8 rows
 * combine exactly into two int64 halves, and the only rounding is the final
 * conversion to f64 (then an exact power-of-two scale).
 *
 * Fragment maps (32x32x32 i8): A lane l = row (l & 31) x 16 consecutive k of
 * k-group l >> 5, B likewise with column (l & 31); the same (lane half, byte)
 * -> k map on both operands makes the product the sum over the K step.
 * Accumulator: lane l = column (block) l & 31, register 4q + i = row
 * 8q + 4(l >> 5) + i, which the tables assign to coefficient 2q + (l >> 5),
 * digit row 4t + i (t = M tile): each lane ends with every digit row of 4
 * coefficients of its block, and one lane-half exchange gives lane b all 8
 * of block b. */
typedef int32_t nm_i4 __attribute__((ext_vector_type(4)));
typedef int32_t nm_i16 __attribute__((ext_vector_type(16)));

/* Feeding it: a tile is 64 blocks (~18.7 KB of PCM).  With a tile per wave
 * in flight the chip sits at ~5 TB/s, so tiles travel HBM -> LDS directly by
 * LDS-DMA (global_load_lds_dwordx4, no registers), one 18 KB slot per wave:
 * the DMA of the wave's next tile is issued as soon as the matrix phase has
 * read the slot and flies during this tile's epilogue.  Four waves per
 * workgroup, two workgroups per CU: 8 slots (147 KB) + the shared tables fit
 * the 160 KiB LDS, and with 8 waves interleaving, ~6 of the 8 tiles are in
 * flight at any time. */
constexpr int NM_WAVES = 4;
#ifndef BPMX_NM_SLOTS
#define BPMX_NM_SLOTS 1
#endif
constexpr int NM_SLOTS = BPMX_NM_SLOTS;             /* LDS tile slots per wave */
constexpr int NM_MINW = 2;                        /* waves per SIMD the register budget must allow */
constexpr int NM_NDMA = 18;                      /* DMA wave-instructions per tile, always all issued, all lanes on */
constexpr int NM_SLOT_CH = NM_NDMA * 64;          /* 16-byte chunks per slot (18,432 B) */

/* blocks per tile the slot holds: every k of the last block's K steps (+2
 * samples for the odd-offset align) must stay inside the slot */
__host__ __device__ constexpr int nm_tile_blocks(int ds, int ks) {
    return ((NM_SLOT_CH * 8 - 7 - 32 * ks - 2) / ds + 1) < 64 ? ((NM_SLOT_CH * 8 - 7 - 32 * ks - 2) / ds + 1) : 64;
}

template <int KS>
__global__ __launch_bounds__(64 * NM_WAVES, NM_MINW) void k_native_blocks_mfma(NatBlockArgs A, const nm_i4 *__restrict__ afrag,
                                                                      const nm_i16 *__restrict__ ainit,
                                                                      const double *__restrict__ cscale) {
    typedef nat_u4 u4;
    __shared__ u4 slots[NM_WAVES * NM_SLOTS][NM_SLOT_CH];
    __shared__ double s_et[ET_SIZE];
    __shared__ nm_i16 s_init[4];                        /* accumulator start values [M tile][lane half] */
    nat_stage_epilogue_tables(A, s_et);
    for (int i = threadIdx.x; i < 4; i += blockDim.x) s_init[i] = ainit[(i >> 1) * 64 + (i & 1) * 32];
    /* wave-uniform (readfirstlane): tile headers must come through the scalar cache */
    const int lane = lane_id(), hf = lane >> 5, wv = __builtin_amdgcn_readfirstlane(wave_id());
    const int16_t *pcm = (const int16_t *)A.pcm;
    const int64_t total = A.total;
    const int ds = A.ds, bt = A.bt;
    const int nch = (7 + bt * ds + 1 + 7) >> 3;          /* <= NM_SLOT_CH (host: nm_tile_blocks) */
    nm_i4 af[2][KS][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int v = 0; v < 2; ++v) af[t][s][v] = afrag[((t * KS + s) * 2 + v) * 64 + lane];
    double sc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) sc[q] = cscale[2 * q + hf];
    __syncthreads();                                      /* s_et, s_init */

    /* chunk q of a tile -> slot chunk q (lane l of DMA r moves chunk 64r + l) */
    /* Exactly NM_NDMA instructions per tile with every lane on (the vmcnt
     * arithmetic below depends on it): chunks past the tile or the batch
     * re-read the batch's last whole chunk into the slot's spare room. */
    const int64_t clast = (total & ~(int64_t)7) - 8;
    auto dma = [&](int64_t s0, u4 *slot) {
        const int64_t a0 = s0 & ~(int64_t)7;
        /* the chunk count opaque here: otherwise the per-r lane masks
         * (q < nch) are hoisted out of the tile loop into ~36 SGPRs, which
         * spill, and every refill pays a readlane per mask */
        int nchv = nch, lanev = lane;
        asm volatile("" : "+s"(nchv), "+v"(lanev));
#pragma unroll
        for (int r = 0; r < NM_NDMA; ++r) {
            const int q = r * 64 + lanev;
            int64_t c = a0 + (int64_t)q * 8;
            c = (q < nchv && c + 8 <= total) ? c : clast;
            /* inline asm, not __builtin_amdgcn_global_load_lds: the compiler cannot
             * tell the slots apart and would put a vmcnt(0) before the next LDS
             * read, draining the other slot's DMA too.  The waits are explicit
             * (vmcnt below); a compiler-generated wait can only over-wait. */
            const uint32_t m0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)(slot + r * 64);
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" BPMX_NM_POLICY
                         :: "v"(pcm + c), "s"(m0) : "memory");
        }
    };
    const int64_t stride = (int64_t)gridDim.x * NM_WAVES;
    int64_t t = (int64_t)blockIdx.x * NM_WAVES + wv;
    /* Tile headers travel one tile ahead: the next header's scalar load is
     * issued before this tile's DMA wait, so the refill below never waits on
     * a header round trip (with one slot per wave that wait would sit between
     * the slot's read and its next DMA). */
    NatTile tl{};
    if (t < A.n_tiles) tl = nat_tile_ld(A.tiles, t);
    if (t < A.n_tiles) dma(tl.s0, slots[NM_SLOTS * wv]);
    if (NM_SLOTS == 2 && t + stride < A.n_tiles) dma(nat_tile_ld(A.tiles, t + stride).s0, slots[NM_SLOTS * wv + 1]);
    for (int k = 0; t < A.n_tiles; ++k, t += stride) {
        u4 *slot = slots[NM_SLOTS * wv + (NM_SLOTS == 2 ? (k & 1) : 0)];
        const int64_t tr = t + NM_SLOTS * stride;               /* the tile this slot is refilled with */
        NatTile tn{};
        if (tr < A.n_tiles) tn = nat_tile_ld(A.tiles, tr);
        /* Issued after this tile's DMA: the next tile's NM_NDMA (when there is
         * a next tile) and a few epilogue stores.  vmcnt retires in issue
         * order, so <= NM_NDMA outstanding covers this tile (over-waiting by
         * at most the stores' count of the next tile's chunks); with no next
         * tile, wait for everything. */
        if (NM_SLOTS == 2 && t + stride < A.n_tiles) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NM_NDMA) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        /* the slot is the scarce resource: its reader runs ahead of the other
         * waves' epilogues until the refill is issued */
        __builtin_amdgcn_s_setprio(2);
        const int coff = (int)(tl.s0 & 7);
        {
            const int64_t a0 = tl.s0 - coff, tail0 = total & ~(int64_t)7;
            if ((total & 7) && a0 + (int64_t)nch * 8 > tail0 && lane < (int)(total & 7))   /* last tile of the batch */
                ((int16_t *)slot)[tail0 - a0 + lane] = pcm[tail0 + lane];
        }
        const int Lt = tl.nb - tl.j0 < bt ? tl.nb - tl.j0 : bt;
        const uint32_t *tw = (const uint32_t *)slot;
        double res[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
        for (int n = 0; n < 2; ++n) {
            const int b = 32 * n + (lane & 31);
            const int hw0 = coff + (b < Lt ? b : 0) * ds + 16 * hf;      /* halfword index of k-group start */
            const uint32_t sh = (hw0 & 1) ? 16u : 0u;
            nm_i16 acc0 = s_init[hf], acc1 = s_init[2 + hf];
#ifdef BPMX_NM_NOMFMA                                         /* timing diagnostic: no matrix phase (wrong outputs) */
            acc0[0] += (int)tw[hw0 >> 1];
#else
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const uint32_t *p = tw + ((hw0 + 32 * s) >> 1);
                uint32_t w[9];
#pragma unroll
                for (int i = 0; i < 9; ++i) w[i] = p[i];
                nm_i4 bh, bl;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t e0 = __builtin_amdgcn_alignbit(w[2 * i + 1], w[2 * i], sh);
                    const uint32_t e1 = __builtin_amdgcn_alignbit(w[2 * i + 2], w[2 * i + 1], sh);
                    bh[i] = (int32_t)__builtin_amdgcn_perm(e1, e0, 0x07050301u);
                    bl[i] = (int32_t)(__builtin_amdgcn_perm(e1, e0, 0x06040200u) ^ 0x80808080u);
                }
                acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[0][s][0], bl, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[1][s][0], bl, acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[0][s][1], bh, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[1][s][1], bh, acc1, 0, 0, 0);
            }
#endif
            /* |acc| <= 2*160*128*128 + 128*147*128 < 2^23, so a row pair
             * a_r + 256 a_(r+1) fits int32; two pairs combine exactly in f64
             * (< 2^48), and H 2^32 + L is the one rounding. */
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int32_t p01 = acc0[4 * q] + acc0[4 * q + 1] * 256, p23 = acc0[4 * q + 2] + acc0[4 * q + 3] * 256;
                const int32_t p45 = acc1[4 * q] + acc1[4 * q + 1] * 256, p67 = acc1[4 * q + 2] + acc1[4 * q + 3] * 256;
                const double L = __builtin_fma((double)p23, 65536.0, (double)p01);
                const double H = __builtin_fma((double)p67, 65536.0, (double)p45);
                res[n][q] = __builtin_fma(H, 4294967296.0, L) * sc[q];
            }
        }
        const int j = tl.j0 + lane;
        const bool valid = lane < bt && j < tl.nb;
        const double x0 = valid ? (double)((const int16_t *)slot)[coff + lane * ds] : 0.0;
        /* the slot is read: refill it with the tile after next (two slots) or
         * the next one (one slot: it flies during this epilogue) */
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (tr < A.n_tiles) dma(tn.s0, slot);
        __builtin_amdgcn_s_setprio(0);
        /* lane half 0 holds even coefficients, half 1 odd ones; N tile n = blocks 32n.. */
        double cf[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const double other = __shfl_xor(hf ? res[0][q] : res[1][q], 32);
            cf[2 * q] = hf ? other : res[0][q];
            cf[2 * q + 1] = hf ? res[1][q] : other;
        }
#ifdef BPMX_NM_NOEPI                                          /* timing diagnostic: no epilogue (wrong outputs) */
        if (cf[0] == 1.2345e300 && cf[7] == x0) A.gam[0] = cf[3];
#else
        nat_tile_epilogue(A, s_et, tl, t, lane, valid, V4{cf[0], cf[1], cf[2], cf[3]}, V4{cf[4], cf[5], cf[6], cf[7]},
                          x0);
#endif
        if (NM_SLOTS == 1) tl = tn;
        else if (t + stride < A.n_tiles) tl = nat_tile_ld(A.tiles, t + stride);
    }
}
template __global__ void k_native_blocks_mfma<3>(NatBlockArgs, const nm_i4 *, const nm_i16 *, const double *);
template __global__ void k_native_blocks_mfma<5>(NatBlockArgs, const nm_i4 *, const nm_i16 *, const double *);

/* ---------------------------------------------------------------------- */

/* ---------------------------------------------------------------------- */
/* int16 mono beyond k_native_blocks_mfma's K <= 160, and int16 stereo: the
 * same exact integer GEMM with K = channels x (ds + 1) <= 640.
 *
 * Stereo enters the K dimension as it lies in memory (L0 R0 L1 R1 ...), each
 * coefficient digit duplicated for the two channels, so one accumulation
 * gives sum_i q_i (L_i + R_i) exactly; the channel mean (bpm_analysis.py:1016,
 * an exact f64 halving) is applied after the one rounding.  With K up to 640,
 * |acc| < 2^25, so the digit rows combine in f64 (exact below 2^53).
 *
 * The coefficient fragments stay in registers (4 M tiles x KS K steps), so a
 * workgroup is four waves, one per SIMD.  Each wave owns two LDS-DMA slots
 * (r03): a tile of bt <= 64 blocks arrives as sub-tiles of bs <= 16 blocks,
 * each into the slot the sub-tile before last used, so while the wave
 * multiplies one slot the other is in flight, and both fly during the tile's
 * epilogue.  (The r02 kernel had one 38 KB slot per wave and 32-block stereo
 * tiles: its DMA, matrix phase and epilogue added up — C5 7.1-7.4 ms against
 * 4.9 ms for the DMA alone; this one 6.5 ms.)  Eight 19 KB slots per CU hold
 * 16 stereo blocks each at ds = 300, so the product runs on
 * v_mfma_i32_16x16x64_i8 (N = 16 blocks, K steps of 64 samples): 4 M tiles
 * of 16 digit rows, lane l = block l & 15 and K group l >> 4 on B;
 * accumulator register i of M tile m in lane group g is digit row 4 (m & 1)
 * + i of coefficient 2 g + (m >> 1), so each lane ends with all digit rows of
 * two coefficients of its block.  A sub-tile's results move to the lanes of
 * its blocks (lane = block within the tile) by bpermutes, and the epilogue
 * runs once per 64 blocks with every lane busy.  Step s + 1's LDS words are
 * requested before step s's products issue (one wave per SIMD: nothing else
 * hides the LDS latency). */
constexpr int NB_WAVES = 4, NB_SLOTS = 2, NB_NDMA = 19;   /* waves, slots per wave, DMA instructions (KiB) per slot */
__host__ __device__ inline int nb_sub_blocks(int ds, int ch, int ks64, int ndma) {
    const int hw = ndma * 64 * 8;                    /* halfwords per slot */
    const int b = (hw - 7 - 64 * ks64 - 2) / (ds * ch) + 1;
    return b < 16 ? b : 16;                          /* one 16-column N tile per sub-tile */
}
template <int N>
__device__ __forceinline__ void nb_wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
/* wait until at most k sub-tiles' DMA (k * NDMA instructions) are outstanding */
template <int NDMA, int K>
__device__ __forceinline__ void nb_wait_subs(int k) {
    if constexpr (K == 0) nb_wait_vm<0>();
    else {
        if (k >= K) nb_wait_vm<K * NDMA>();
        else nb_wait_subs<NDMA, K - 1>(k);
    }
}

template <int KS, int NS, int NDMA, int NW>
__global__ __launch_bounds__(64 * NW, 1) void k_native_blocks_mfma_big(NatBlockArgs A, const nm_i4 *__restrict__ afrag,
                                                                     const nm_i4 *__restrict__ ainit,
                                                                     const double *__restrict__ cscale, int bs) {
    typedef nat_u4 u4;
    extern __shared__ __align__(16) unsigned char nb_smem[];
    __shared__ double s_et[ET_SIZE];
    __shared__ nm_i4 s_init[4][4];                      /* [M tile][lane group] */
    nat_stage_epilogue_tables(A, s_et);
    for (int i = threadIdx.x; i < 16; i += blockDim.x) s_init[i >> 2][i & 3] = ainit[i];
    const int lane = lane_id(), g4 = lane >> 4, wv = __builtin_amdgcn_readfirstlane(wave_id());
    const int16_t *pcm = (const int16_t *)A.pcm;
    const int64_t total = A.total;                        /* int16 elements */
    const int ds = A.ds, bt = A.bt, ch = A.channels, bstride = ds * ch;
    constexpr int SLOT_CH = NDMA * 64;
    u4 *const slots = (u4 *)nb_smem + NS * wv * SLOT_CH;
    const int nch = (7 + bs * bstride + ch + 7) >> 3;    /* chunks a sub-tile may touch (<= SLOT_CH) */
    nm_i4 af[4][KS];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int s = 0; s < KS; ++s) af[m][s] = afrag[(m * KS + s) * 64 + lane];
    const double sc0 = cscale[2 * g4] * (ch == 2 ? 0.5 : 1.0), sc1 = cscale[2 * g4 + 1] * (ch == 2 ? 0.5 : 1.0);   /* exact */
    __syncthreads();
    const int64_t clast = (total & ~(int64_t)7) - 8;
    /* exactly NDMA instructions per sub-tile, every lane on (the vmcnt
     * waits below count them); chunks past the sub-tile re-read the batch's
     * last whole chunk */
    auto dma = [&](int64_t e0, u4 *slot) {
        const int64_t a0 = e0 & ~(int64_t)7;
        int nchv = nch, lanev = lane;                     /* opaque: no hoisted lane masks (k_native_blocks_mfma) */
        asm volatile("" : "+s"(nchv), "+v"(lanev));
#pragma unroll
        for (int r = 0; r < NDMA; ++r) {
            const int q = r * 64 + lanev;
            int64_t c = a0 + (int64_t)q * 8;
            c = (q < nchv && c + 8 <= total) ? c : clast;
            const uint32_t m0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)(slot + r * 64);
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                         :: "v"(pcm + c), "s"(m0) : "memory");
        }
    };
    auto nsub_of = [&](const NatTile &h) {
        const int Lt = h.nb - h.j0 < bt ? h.nb - h.j0 : bt;
        return (Lt + bs - 1) / bs;
    };
    const int64_t stride = (int64_t)gridDim.x * NW, t0 = (int64_t)blockIdx.x * NW + wv;
    /* producer: the next sub-tile to fetch (tile pt, sub-tile pu) */
    int64_t pt = t0;
    int pu = 0;
    NatTile ptl{};
    if (pt < A.n_tiles) ptl = nat_tile_ld(A.tiles, pt);
    int64_t issued = 0;
    auto produce = [&](u4 *slot) {
        dma((ptl.s0 + (int64_t)pu * bs * ds) * ch, slot);
        ++issued;
        if (++pu >= nsub_of(ptl)) {
            pu = 0;
            pt += stride;
            if (pt < A.n_tiles) ptl = nat_tile_ld(A.tiles, pt);
        }
    };
#pragma unroll
    for (int k = 0; k < NS; ++k)
        if (pt < A.n_tiles) produce(slots + k * SLOT_CH);
    int64_t g = 0;                                        /* sub-tiles consumed */
    for (int64_t t = t0; t < A.n_tiles; t += stride) {
        const NatTile tl = nat_tile_ld(A.tiles, t);
        const int Lt = tl.nb - tl.j0 < bt ? tl.nb - tl.j0 : bt;
        const int ns = (Lt + bs - 1) / bs;
        double cf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        double x0 = 0.0;
        for (int u = 0; u < ns; ++u, ++g) {
            u4 *slot = slots + (int)(g % NS) * SLOT_CH;
            /* DMAs retire in issue order: with k later sub-tiles in flight,
             * <= k NDMA outstanding means this one landed (the epilogue's few
             * stores, issued later, only make it over-wait) */
            nb_wait_subs<NDMA, NS - 1>((int)(issued - g - 1));
            const int64_t e0 = (tl.s0 + (int64_t)u * bs * ds) * ch;
            const int coff = (int)(e0 & 7);
            {
                const int64_t a0 = e0 - coff, tail0 = total & ~(int64_t)7;
                if ((total & 7) && a0 + (int64_t)nch * 8 > tail0 && lane < (int)(total & 7))   /* batch's last chunk */
                    ((int16_t *)slot)[tail0 - a0 + lane] = pcm[tail0 + lane];
                __builtin_amdgcn_wave_barrier();
            }
            const int Ls = Lt - u * bs < bs ? Lt - u * bs : bs;
            const uint32_t *tw = (const uint32_t *)slot;
            double val0, val1;                            /* coefficients 2 g4, 2 g4 + 1 of block lane & 15 */
            {
                const int b = lane & 15;
                const int hw0 = coff + (b < Ls ? b : 0) * bstride + 16 * g4;
                const uint32_t sh = (hw0 & 1) ? 16u : 0u;
                nm_i4 l[4], h[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) { l[m] = s_init[m][g4]; h[m] = nm_i4{0, 0, 0, 0}; }
#ifndef BPMX_NB_SKIP_MFMA            /* diagnostic builds (tools/build_variant.sh): phase timing */
                const uint32_t *p = tw + (hw0 >> 1);
                uint32_t w[9];
#pragma unroll
                for (int i = 0; i < 9; ++i) w[i] = p[i];
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    nm_i4 bh, bl;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const uint32_t e0w = __builtin_amdgcn_alignbit(w[2 * i + 1], w[2 * i], sh);
                        const uint32_t e1w = __builtin_amdgcn_alignbit(w[2 * i + 2], w[2 * i + 1], sh);
                        bh[i] = (int32_t)__builtin_amdgcn_perm(e1w, e0w, 0x07050301u);
                        bl[i] = (int32_t)(__builtin_amdgcn_perm(e1w, e0w, 0x06040200u) ^ 0x80808080u);
                    }
                    if (s + 1 < KS) {
#pragma unroll
                        for (int i = 0; i < 9; ++i) w[i] = p[32 * (s + 1) + i];
                    }
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        l[m] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[m][s], bl, l[m], 0, 0, 0);
                        h[m] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[m][s], bh, h[m], 0, 0, 0);
                    }
                }
#else
                l[0][0] = (int)tw[hw0 >> 1];
#endif
                /* digit rows R_r = l_r + h_(r-1): coefficient 2 g4 + k has rows 0-3 in M tile 2k, 4-7 in 2k + 1 */
                double v2[2];
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const nm_i4 la = l[2 * k], lb = l[2 * k + 1], ha = h[2 * k], hb = h[2 * k + 1];
                    const double r0 = (double)la[0], r1 = (double)(la[1] + ha[0]);
                    const double r2 = (double)(la[2] + ha[1]), r3 = (double)(la[3] + ha[2]);
                    const double r4 = (double)(lb[0] + ha[3]), r5 = (double)(lb[1] + hb[0]);
                    const double r6 = (double)(lb[2] + hb[1]), r7 = (double)(lb[3] + hb[2]);
                    const double L = __builtin_fma(r3, 16777216.0, __builtin_fma(r2, 65536.0, __builtin_fma(r1, 256.0, r0)));
                    const double H = __builtin_fma(r7, 16777216.0, __builtin_fma(r6, 65536.0, __builtin_fma(r5, 256.0, r4)));
                    v2[k] = __builtin_fma(H, 4294967296.0, L);
                }
                val0 = v2[0] * sc0;
                val1 = v2[1] * sc1;
            }
            /* this sub-tile's blocks are tile lanes [u bs, u bs + Ls) */
            const int c = lane - u * bs;
            const bool mine = c >= 0 && c < Ls;
            if (mine) {
                const int16_t *fr = (const int16_t *)slot + coff + c * bstride;
                x0 = ch == 2 ? 0.5 * (double)((int)fr[0] + (int)fr[1]) : (double)fr[0];
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   /* the slot is read: refill it */
            if (pt < A.n_tiles) produce(slot);
            const int src = mine ? c : 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double e = __shfl(val0, src + 16 * q), o = __shfl(val1, src + 16 * q);
                if (mine) { cf[2 * q] = e; cf[2 * q + 1] = o; }
            }
        }
        const int j = tl.j0 + lane;
        const bool valid = lane < bt && j < tl.nb;
#ifndef BPMX_NB_SKIP_EPI
        nat_tile_epilogue(A, s_et, tl, t, lane, valid, V4{cf[0], cf[1], cf[2], cf[3]}, V4{cf[4], cf[5], cf[6], cf[7]},
                          x0);
#else
        if (valid && cf[0] == 12345.0) A.gam[0] = x0;
#endif
    }
}
template __global__ void k_native_blocks_mfma_big<5, NB_SLOTS, NB_NDMA, NB_WAVES>(NatBlockArgs, const nm_i4 *, const nm_i4 *,
                                                                                const double *, int);
template __global__ void k_native_blocks_mfma_big<10, NB_SLOTS, NB_NDMA, NB_WAVES>(NatBlockArgs, const nm_i4 *, const nm_i4 *,
                                                                                 const double *, int);

/* ---------------------------------------------------------------------- */
/* int16 interleaved PCM (stereo; also mono beyond the matrix-core path's
 * ds + 1 <= 160), f64 VALU block projections fed by LDS-DMA.
 *
 * At 96 kHz stereo a frame is 4 bytes and costs 8 f64 FMAs on the mean, so the
 * VALU work (~1.7 ms per 30 GB of PCM chip-wide) sits below the HBM time: the
 * kernel has to keep bytes in flight and the coefficients close.  Each wave
 * owns one LDS slot (four waves per workgroup, one workgroup per CU) and walks
 * the tile list: the slot is filled by global_load_lds_dwordx4 straight from
 * HBM (no registers), and the next tile's DMA is issued as soon as the slot
 * has been read, so it flies during this tile's epilogue and the other waves'
 * work.  The (ds + 1) x 8 coefficient table lives in LDS too: at ds = 300 it
 * is 19 KB, more than the scalar cache holds, and scalar loads that miss to L2
 * serialise the wave (measured: 36 ms for a 30 GB C5 shard).  Two lanes share
 * a block (lane b and b + 32: the first and second half of its frames), so a
 * wave-uniform coefficient read (ds_read_b128 broadcast, one address per lane
 * group) feeds up to 64 frame-block products; the halves are added with one
 * lane exchange before the tile epilogue.
 *
 * Channel mean: sum_i c_i (L_i + R_i) / 2 is accumulated as sum_i c_i (L_i + R_i)
 * and halved at the end — every partial sum differs by an exact factor of 2,
 * so this equals accumulating c_i * ((L_i + R_i) / 2), the f64 mean the
 * reference forms (bpm_analysis.py:1016). */
constexpr int ND_WAVES = 4;
constexpr int ND_LDS = 160 * 1024;

/* host: DMA wave-instructions per tile (1 KiB each) so that four slots, the
 * coefficient table and the epilogue constants fit the CU's LDS */
inline int nd_ndma(int ds) {
    const int coef = (ds + 1) * 64;
    const int n = (ND_LDS - coef - 1024) / (ND_WAVES * 1024);
    return n < 38 ? n : 38;
}
/* blocks per tile: the slot holds the <= 7-element alignment offset and
 * (bt ds + 1) frames of ch int16 elements; at most 32 (two lanes per block) */
inline int nd_tile_blocks(int ds, int ch) {
    const int n = nd_ndma(ds);
    if (n < 1) return 0;
    const int b = ((n * 64 * 8 - 7) / ch - 1) / ds;
    return b < 32 ? b : 32;
}
inline size_t nd_lds_bytes(int ds) { return (size_t)nd_ndma(ds) * ND_WAVES * 1024 + (size_t)(ds + 1) * 64 + ET_SIZE * 8; }

template <int CH>
__global__ __launch_bounds__(64 * ND_WAVES, 1) void k_native_blocks_dma(NatBlockArgs A, int ndma) {
    typedef nat_u4 u4;
    extern __shared__ __align__(16) unsigned char nd_smem[];
    const int ds = A.ds, bt = A.bt;
    const int slot_ch = ndma * 64;                        /* 16-byte chunks per slot */
    u4 *slots = (u4 *)nd_smem;
    double *s_coef = (double *)(slots + ND_WAVES * slot_ch);   /* [ds + 1][8] */
    double *s_et = s_coef + (ds + 1) * 8;
    nat_stage_epilogue_tables(A, s_et);
    {
        const double2 *src = (const double2 *)(A.tab + TB_COEF);
        double2 *dst = (double2 *)s_coef;
        for (int k = threadIdx.x; k < (ds + 1) * 4; k += blockDim.x) dst[k] = src[k];
    }
    const int lane = lane_id(), wv = __builtin_amdgcn_readfirstlane(wave_id());
    const int16_t *pcm = (const int16_t *)A.pcm;
    const int64_t total = A.total;                        /* int16 elements in the batch */
    const int nch = (7 + (bt * ds + 1) * CH + 7) >> 3;    /* chunks a tile may touch (<= slot_ch) */
    __syncthreads();                                      /* s_et, s_coef */
    const int64_t clast = (total & ~(int64_t)7) - 8;
    auto dma = [&](int64_t e0, u4 *slot) {
        const int64_t a0 = e0 & ~(int64_t)7;
        for (int r = 0; r < ndma; ++r) {
            const int q = r * 64 + lane;
            int64_t c = a0 + (int64_t)q * 8;
            c = (q < nch && c + 8 <= total) ? c : clast;
            const uint32_t m0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)(slot + r * 64);
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                         :: "v"(pcm + c), "s"(m0) : "memory");
        }
    };
    const int64_t stride = (int64_t)gridDim.x * ND_WAVES;
    int64_t t = (int64_t)blockIdx.x * ND_WAVES + wv;
    u4 *slot = slots + wv * slot_ch;
    const int blk = lane & 31, hf = lane >> 5;
    const int half = (ds + 2) >> 1;                       /* frames [0, half) | [half, ds] */
    const int i0 = hf ? half : 0, i1 = hf ? ds + 1 : half;
    NatTile tl{};
    if (t < A.n_tiles) {
        tl = nat_tile_ld(A.tiles, t);
        dma(tl.s0 * CH, slot);
    }
    for (; t < A.n_tiles; t += stride) {
        const int64_t tr = t + stride;
        NatTile tn{};
        if (tr < A.n_tiles) tn = nat_tile_ld(A.tiles, tr);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int64_t e0 = tl.s0 * CH;
        const int coff = (int)(e0 & 7);                    /* elements before the tile's first frame */
        {
            const int64_t a0 = e0 - coff, tail0 = total & ~(int64_t)7;
            if ((total & 7) && a0 + (int64_t)nch * 8 > tail0 && lane < (int)(total & 7))   /* last tile of the batch */
                ((int16_t *)slot)[tail0 - a0 + lane] = pcm[tail0 + lane];
            __builtin_amdgcn_wave_barrier();
        }
        const int Lt = tl.nb - tl.j0 < bt ? tl.nb - tl.j0 : bt;
        double u0 = 0, u1 = 0, u2 = 0, u3 = 0, v0 = 0, v1 = 0, v2 = 0, v3 = 0, x0 = 0;
        if (blk < Lt) {
            auto acc = [&](double xv, int i) {
                const double2 *c2 = (const double2 *)(s_coef + i * 8);
                const double2 ca = c2[0], cb = c2[1], cc = c2[2], cd = c2[3];
                u0 = __builtin_fma(ca.x, xv, u0); u1 = __builtin_fma(ca.y, xv, u1);
                u2 = __builtin_fma(cb.x, xv, u2); u3 = __builtin_fma(cb.y, xv, u3);
                v0 = __builtin_fma(cc.x, xv, v0); v1 = __builtin_fma(cc.y, xv, v1);
                v2 = __builtin_fma(cd.x, xv, v2); v3 = __builtin_fma(cd.y, xv, v3);
            };
            if constexpr (CH == 2) {
                const uint32_t *fr = (const uint32_t *)slot + (coff >> 1) + blk * ds;   /* one word per frame */
                auto sum = [](uint32_t w) { return (double)((int)(int16_t)(w & 0xFFFFu) + ((int)w >> 16)); };
                x0 = sum(fr[0]);
                int i = i0;
                for (; i + 4 <= i1; i += 4) {
                    const uint32_t w0 = fr[i], w1 = fr[i + 1], w2 = fr[i + 2], w3 = fr[i + 3];
                    acc(sum(w0), i); acc(sum(w1), i + 1); acc(sum(w2), i + 2); acc(sum(w3), i + 3);
                }
                for (; i < i1; ++i) acc(sum(fr[i]), i);
            } else {
                const int16_t *fr = (const int16_t *)slot + coff + blk * ds;
                x0 = (double)fr[0];
                int i = i0;
                for (; i + 4 <= i1; i += 4) {
                    const double a = fr[i], b = fr[i + 1], c = fr[i + 2], d = fr[i + 3];
                    acc(a, i); acc(b, i + 1); acc(c, i + 2); acc(d, i + 3);
                }
                for (; i < i1; ++i) acc((double)fr[i], i);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   /* the slot is read: refill it */
        if (tr < A.n_tiles) dma(tn.s0 * CH, slot);
        /* the second half's sums join the first (lane b += lane b + 32) */
        u0 += __shfl_xor(u0, 32); u1 += __shfl_xor(u1, 32); u2 += __shfl_xor(u2, 32); u3 += __shfl_xor(u3, 32);
        v0 += __shfl_xor(v0, 32); v1 += __shfl_xor(v1, 32); v2 += __shfl_xor(v2, 32); v3 += __shfl_xor(v3, 32);
        if (CH == 2) { u0 *= 0.5; u1 *= 0.5; u2 *= 0.5; u3 *= 0.5; v0 *= 0.5; v1 *= 0.5; v2 *= 0.5; v3 *= 0.5; x0 *= 0.5; }
        const bool valid = lane < Lt;
        nat_tile_epilogue(A, s_et, tl, t, lane, valid, V4{u0, u1, u2, u3}, V4{v0, v1, v2, v3}, x0);
        tl = tn;
    }
}
template __global__ void k_native_blocks_dma<1>(NatBlockArgs, int);
template __global__ void k_native_blocks_dma<2>(NatBlockArgs, int);

/* One wave per recording:
 *   head  15 padded samples, exact sosfilt steps -> S at block 0 (lane 0);
 *   tiles S0_(t+1) = M^T S0_t + incl_t (forward carries, stored per tile):
 *         a parallel affine scan — lane l composes its run of tiles into one
 *         map (P, a) (P a power of M^T: in modal coordinates two 2x2 rotation
 *         blocks = two complex numbers), Kogge-Stone over the lanes, then each
 *         lane replays its run from its carry-in;
 *   partial last tile: exact block recursion forward, then backward with
 *         its decimated outputs (lane 0);
 *   tail  [c_(nd-1), ne): exact forward then backward per-sample recursion
 *         -> Q at block nb and yd[nd-1] (lane 0);
 *   tiles Qe_t stored, Q_start = M^T Qe_t + R0_t + G0 S0_t (backward): the
 *         same scan mirrored (maps composed right to left, shuffles down). */
struct Cx2 { double a1, b1, a2, b2; };   /* diag([[a1, b1], [-b1, a1]], [[a2, b2], [-b2, a2]]) */
__device__ __forceinline__ Cx2 cx2_mul(const Cx2 &x, const Cx2 &y) {
    return Cx2{x.a1 * y.a1 - x.b1 * y.b1, x.a1 * y.b1 + x.b1 * y.a1, x.a2 * y.a2 - x.b2 * y.b2,
               x.a2 * y.b2 + x.b2 * y.a2};
}
__device__ __forceinline__ V4 cx2_mv(const Cx2 &r, const V4 &x) {
    return V4{r.a1 * x.a + r.b1 * x.b, -r.b1 * x.a + r.a1 * x.b, r.a2 * x.c + r.b2 * x.d, -r.b2 * x.c + r.a2 * x.d};
}
__device__ __forceinline__ Cx2 shfl_cx2(const Cx2 &x, int src) {
    return Cx2{__shfl(x.a1, src), __shfl(x.b1, src), __shfl(x.a2, src), __shfl(x.b2, src)};
}
__device__ __forceinline__ Cx2 shfl_up_cx2(const Cx2 &x, int d) {
    return Cx2{__shfl_up(x.a1, d), __shfl_up(x.b1, d), __shfl_up(x.a2, d), __shfl_up(x.b2, d)};
}
__device__ __forceinline__ Cx2 shfl_down_cx2(const Cx2 &x, int d) {
    return Cx2{__shfl_down(x.a1, d), __shfl_down(x.b1, d), __shfl_down(x.a2, d), __shfl_down(x.b2, d)};
}

constexpr int NAT_CPF = 8;      /* tiles per lane held in registers by k_native_carry */
__global__ __launch_bounds__(64) void k_native_carry(NatCarryArgs A, SosStep SS) {
    const int f = blockIdx.x;
    if (f >= A.n_files) return;
    if (A.io.flags && threadIdx.x == 0) init_out_one(A.io, f);   /* k_init_out's work for f */
    if (!A.active[f]) return;
    const int lane = threadIdx.x;
    const int64_t nd = A.doff[f + 1] - A.doff[f];
    const int64_t nb = nd - 1;
    const int ds = A.ds, bt = A.bt;
    const int64_t t0 = A.toff[f];
    const int64_t Tf = nb / bt;                             /* full tiles */
    /* what lane 0's sequential recursions read comes through LDS first: the
     * head's 16 samples, the tail's <= ds+1 samples (+16 for the mirror), the
     * partial tile's block records */
    __shared__ double s_head[16], s_tail[NAT_DSMAX + 20], s_ytl[NAT_DSMAX + 20], s_part[64 * NAT_PART];
    const int64_t n = A.foff[f + 1] - A.foff[f];
    const int64_t fb = A.foff[f];
    const int64_t base = (nd - 1) * ds;                     /* x index of c_{nd-1} */
    const int64_t ntl = n - base;                           /* real tail samples (<= ds + 1) */
    const int Lp = (int)(nb - Tf * bt);                     /* blocks in the partial tile */
    const int64_t tlo = n - 17 < base ? n - 17 : base;      /* mirror reads reach x[n-17] */
    for (int k = lane; k < 16; k += 64) s_head[k] = frame_value(A.pcm, A.dtype, A.channels, fb + k);
    for (int64_t k = lane; k < n - tlo; k += 64) s_tail[k] = frame_value(A.pcm, A.dtype, A.channels, fb + tlo + k);
    for (int k = lane; k < Lp * NAT_PART; k += 64) s_part[k] = A.part[(int64_t)f * 64 * NAT_PART + k];
    const int wdt = work_dtype(A.dtype, A.channels);
    const double *tb = A.tab, *tt = A.tt;
    const M4 Mm = nat_ld16(tb + TB_M), Pm = nat_ld16(tb + TB_P), G0 = nat_ld16(tt + TT_G0);
    const Cx2 MT{tt[TT_MT + 0], tt[TT_MT + 1], tt[TT_MT + 10], tt[TT_MT + 11]};   /* M^T, modal: rotation blocks */
    const V4 Cv = nat_ld4(tb + TB_C);
    const double Dd = tb[TB_D];
    const V4 zi = nat_ld4(tb + TB_ZI);
    const M4 Vm = nat_ld16(tb + TB_V), Vi = nat_ld16(tt + TT_VI);   /* modal <-> original state */
    const double *agg = A.agg + t0 * 8;
    double *car = A.carry + t0 * 8;
    double *yd = A.yd + A.doff[f];
    const Cx2 ID{1, 0, 1, 0};
    const V4 Z4{0, 0, 0, 0};
    /* this lane's run of tiles [tb0, te0) */
    const int64_t CH = (Tf + 63) / 64;
    const int64_t tb0 = min<int64_t>(Tf, (int64_t)lane * CH), te0 = min<int64_t>(Tf, tb0 + CH);

    /* head: 15 padded samples -> S at block 0 */
    V4 S{0, 0, 0, 0};
    __syncthreads();
    if (lane == 0) {
        const double x0 = s_head[0];
        const double e0 = odd_ext(wdt, x0, s_head[15]);
        V4 z{zi.a * e0, zi.b * e0, zi.c * e0, zi.d * e0};
        for (int k = 0; k < 15; ++k) (void)SS.step(z, odd_ext(wdt, x0, s_head[15 - k]));
        S = mv(Vi, z);                                      /* tables are modal */
    }
    S = V4{__shfl(S.a, 0), __shfl(S.b, 0), __shfl(S.c, 0), __shfl(S.d, 0)};

    /* forward tile carries: car[t][0..3] = S0_t; car[t][4..7] temporarily
     * holds b_t = R0_t + G0 S0_t for the backward scan (same lane, same run) */
    /* runs of at most NAT_CPF tiles (recordings up to ~108 s at 302 Hz) keep
     * their tile records in registers: every load issued before the compose,
     * and b_t stays in registers for the backward scan instead of a round trip
     * through car[t][4..7].  Longer runs go in chunks of NAT_CPF tiles with
     * the chunk's loads issued first (one memory latency per chunk, not per
     * tile) */
    const bool pf = CH <= NAT_CPF;                          /* wave-uniform */
    V4 ag[NAT_CPF], ar[NAT_CPF], bbr[NAT_CPF];
    {
        Cx2 P = ID;
        V4 acc = Z4;
        if (pf) {
#pragma unroll
            for (int u = 0; u < NAT_CPF; ++u) {
                if (tb0 + u < te0) {
                    ag[u] = nat_ld4(agg + (tb0 + u) * 8);
                    ar[u] = nat_ld4(agg + (tb0 + u) * 8 + 4);
                }
            }
#pragma unroll
            for (int u = 0; u < NAT_CPF; ++u) {
                if (tb0 + u < te0) {
                    acc = add4(cx2_mv(MT, acc), ag[u]);
                    P = cx2_mul(MT, P);
                }
            }
        } else {                                            /* long runs: chunks of NAT_CPF, loads first */
            for (int64_t c0 = tb0; c0 < te0; c0 += NAT_CPF) {
                V4 g[NAT_CPF];
#pragma unroll
                for (int u = 0; u < NAT_CPF; ++u)
                    if (c0 + u < te0) g[u] = nat_ld4(agg + (c0 + u) * 8);
#pragma unroll
                for (int u = 0; u < NAT_CPF; ++u) {
                    if (c0 + u < te0) {
                        acc = add4(cx2_mv(MT, acc), g[u]);
                        P = cx2_mul(MT, P);
                    }
                }
            }
        }
        /* inclusive Kogge-Stone over lanes: x_l <- x_l o x_(l-d) */
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int d = 1 << k;
            const Cx2 Pe = shfl_up_cx2(P, d);
            const V4 ae = shfl_up_v(acc, d);
            if (lane >= d) {
                acc = add4(cx2_mv(P, ae), acc);
                P = cx2_mul(P, Pe);
            }
        }
        Cx2 Px = shfl_up_cx2(P, 1);
        V4 ax = shfl_up_v(acc, 1);
        if (lane == 0) { Px = ID; ax = Z4; }
        V4 s = add4(cx2_mv(Px, S), ax);                     /* carry into this lane's run */
        if (pf) {
#pragma unroll
            for (int u = 0; u < NAT_CPF; ++u) {
                if (tb0 + u < te0) {
                    bbr[u] = add4(ar[u], mv(G0, s));
                    double *cw = car + (tb0 + u) * 8;
                    cw[0] = s.a; cw[1] = s.b; cw[2] = s.c; cw[3] = s.d;
                    s = add4(cx2_mv(MT, s), ag[u]);
                }
            }
        } else {
            for (int64_t c0 = tb0; c0 < te0; c0 += NAT_CPF) {
                V4 inc[NAT_CPF], r0[NAT_CPF];
#pragma unroll
                for (int u = 0; u < NAT_CPF; ++u) {
                    if (c0 + u < te0) {
                        inc[u] = nat_ld4(agg + (c0 + u) * 8);
                        r0[u] = nat_ld4(agg + (c0 + u) * 8 + 4);
                    }
                }
#pragma unroll
                for (int u = 0; u < NAT_CPF; ++u) {
                    if (c0 + u < te0) {
                        const V4 bb = add4(r0[u], mv(G0, s));
                        double *cw = car + (c0 + u) * 8;
                        cw[0] = s.a; cw[1] = s.b; cw[2] = s.c; cw[3] = s.d;
                        cw[4] = bb.a; cw[5] = bb.b; cw[6] = bb.c; cw[7] = bb.d;
                        s = add4(cx2_mv(MT, s), inc[u]);
                    }
                }
            }
        }
        /* S after the last full tile: the run holding tile Tf-1 */
        if (Tf > 0) {
            const int owner = (int)((Tf - 1) / CH);
            S = V4{__shfl(s.a, owner), __shfl(s.b, owner), __shfl(s.c, owner), __shfl(s.d, owner)};
        }
    }
    /* partial tile forward, tail, partial tile backward */
    V4 q{0, 0, 0, 0};
    /* the partial tile's block recursions, S_(b+1) = M S_b + u_b forward and
     * q_b = M q_(b+1) + P S_b + v_b backward, as lane scans (lane b = block b,
     * Lp <= 63; M in modal coordinates is two rotation blocks) */
    const Cx2 M1{Mm.m[0], Mm.m[1], Mm.m[10], Mm.m[11]};
    double *pp = s_part;
    {
        Cx2 P = lane < Lp ? M1 : ID;
        V4 acc = lane < Lp ? V4{pp[lane * NAT_PART + 0], pp[lane * NAT_PART + 1], pp[lane * NAT_PART + 2],
                                pp[lane * NAT_PART + 3]}
                           : Z4;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int d = 1 << k;
            const Cx2 Pe = shfl_up_cx2(P, d);
            const V4 ae = shfl_up_v(acc, d);
            if (lane >= d) {
                acc = add4(cx2_mv(P, ae), acc);
                P = cx2_mul(P, Pe);
            }
        }
        const V4 Sn = add4(cx2_mv(P, S), acc);                  /* S_(b+1) */
        V4 Sb = shfl_up_v(Sn, 1);
        if (lane == 0) Sb = S;
        if (lane < Lp) {
            double *r = pp + lane * NAT_PART;
            r[12] = Sb.a; r[13] = Sb.b; r[14] = Sb.c; r[15] = Sb.d;
        }
        if (Lp > 0) S = V4{__shfl(Sn.a, Lp - 1), __shfl(Sn.b, Lp - 1), __shfl(Sn.c, Lp - 1), __shfl(Sn.d, Lp - 1)};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    auto xt = [&](int64_t k) { return s_tail[k - tlo]; };   /* k in [tlo, n) */
    const int64_t nt = ntl + 15;                            /* tail length incl. right pad */
    const double xl = xt(n - 1);
    auto tin = [&](int64_t k) {                             /* tail input k: the samples, then the odd extension */
        const int64_t xi = base + k;
        return xi < n ? xt(xi) : odd_ext(wdt, xl, xt(n - 2 - (xi - n)));
    };
    if (A.ttab && nt <= NAT_TT_PAR) {
        /* lane-parallel: y_k = C A^k z0 + sum_(m <= k) h_m u_(k-m), then the
         * backward pass's final state q = A^(nt-1) zi y_(nt-1) +
         * sum_(k >= 1) A^(k-1) B y_k as a wave sum (agrees with the serial
         * recursion to rounding; that took half of this kernel on lane 0) */
        const V4 z0 = mv(Vm, S);
        for (int64_t k = lane; k < nt; k += 64) {
            const double *tr = A.ttab + k * 16;
            double y = dot4(V4{tr[0], tr[1], tr[2], tr[3]}, z0);
            for (int64_t m = 0; m <= k; ++m) y = __builtin_fma(A.ttab[m * 16 + 12], tin(k - m), y);
            s_ytl[k] = y;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const double y0 = s_ytl[nt - 1];
        V4 acc{0, 0, 0, 0};
        for (int64_t k = 1 + lane; k < nt; k += 64) {
            const double *tr = A.ttab + (k - 1) * 16 + 4;
            const double yk = s_ytl[k];
            acc = V4{__builtin_fma(tr[0], yk, acc.a), __builtin_fma(tr[1], yk, acc.b), __builtin_fma(tr[2], yk, acc.c),
                     __builtin_fma(tr[3], yk, acc.d)};
        }
        for (int o = 32; o > 0; o >>= 1)
            acc = V4{acc.a + __shfl_xor(acc.a, o), acc.b + __shfl_xor(acc.b, o), acc.c + __shfl_xor(acc.c, o),
                     acc.d + __shfl_xor(acc.d, o)};
        const double *tz = A.ttab + (nt - 1) * 16 + 8;
        q = V4{__builtin_fma(tz[0], y0, acc.a), __builtin_fma(tz[1], y0, acc.b), __builtin_fma(tz[2], y0, acc.c),
               __builtin_fma(tz[3], y0, acc.d)};
    } else if (lane == 0) {
        V4 z = mv(Vm, S);                                   /* the exact recursion runs in the original basis */
#ifdef NAT_DIAG_NOSOS
        for (int64_t k = 0; k < nt; ++k) s_ytl[k] = 0.0;    /* diagnostic: the tail recursion's share (wrong yd) */
        if (false)
#endif
        for (int64_t k = 0; k < nt; ++k) s_ytl[k] = SS.step(z, tin(k));
        const double y0 = s_ytl[nt - 1];
        q = V4{zi.a * y0, zi.b * y0, zi.c * y0, zi.d * y0};
#ifndef NAT_DIAG_NOSOS
        for (int64_t k = nt - 1; k >= 1; --k) (void)SS.step(q, s_ytl[k]);
#endif
    }
    q = V4{__shfl(q.a, 0), __shfl(q.b, 0), __shfl(q.c, 0), __shfl(q.d, 0)};
    q = mv(Vi, q);
    if (lane == 0) yd[nd - 1] = dot4(Cv, q) + Dd * s_ytl[0];
    {
        V4 Sj{0, 0, 0, 0}, w{0, 0, 0, 0};
        double xj = 0.0;
        if (lane < Lp) {
            const double *r = pp + lane * NAT_PART;
            Sj = V4{r[12], r[13], r[14], r[15]};
            w = add4(mv(Pm, Sj), V4{r[4], r[5], r[6], r[7]});
            xj = r[8];
        }
        Cx2 P = lane < Lp ? M1 : ID;
        V4 acc = w;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int d = 1 << k;
            const Cx2 Pe = shfl_down_cx2(P, d);
            const V4 ae = shfl_down_v(acc, d);
            if (lane + d < 64) {
                acc = add4(cx2_mv(P, ae), acc);
                P = cx2_mul(P, Pe);
            }
        }
        const V4 qb = add4(cx2_mv(P, q), acc);                  /* q_b */
        if (lane < Lp) yd[Tf * bt + lane] = dot4(Cv, qb) + Dd * (dot4(Cv, Sj) + Dd * xj);
        q = V4{__shfl(qb.a, 0), __shfl(qb.b, 0), __shfl(qb.c, 0), __shfl(qb.d, 0)};
    }
    /* backward tile carries: car[t][4..7] = Qe_t; Qe_(t-1) = M^T Qe_t + b_t.
     * Lane l's run maps the Qe entering its last tile to the Qe leaving its
     * first: (P, a) composed right to left; the scan runs from lane 63 down. */
    {
        Cx2 P = ID;
        V4 acc = Z4;
        if (pf) {
#pragma unroll
            for (int u = NAT_CPF - 1; u >= 0; --u) {
                if (tb0 + u < te0) {
                    acc = add4(cx2_mv(MT, acc), bbr[u]);
                    P = cx2_mul(MT, P);
                }
            }
        } else {
            for (int64_t c1 = te0 - 1; c1 >= tb0; c1 -= NAT_CPF) {   /* tiles c1, c1 - 1, ... */
                V4 g[NAT_CPF];
#pragma unroll
                for (int u = 0; u < NAT_CPF; ++u)
                    if (c1 - u >= tb0) g[u] = nat_ld4(car + (c1 - u) * 8 + 4);
#pragma unroll
                for (int u = 0; u < NAT_CPF; ++u) {
                    if (c1 - u >= tb0) {
                        acc = add4(cx2_mv(MT, acc), g[u]);
                        P = cx2_mul(MT, P);
                    }
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int d = 1 << k;
            const Cx2 Pe = shfl_down_cx2(P, d);
            const V4 ae = shfl_down_v(acc, d);
            if (lane + d < 64) {
                acc = add4(cx2_mv(P, ae), acc);
                P = cx2_mul(P, Pe);
            }
        }
        Cx2 Px = shfl_down_cx2(P, 1);
        V4 ax = shfl_down_v(acc, 1);
        if (lane == 63) { Px = ID; ax = Z4; }
        V4 qq = add4(cx2_mv(Px, q), ax);                    /* Qe entering this lane's last tile */
        if (pf) {
#pragma unroll
            for (int u = NAT_CPF - 1; u >= 0; --u) {
                if (tb0 + u < te0) {
                    double *cw = car + (tb0 + u) * 8;
                    cw[4] = qq.a; cw[5] = qq.b; cw[6] = qq.c; cw[7] = qq.d;
                    qq = add4(cx2_mv(MT, qq), bbr[u]);
                }
            }
        } else {
            for (int64_t c1 = te0 - 1; c1 >= tb0; c1 -= NAT_CPF) {
                V4 g[NAT_CPF];
#pragma unroll
                for (int u = 0; u < NAT_CPF; ++u)                  /* the chunk's b_t, read before it is overwritten */
                    if (c1 - u >= tb0) g[u] = nat_ld4(car + (c1 - u) * 8 + 4);
#pragma unroll
                for (int u = 0; u < NAT_CPF; ++u) {
                    if (c1 - u >= tb0) {
                        double *cw = car + (c1 - u) * 8;
                        cw[4] = qq.a; cw[5] = qq.b; cw[6] = qq.c; cw[7] = qq.d;
                        qq = add4(cx2_mv(MT, qq), g[u]);
                    }
                }
            }
        }
    }
}

/* yd_j = alpha_b . Qe_t + beta_b . S0_t + gamma_j over full tiles (lane = block) */
__global__ __launch_bounds__(64) void k_native_yd(NatYdArgs A) {
    const int64_t t = blockIdx.x;
    const NatTile tl = nat_tile_ld(A.tiles, t);
    const int bt = A.bt, lane = threadIdx.x;
    if (tl.nb - tl.j0 < bt || lane >= bt) return;          /* partial tiles: k_native_carry */
    if (A.skip && A.skip[tl.f]) return;                    /* uniform: yd made by k_hilbert_env */
    const double *c = A.carry + t * 8;
    const V4 S0 = nat_ld4(c), Qe = nat_ld4(c + 4);
    const V4 al = nat_ld4(A.tt + TT_ALPHA + 4 * lane), be = nat_ld4(A.tt + TT_BETA + 4 * lane);
    /* gamma is read once: a non-temporal load (r05 A/B: 0.095 -> 0.084 ms) */
    A.yd[tl.ybase + lane] = dot4(al, Qe) + dot4(be, S0) + __builtin_nontemporal_load(A.gam + tl.gbase + lane);
}

/* ---------------------------------------------------------------------- */
/* Hilbert transform on the R2C half spectrum: W_k = -i Y_k for 0 < k < N/2,
 * W_0 = W_(N/2) = 0.  A C2R of W gives N * Im(analytic signal): scipy's
 * hilbert (ifft(fft(x) * h), h = 1, 2, ..., 2, [1], 0, ...) has imaginary part
 * (2/N) Re sum_(0<k<N/2) (-i X_k) e^(2 pi i k n / N), and X_0, X_(N/2) are real. */
__global__ __launch_bounds__(256) void k_hilbert_rotate(double2 *z, const int64_t *doff, const int32_t *active,
                                                        int f_begin, int f_end) {
    const int f = f_begin + blockIdx.y;
    if (f >= f_end || !active[f]) return;
    const int64_t n = doff[f + 1] - doff[f];
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k > n / 2) return;
    double2 *zf = z + doff[f];
    const double2 c = zf[k];
    zf[k] = (k == 0 || 2 * k == n) ? make_double2(0.0, 0.0) : make_double2(c.y, -c.x);
}

/* |z| = sqrt(y^2 + (h/N)^2) (h: unnormalised C2R output) and the centred
 * rolling mean (window w, min_periods 1), LDS-tiled */
constexpr int NE_T = 256;
__global__ __launch_bounds__(NE_T) void k_native_env(NatEnvArgs A) {
    __shared__ double mag[NE_T + 2 * 1024];
    const int f = blockIdx.y;
    if (f >= A.n_files || !A.active[f] || A.skip[f]) return;
    const int64_t n = A.doff[f + 1] - A.doff[f];
    const int64_t i0 = (int64_t)blockIdx.x * NE_T;
    if (i0 >= n) return;
    const int64_t w = A.window, off = (w - 1) / 2;
    const int64_t lo = i0 + 1 + off - w < 0 ? 0 : i0 + 1 + off - w;
    const int64_t hiE = i0 + NE_T + off < n ? i0 + NE_T + off : n;   /* exclusive */
    const double *y = A.y + A.doff[f], *h = A.h + A.doff[f];
    const double inv = 1.0 / (double)n;
    for (int64_t p = lo + threadIdx.x; p < hiE; p += NE_T) {
        const double re = y[p], im = h[p] * inv;
        mag[p - lo] = sqrt(re * re + im * im);
    }
    __syncthreads();
    const int64_t i = i0 + threadIdx.x;
    if (i >= n) return;
    int64_t s, e;
    win_bounds(i, n, w, s, e);
    double sum = 0.0;
    for (int64_t p = s; p < e; ++p) sum += mag[p - lo];
    A.env[A.doff[f] + i] = sum / (double)(e - s);
}

/* ---------------------------------------------------------------------- */
namespace {
struct FftPlans {
    rocfft_plan fwd = nullptr, inv = nullptr;
    size_t work = 0;
};
/* process-wide, shared by contexts on any thread: find/insert under g_plans_mu
 * (nodes are never erased, so returned pointers stay valid) */
std::map<std::tuple<int, int64_t, int64_t>, FftPlans> g_plans;   /* (device, nd, batch) */
std::mutex g_plans_mu;

int fft_fail(const char *what, rocfft_status st) {
    return fail(BPMX_E_HIP, std::string(what) + " failed (rocfft status " + std::to_string((int)st) + ")");
}

}  // namespace

int rocfft_setup_once() {
    static std::once_flag once;
    static rocfft_status st = rocfft_status_success;
    std::call_once(once, [] { st = rocfft_setup(); });
    return st == rocfft_status_success ? BPMX_OK : fft_fail("rocfft_setup", st);
}

namespace {
int get_plans(int dev, int64_t nd, int64_t batch, FftPlans **out) {
    if (const int rc = rocfft_setup_once(); rc != BPMX_OK) return rc;
    auto key = std::make_tuple(dev, nd, batch);
    std::lock_guard<std::mutex> g(g_plans_mu);
    auto it = g_plans.find(key);
    if (it != g_plans.end()) { *out = &it->second; return BPMX_OK; }
    FftPlans p;
    const size_t len = (size_t)nd;
    rocfft_plan_description d1 = nullptr, d2 = nullptr;
    rocfft_status st;
    if ((st = rocfft_plan_description_create(&d1)) != rocfft_status_success) return fft_fail("plan_description", st);
    /* real input distance nd, complex output distance nd (room for the full spectrum) */
    st = rocfft_plan_description_set_data_layout(d1, rocfft_array_type_real, rocfft_array_type_hermitian_interleaved,
                                                 nullptr, nullptr, 1, nullptr, len, 1, nullptr, len);
    if (st != rocfft_status_success) return fft_fail("set_data_layout(r2c)", st);
    st = rocfft_plan_create(&p.fwd, rocfft_placement_notinplace, rocfft_transform_type_real_forward,
                            rocfft_precision_double, 1, &len, (size_t)batch, d1);
    if (st != rocfft_status_success) return fft_fail("plan_create(r2c)", st);
    if ((st = rocfft_plan_description_create(&d2)) != rocfft_status_success) return fft_fail("plan_description", st);
    st = rocfft_plan_description_set_data_layout(d2, rocfft_array_type_hermitian_interleaved,
                                                 rocfft_array_type_real, nullptr, nullptr, 1, nullptr, len, 1,
                                                 nullptr, len);
    if (st != rocfft_status_success) return fft_fail("set_data_layout(c2r)", st);
    st = rocfft_plan_create(&p.inv, rocfft_placement_notinplace, rocfft_transform_type_real_inverse,
                            rocfft_precision_double, 1, &len, (size_t)batch, d2);
    if (st != rocfft_status_success) return fft_fail("plan_create(c2r)", st);
    rocfft_plan_description_destroy(d1);
    rocfft_plan_description_destroy(d2);
    size_t w1 = 0, w2 = 0;
    rocfft_plan_get_work_buffer_size(p.fwd, &w1);
    rocfft_plan_get_work_buffer_size(p.inv, &w2);
    p.work = std::max(w1, w2);
    auto res = g_plans.emplace(key, p);
    *out = &res.first->second;
    return BPMX_OK;
}
}  // namespace

/* ---------------------------------------------------------------------- */
/* host: block-state tables (native_tables.py restated in C++, long double) */
namespace {
typedef long double LD;
struct LM { LD m[16]; };
LM lm_mul(const LM &X, const LM &Y) {
    LM R;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            LD acc = 0;
            for (int k = 0; k < 4; ++k) acc += X.m[i * 4 + k] * Y.m[k * 4 + j];
            R.m[i * 4 + j] = acc;
        }
    return R;
}
void lm_vec(const LM &X, const LD *v, LD *out) {
    for (int i = 0; i < 4; ++i) {
        LD acc = 0;
        for (int k = 0; k < 4; ++k) acc += X.m[i * 4 + k] * v[k];
        out[i] = acc;
    }
}

/* real basis of the two conjugate eigenvector pairs of A: V, V^-1.  False
 * when A has a real eigenvalue (then M' would not be two rotation blocks). */
bool modal_basis(const LM &A, LM *V, LM *Vi) {
    typedef std::complex<LD> CX;
    /* eigenvalues: A is block lower-triangular, its diagonal blocks are the
     * sections' companion forms [[-a1, 1], [-a2, 0]] */
    CX lam[2];
    for (int b = 0; b < 2; ++b) {
        const LD a1 = -A.m[(2 * b) * 4 + 2 * b], a2 = -A.m[(2 * b + 1) * 4 + 2 * b];
        const LD disc = a1 * a1 - 4 * a2;
        if (disc >= 0) return false;
        lam[b] = CX(-a1 / 2, sqrtl(-disc) / 2);
    }
    for (int b = 0; b < 2; ++b) {
        /* null vector of (A - lam I) by Gaussian elimination with partial pivoting */
        CX M[4][4];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) M[i][j] = CX(A.m[i * 4 + j], 0) - (i == j ? lam[b] : CX(0, 0));
        int piv_col[4], rank = 0;
        bool is_piv[4] = {false, false, false, false};
        for (int c = 0; c < 4 && rank < 4; ++c) {
            int best = -1;
            LD bv = 0;
            for (int r = rank; r < 4; ++r)
                if (std::abs(M[r][c]) > bv) { bv = std::abs(M[r][c]); best = r; }
            if (best < 0 || bv < 1e-14L) continue;
            for (int j = 0; j < 4; ++j) std::swap(M[rank][j], M[best][j]);
            for (int r = 0; r < 4; ++r) {
                if (r == rank) continue;
                const CX fct = M[r][c] / M[rank][c];
                for (int j = 0; j < 4; ++j) M[r][j] -= fct * M[rank][j];
            }
            piv_col[rank++] = c;
            is_piv[c] = true;
        }
        if (rank != 3) return false;
        int fr = 0;
        while (is_piv[fr]) ++fr;
        CX v[4];
        v[fr] = CX(1, 0);
        for (int r = 0; r < rank; ++r) v[piv_col[r]] = -M[r][fr] / M[r][piv_col[r]];
        /* A (vr + i vi) = lam (vr + i vi): in the basis [vr, vi] the block is
         * [[Re, Im], [-Im, Re]] (column convention, see build_tables) */
        for (int i = 0; i < 4; ++i) {
            V->m[i * 4 + 2 * b] = v[i].real();
            V->m[i * 4 + 2 * b + 1] = v[i].imag();
        }
    }
    /* V^-1 by Gauss-Jordan */
    LD W[4][8];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) W[i][j] = j < 4 ? V->m[i * 4 + j] : (j - 4 == i ? 1 : 0);
    for (int c = 0; c < 4; ++c) {
        int best = c;
        for (int r = c + 1; r < 4; ++r)
            if (fabsl(W[r][c]) > fabsl(W[best][c])) best = r;
        if (fabsl(W[best][c]) < 1e-30L) return false;
        for (int j = 0; j < 8; ++j) std::swap(W[c][j], W[best][j]);
        const LD d = W[c][c];
        for (int j = 0; j < 8; ++j) W[c][j] /= d;
        for (int r = 0; r < 4; ++r) {
            if (r == c) continue;
            const LD fct = W[r][c];
            for (int j = 0; j < 8; ++j) W[r][j] -= fct * W[c][j];
        }
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) Vi->m[i * 4 + j] = W[i][4 + j];
    return true;
}

std::vector<double> build_tables(const double *sos, const double *sos_zi, int L, int T, std::vector<LD> *coefld) {
    /* probe the cascade step: s' = A s + B u, y = C s + D u */
    auto step = [&](const LD *z, LD u, LD *zo) -> LD {
        const LD *a = nullptr; (void)a;
        LD x1 = (LD)sos[0] * u + z[0];
        zo[0] = (LD)sos[1] * u - (LD)sos[4] * x1 + z[1];
        zo[1] = (LD)sos[2] * u - (LD)sos[5] * x1;
        LD y = (LD)sos[6] * x1 + z[2];
        zo[2] = (LD)sos[7] * x1 - (LD)sos[10] * y + z[3];
        zo[3] = (LD)sos[8] * x1 - (LD)sos[11] * y;
        return y;
    };
    LM A;
    LD Bv[4], Cv[4], D;
    for (int k = 0; k < 4; ++k) {
        LD e[4] = {0, 0, 0, 0}, zo[4];
        e[k] = 1;
        Cv[k] = step(e, 0, zo);
        for (int i = 0; i < 4; ++i) A.m[i * 4 + k] = zo[i];
    }
    {
        LD e[4] = {0, 0, 0, 0};
        D = step(e, 1, Bv);
    }
    /* modal coordinates: V = [Re v1, Im v1, Re v2, Im v2] from one eigenvector
     * of each conjugate pole pair, so V^-1 A V = diag(R(l1), R(l2)) with
     * R(l) = [[Re l, Im l], [-Im l, Re l]].  The blocks are then set to that
     * exact form (the off-block residue of the long-double transform is
     * ~1e-19 relative and is dropped), B' = V^-1 B, C' = C V. */
    LM V{}, Vi{};
    const bool modal = modal_basis(A, &V, &Vi);
    if (modal) {
        const LM Am = lm_mul(Vi, lm_mul(A, V));
        LM R{};
        for (int b = 0; b < 2; ++b) {
            const int o = 2 * b;
            const LD re = (Am.m[o * 4 + o] + Am.m[(o + 1) * 4 + o + 1]) / 2;
            const LD im = (Am.m[o * 4 + o + 1] - Am.m[(o + 1) * 4 + o]) / 2;
            R.m[o * 4 + o] = re; R.m[o * 4 + o + 1] = im;
            R.m[(o + 1) * 4 + o] = -im; R.m[(o + 1) * 4 + o + 1] = re;
        }
        A = R;
        LD b2[4], c2[4];
        lm_vec(Vi, Bv, b2);
        for (int c = 0; c < 4; ++c) {
            LD acc = 0;
            for (int k = 0; k < 4; ++k) acc += Cv[k] * V.m[k * 4 + c];
            c2[c] = acc;
        }
        for (int k = 0; k < 4; ++k) { Bv[k] = b2[k]; Cv[k] = c2[k]; }
    } else {                                  /* real poles: stay in the original basis */
        for (int i = 0; i < 16; ++i) V.m[i] = Vi.m[i] = (i % 5 == 0) ? 1 : 0;
    }
    std::vector<LM> pw(L + 2);
    for (int i = 0; i < 16; ++i) pw[0].m[i] = (i % 5 == 0) ? 1 : 0;
    for (int i = 1; i <= L + 1; ++i) pw[i] = lm_mul(A, pw[i - 1]);
    std::vector<LD> AB((size_t)(L + 1) * 4), h(L + 1);
    for (int i = 0; i <= L; ++i) {
        lm_vec(pw[i], Bv, &AB[(size_t)i * 4]);
        LD acc = 0;
        for (int k = 0; k < 4; ++k) acc += Cv[k] * AB[(size_t)i * 4 + k];
        h[i] = acc;                                                     /* C A^i B */
    }
    LM P;
    for (int i = 0; i < 16; ++i) P.m[i] = 0;
    for (int i = 1; i <= L; ++i) {
        LD CA[4];
        for (int c = 0; c < 4; ++c) {
            LD acc = 0;
            for (int k = 0; k < 4; ++k) acc += Cv[k] * pw[i].m[k * 4 + c];
            CA[c] = acc;
        }
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) P.m[r * 4 + c] += AB[(size_t)(i - 1) * 4 + r] * CA[c];
    }
    std::vector<double> out(64 + 8 * (size_t)(L + 1) + TT_SIZE, 0.0);
    for (int i = 0; i < 16; ++i) out[TB_V + i] = (double)V.m[i];
    for (int i = 0; i < 4; ++i) { out[TB_B + i] = (double)Bv[i]; out[TB_C + i] = (double)Cv[i]; }
    out[TB_D] = (double)D;
    for (int i = 0; i < 16; ++i) { out[TB_M + i] = (double)pw[L].m[i]; out[TB_P + i] = (double)P.m[i]; }
    for (int i = 0; i < 4; ++i) out[TB_ZI + i] = sos_zi[i];
    for (int ip = 0; ip <= L; ++ip) {
        double *c = &out[TB_COEF + (size_t)ip * 8];
        if (ip < L) {
            LD F[4];
            lm_vec(pw[L - 1 - ip], Bv, F);
            for (int k = 0; k < 4; ++k) c[k] = (double)F[k];
        }
        LD g[4] = {0, 0, 0, 0};
        if (ip >= 1)
            for (int k = 0; k < 4; ++k) g[k] = AB[(size_t)(ip - 1) * 4 + k] * D;
        for (int i = ip + 1; i <= L; ++i)
            for (int k = 0; k < 4; ++k) g[k] += AB[(size_t)(i - 1) * 4 + k] * h[i - 1 - ip];
        for (int k = 0; k < 4; ++k) c[4 + k] = (double)g[k];
        if (coefld) {
            LD *cl = &(*coefld)[(size_t)ip * 8];
            if (ip < L) lm_vec(pw[L - 1 - ip], Bv, cl);
            else cl[0] = cl[1] = cl[2] = cl[3] = 0;
            for (int k = 0; k < 4; ++k) cl[4 + k] = g[k];
        }
    }
    /* tile tables (native_tables.tile_tables): M^(2^k), M^T, G_0, alpha_b, beta_b */
    {
        const LM &M = pw[L];
        std::vector<LM> Mp(T + 1);
        for (int i = 0; i < 16; ++i) Mp[0].m[i] = (i % 5 == 0) ? 1 : 0;
        for (int b = 1; b <= T; ++b) Mp[b] = lm_mul(M, Mp[b - 1]);
        std::vector<LM> G(T + 1);
        for (int i = 0; i < 16; ++i) G[T].m[i] = 0;
        for (int b = T - 1; b >= 0; --b) {                      /* G_b = P M^b + M G_{b+1} */
            const LM a = lm_mul(P, Mp[b]), c = lm_mul(M, G[b + 1]);
            for (int i = 0; i < 16; ++i) G[b].m[i] = a.m[i] + c.m[i];
        }
        auto rowC = [&](const LM &X, LD *r) {                   /* r = C X */
            for (int c2 = 0; c2 < 4; ++c2) {
                LD acc = 0;
                for (int k = 0; k < 4; ++k) acc += Cv[k] * X.m[k * 4 + c2];
                r[c2] = acc;
            }
        };
        double *tt = &out[TB_COEF + 8 * (size_t)(L + 1)];
        LM K = M;
        for (int k = 0; k < 6; ++k) {             /* rotation form (a1, b1, a2, b2); M' is block diagonal */
            tt[TT_KPOW + 4 * k + 0] = (double)K.m[0];
            tt[TT_KPOW + 4 * k + 1] = (double)K.m[1];
            tt[TT_KPOW + 4 * k + 2] = (double)K.m[10];
            tt[TT_KPOW + 4 * k + 3] = (double)K.m[11];
            K = lm_mul(K, K);
        }
        for (int i = 0; i < 16; ++i) tt[TT_VI + i] = (double)Vi.m[i];
        for (int i = 0; i < 16; ++i) { tt[TT_MT + i] = (double)Mp[T].m[i]; tt[TT_G0 + i] = (double)G[0].m[i]; }
        for (int b = 0; b < T; ++b) {
            LD al[4], cg[4], cm[4];
            rowC(Mp[T - b], al);
            rowC(G[b], cg);
            rowC(Mp[b], cm);
            for (int k = 0; k < 4; ++k) {
                tt[TT_ALPHA + 4 * b + k] = (double)al[k];
                tt[TT_BETA + 4 * b + k] = (double)(cg[k] + D * cm[k]);
            }
        }
    }
    return out;
}

/* int8-MFMA tables for k_native_blocks_mfma (layout in 32-bit words):
 *   [0, 16)                 scale_c = 2^(e_c - P), 8 doubles
 *   [16, 16 + 2*64*16)      initial accumulators [M tile][lane][16]: 128 * sum_k d_r(k, c)
 *   then                    A fragments [M tile][K step][variant][lane][4 words]
 * from the long-double coefficients (R = ds + 1 rows x 8). */
constexpr int NM_P = 54, NM_D = 7;
std::vector<int32_t> build_mfma(const std::vector<LD> &cl, int R, int KS) {
    std::vector<int64_t> q((size_t)R * 8);
    std::vector<double> scale(8);
    for (int c = 0; c < 8; ++c) {
        LD mx = 0;
        for (int i = 0; i < R; ++i) mx = std::max(mx, fabsl(cl[(size_t)i * 8 + c]));
        int e = 0;
        if (mx > 0) frexpl(mx, &e);                          /* mx < 2^e */
        scale[c] = ldexp(1.0, e - NM_P);
        for (int i = 0; i < R; ++i) q[(size_t)i * 8 + c] = llroundl(ldexpl(cl[(size_t)i * 8 + c], NM_P - e));
    }
    /* balanced base-256 digits, d[(k * 8 + c) * 8 + r], r < NM_D (row 7 stays 0) */
    std::vector<int8_t> d((size_t)R * 64, 0);
    for (int i = 0; i < R * 8; ++i) {
        int64_t v = q[i];
        for (int r = 0; r < NM_D; ++r) {
            int dg = (int)(v & 255);
            if (dg >= 128) dg -= 256;
            d[(size_t)i * 8 + r] = (int8_t)dg;
            v = (v - dg) >> 8;
        }
    }
    auto dig = [&](int k, int c, int r) -> int { return (k < R && r >= 0 && r < 8) ? d[((size_t)k * 8 + c) * 8 + r] : 0; };
    std::vector<int32_t> w(16 + 2 * 64 * 16 + (size_t)2 * KS * 2 * 64 * 4, 0);
    std::memcpy(w.data(), scale.data(), 64);
    int32_t *init = w.data() + 16;
    for (int t = 0; t < 2; ++t)
        for (int l = 0; l < 64; ++l)
            for (int reg = 0; reg < 16; ++reg) {
                const int c = 2 * (reg >> 2) + (l >> 5), r = 4 * t + (reg & 3);
                int64_t sum = 0;
                for (int k = 0; k < R; ++k) sum += dig(k, c, r);
                init[(t * 64 + l) * 16 + reg] = (int32_t)(128 * sum);
            }
    int32_t *af = init + 2 * 64 * 16;
    for (int t = 0; t < 2; ++t)
        for (int st = 0; st < KS; ++st)
            for (int v = 0; v < 2; ++v)
                for (int l = 0; l < 64; ++l) {
                    const int rho = l & 31;
                    const int c = 2 * (rho >> 3) + ((rho >> 2) & 1), r = 4 * t + (rho & 3) - v;
                    for (int j = 0; j < 16; ++j) {
                        const int k = 32 * st + 16 * (l >> 5) + j;
                        const uint32_t byte = (uint8_t)(int8_t)dig(k, c, r);
                        af[(((t * KS + st) * 2 + v) * 64 + l) * 4 + j / 4] |= (int32_t)(byte << (8 * (j & 3)));
                    }
                }
    return w;
}

/* tables for k_native_blocks_mfma_big (v_mfma_i32_16x16x64_i8), the digits of build_mfma
 * with K = CH x R, each coefficient repeated for the CH interleaved channels:
 *   [0, 16) scale | [16, 80) initial accumulators [M tile m][lane group g][4]
 *   | A fragments [m][K step][lane][4 words]
 * M tile m, row rho = 4 g + i: coefficient 2 g + (m >> 1), digit row 4 (m & 1) + i;
 * lane l of a fragment: row l & 15, K = 64 step + 16 (l >> 4) + byte. */
std::vector<int32_t> build_mfma_big(const std::vector<LD> &cl, int R, int KS, int CH) {
    std::vector<int64_t> q((size_t)R * 8);
    std::vector<double> scale(8);
    for (int c = 0; c < 8; ++c) {
        LD mx = 0;
        for (int i = 0; i < R; ++i) mx = std::max(mx, fabsl(cl[(size_t)i * 8 + c]));
        int e = 0;
        if (mx > 0) frexpl(mx, &e);
        scale[c] = ldexp(1.0, e - NM_P);
        for (int i = 0; i < R; ++i) q[(size_t)i * 8 + c] = llroundl(ldexpl(cl[(size_t)i * 8 + c], NM_P - e));
    }
    std::vector<int8_t> d((size_t)R * 64, 0);
    for (int i = 0; i < R * 8; ++i) {
        int64_t v = q[i];
        for (int r = 0; r < NM_D; ++r) {
            int dg = (int)(v & 255);
            if (dg >= 128) dg -= 256;
            d[(size_t)i * 8 + r] = (int8_t)dg;
            v = (v - dg) >> 8;
        }
    }
    const int K = R * CH;
    auto dig = [&](int k, int c, int r) -> int {
        return (k < K && r >= 0 && r < 8) ? d[((size_t)(k / CH) * 8 + c) * 8 + r] : 0;
    };
    std::vector<int32_t> w(16 + 64 + (size_t)4 * KS * 64 * 4, 0);
    std::memcpy(w.data(), scale.data(), 64);
    int32_t *init = w.data() + 16;
    for (int m = 0; m < 4; ++m)
        for (int g = 0; g < 4; ++g)
            for (int i = 0; i < 4; ++i) {
                const int c = 2 * g + (m >> 1), r = 4 * (m & 1) + i;
                int64_t sum = 0;
                for (int k = 0; k < K; ++k) sum += dig(k, c, r);
                init[(m * 4 + g) * 4 + i] = (int32_t)(128 * sum);
            }
    int32_t *af = init + 64;
    for (int m = 0; m < 4; ++m)
        for (int st = 0; st < KS; ++st)
            for (int l = 0; l < 64; ++l) {
                const int rho = l & 15;
                const int c = 2 * (rho >> 2) + (m >> 1), r = 4 * (m & 1) + (rho & 3);
                for (int j = 0; j < 16; ++j) {
                    const int k = 64 * st + 16 * (l >> 4) + j;
                    const uint32_t byte = (uint8_t)(int8_t)dig(k, c, r);
                    af[((m * KS + st) * 64 + l) * 4 + j / 4] |= (int32_t)(byte << (8 * (j & 3)));
                }
            }
    return w;
}
}  // namespace

/* fused-Hilbert plans and their device tables, cached per (device, Nd, window) */
struct HbTables {
    HilbPlan plan;
    size_t lds = 0;
    double2 *dev = nullptr;
};
std::map<std::tuple<int, int64_t, int>, HbTables> g_hb;   /* under g_hb_mu, never erased */
std::mutex g_hb_mu;

HbTables *hb_tables(bpmx_ctx *ctx, int64_t nd, int window, HilbPlan *P, size_t *lds, hipStream_t s, int *rc) {
    const auto key = std::make_tuple(ctx->device, nd, window);
    std::lock_guard<std::mutex> g(g_hb_mu);
    auto it = g_hb.find(key);
    if (it == g_hb.end()) {
        HbTables t;
        std::vector<double2> tabs;
        if (!hilbert_plan(nd, window, &t.plan, &tabs, &t.lds)) {
            t.dev = nullptr;                                   /* remembered: not supported */
        } else {
            if (hipMalloc((void **)&t.dev, tabs.size() * sizeof(double2)) != hipSuccess) {
                *rc = fail(BPMX_E_HIP, "hipMalloc (Hilbert tables) failed");
                return nullptr;
            }
            /* synchronous: the host vector dies here, and this happens once per Nd */
            if (hipMemcpy(t.dev, tabs.data(), tabs.size() * sizeof(double2), hipMemcpyHostToDevice) != hipSuccess) {
                *rc = fail(BPMX_E_HIP, "hipMemcpy (Hilbert tables) failed");
                return nullptr;
            }
        }
        it = g_hb.emplace(key, t).first;
    }
    (void)s;
    if (!it->second.dev) return nullptr;
    *P = it->second.plan;
    *lds = it->second.lds;
    return &it->second;
}

int native_envelope(bpmx_ctx *ctx, const bpmx_params *P, const bpmx_batch *B, const bpmx_out *O, hipStream_t s,
                    int F, const std::vector<int64_t> &foff, const std::vector<int64_t> &doff, int64_t maxnd,
                    const int64_t *d_foff, const int64_t *d_doff, const int32_t *d_active, const QuantArgs *qa,
                    const InitOutArgs *io) {
    const int ds = P->ds;
    if (ds > NAT_DSMAX) return fail(BPMX_E_LIMIT, "native mode supports ds <= " + std::to_string(NAT_DSMAX));
    int rc = BPMX_OK;
    /* tables (cached on the host key; uploaded when they change) */
    /* tables and block offsets: rebuilt / re-uploaded only when they change (the
     * host copies live in the context, so the async upload never outlives them) */
    /* tiles of bt blocks: the int16 path's LDS tile holds <= NB_RCH*512 samples */
    /* matrix-core path: int16 mono, ds + 1 <= 160 (KS K steps of 32 samples) */
    const int mfma_ks = ds + 1 <= 96 ? 3 : (ds + 1 <= 160 ? 5 : 0);
    const bool aligned16 = ((uintptr_t)B->pcm & 15) == 0;
    const bool i16_fast = P->dtype == BPMX_DT_I16 && aligned16 && foff[F] * P->channels >= 16 &&
                          !(P->options & (BPMX_OPT_NATIVE_F64 | BPMX_OPT_NATIVE_DMA));
    const bool use_mfma = mfma_ks && i16_fast && P->channels == 1;
    /* int16 mono beyond K = 160 and int16 stereo: the big-K matrix-core kernel
     * (K = channels x (ds + 1) <= 640, K steps of 64) */
    const int kbig = P->channels * (ds + 1);
    const int big_ks = kbig <= 320 ? 5 : (kbig <= 640 ? 10 : 0);
    const int big_bs = big_ks ? nb_sub_blocks(ds, P->channels, big_ks, NB_NDMA) : 0;
    const bool use_big = !use_mfma && i16_fast && big_ks && (P->channels == 1 || P->channels == 2) && big_bs >= 1;
    /* the rest of int16 stereo (and, on request, mono) through the LDS-DMA f64 kernel */
    const bool use_dma = !use_mfma && !use_big && P->dtype == BPMX_DT_I16 && aligned16 && foff[F] * P->channels >= 16 &&
                         (P->channels == 2 || (P->channels == 1 && (P->options & BPMX_OPT_NATIVE_DMA))) &&
                         !(P->options & BPMX_OPT_NATIVE_F64) && nd_tile_blocks(ds, P->channels) >= 1;
    /* tiles of bt blocks: the LDS tile (slot) must hold the tile's samples */
    const int bt = use_mfma ? nm_tile_blocks(ds, mfma_ks)
                 : use_big  ? big_bs * (64 / big_bs)
                 : (use_dma ? nd_tile_blocks(ds, P->channels) : std::min(64, (NB_RCH * 512 - 16) / ds));
    std::vector<int64_t> key(17);
    for (int i = 0; i < 12; ++i) std::memcpy(&key[i], &P->sos[i], 8);
    key[12] = ds;
    std::memcpy(&key[13], &P->sos_zi[0], 8);
    std::memcpy(&key[14], &P->sos_zi[2], 8);
    key[15] = bt;
    key[16] = use_big ? 1000 * P->channels + big_ks : 0;
    size_t mfma_off = 0;                                     /* in doubles, into nat_tab */
    if (key != ctx->nat_key) {
        std::vector<LD> cl((size_t)(ds + 1) * 8);
        ctx->nat_tab = build_tables(P->sos, P->sos_zi, ds, bt, &cl);
        if (use_big) {
            const std::vector<int32_t> w = build_mfma_big(cl, ds + 1, big_ks, P->channels);
            const size_t o = ctx->nat_tab.size();
            ctx->nat_tab.resize(o + w.size() / 2);
            std::memcpy(ctx->nat_tab.data() + o, w.data(), w.size() * 4);
        } else if (mfma_ks) {
            const std::vector<int32_t> w = build_mfma(cl, ds + 1, mfma_ks);
            const size_t o = ctx->nat_tab.size();
            ctx->nat_tab.resize(o + w.size() / 2);
            std::memcpy(ctx->nat_tab.data() + o, w.data(), w.size() * 4);
        }
        ctx->nat_key = key;
        ctx->nat_tab_dirty = true;
    }
    bool grew = false;
    double *d_tab = (double *)ctx->buf("nat_tab", ctx->nat_tab.size() * 8, &rc, &grew);
    if (grew) ctx->nat_tab_dirty = true;
    if (rc != BPMX_OK) return rc;
    if (ctx->nat_tab_dirty) {
        HIP_TRY(hipMemcpyAsync(d_tab, ctx->nat_tab.data(), ctx->nat_tab.size() * 8, hipMemcpyHostToDevice, s));
        ctx->nat_tab_dirty = false;
    }
    const double *d_tt = d_tab + TB_COEF + 8 * (size_t)(ds + 1);
    mfma_off = TB_COEF + 8 * (size_t)(ds + 1) + TT_SIZE;
    /* geometry: block offsets, per-file tile offsets, the tile list (cached with the context) */
    const int64_t gstr = (bt + 15) / 16 * 16;                 /* gamma row per tile */
    std::vector<int64_t> tk(4 + 2 * (F + 1));
    tk[0] = bt; tk[1] = F; tk[2] = ds; tk[3] = 0;
    for (int f = 0; f <= F; ++f) { tk[4 + f] = foff[f]; tk[5 + F + f] = doff[f]; }
    if (tk != ctx->nat_tkey) {
        std::vector<int64_t> geo(2 * (F + 1), 0);             /* boff | toff */
        std::vector<NatTile> tv;
        for (int f = 0; f < F; ++f) {
            const int64_t nd = doff[f + 1] - doff[f];
            const int64_t nb = nd > 1 ? nd - 1 : 0;
            geo[f + 1] = geo[f] + nb;
            geo[F + 1 + f] = (int64_t)tv.size();
            if (nd <= 15) continue;                          /* inactive (filtfilt would raise) */
            /* gamma: one 128-byte aligned row of gstr doubles per tile, so
             * k_native_blocks writes and k_native_yd reads whole cache lines */
            for (int64_t j0 = 0; j0 < nb; j0 += bt)
                tv.push_back(NatTile{foff[f] + j0 * ds, (int64_t)tv.size() * gstr, doff[f] + j0, (int32_t)j0,
                                     (int32_t)nb, f, 0});
        }
        geo[2 * F + 1] = (int64_t)tv.size();
        ctx->nat_boff = geo;
        ctx->nat_tiles.resize(tv.size() * sizeof(NatTile));
        if (!tv.empty()) std::memcpy(ctx->nat_tiles.data(), tv.data(), ctx->nat_tiles.size());
        ctx->nat_tkey = tk;
        ctx->nat_tiles_dirty = true;
    }
    const int64_t nt = (int64_t)(ctx->nat_tiles.size() / sizeof(NatTile));
    int64_t *d_geo = (int64_t *)ctx->buf("nat_geo", (size_t)(F + 1) * 16, &rc, &grew);
    if (grew) ctx->nat_tiles_dirty = true;
    NatTile *d_tiles = (NatTile *)ctx->buf("nat_tiles", std::max<size_t>(ctx->nat_tiles.size(), 64), &rc, &grew);
    if (grew) ctx->nat_tiles_dirty = true;
    if (rc != BPMX_OK) return rc;
    if (ctx->nat_tiles_dirty) {
        HIP_TRY(hipMemcpyAsync(d_geo, ctx->nat_boff.data(), (size_t)(F + 1) * 16, hipMemcpyHostToDevice, s));
        if (nt > 0)
            HIP_TRY(hipMemcpyAsync(d_tiles, ctx->nat_tiles.data(), ctx->nat_tiles.size(), hipMemcpyHostToDevice, s));
        ctx->nat_tiles_dirty = false;
    }
    double *gam = (double *)ctx->buf("nat_gam", (size_t)std::max<int64_t>(nt * gstr, 1) * 8, &rc);
    double *agg = (double *)ctx->buf("nat_agg", (size_t)std::max<int64_t>(nt, 1) * 64, &rc);
    double *carry = (double *)ctx->buf("nat_carry", (size_t)std::max<int64_t>(nt, 1) * 64, &rc);
    double *part = (double *)ctx->buf("nat_part", (size_t)F * 64 * NAT_PART * 8, &rc);
    double *yd = O->y ? O->y : (double *)ctx->buf("nat_yd", (size_t)doff[F] * 8, &rc);
    double2 *z = (double2 *)ctx->buf("nat_z", (size_t)doff[F] * 16, &rc);
    double *hb = (double *)ctx->buf("nat_h", (size_t)doff[F] * 8, &rc);
    if (rc != BPMX_OK) return rc;
    if (nt > 0) {
        NatBlockArgs a;
        a.pcm = B->pcm; a.tiles = d_tiles; a.n_tiles = nt; a.total = foff[F]; a.bt = bt;
        a.channels = P->channels; a.ds = ds; a.tab = d_tab; a.tt = d_tt; a.gam = gam; a.agg = agg; a.part = part;
        const bool fast = P->dtype == BPMX_DT_I16 && P->channels == 1 && ((uintptr_t)B->pcm & 15) == 0;
        const unsigned grid = (unsigned)std::min<int64_t>(nt, 256 * 8);
        if (use_mfma) {
            const double *mt = d_tab + mfma_off;
            const nm_i16 *init = (const nm_i16 *)(mt + 8);
            const nm_i4 *af = (const nm_i4 *)(mt + 8 + 2 * 64 * 16 / 2);
            /* persistent: one 4-wave workgroup per CU (LDS-bound) */
            unsigned g1 = (unsigned)std::min<int64_t>((nt + NM_WAVES - 1) / NM_WAVES, 256 * (2 / NM_SLOTS));
            if (const char *gv = std::getenv("BPMX_NM_GRID"))    /* diagnostic: fewer persistent workgroups */
                g1 = std::max(1u, std::min(g1, (unsigned)std::atoi(gv)));
            if (mfma_ks == 3)
                LAUNCH(ctx, s, "k_native_blocks", k_native_blocks_mfma<3>, dim3(g1), dim3(64 * NM_WAVES), 0, s, a, af,
                       init, mt);
            else
                LAUNCH(ctx, s, "k_native_blocks", k_native_blocks_mfma<5>, dim3(g1), dim3(64 * NM_WAVES), 0, s, a, af,
                       init, mt);
        } else if (use_big) {
            a.total = foff[F] * P->channels;                 /* int16 elements */
            const double *mt = d_tab + mfma_off;
            const nm_i4 *init = (const nm_i4 *)(mt + 8), *af = (const nm_i4 *)(mt + 8 + 32);
            const unsigned g1 = (unsigned)std::min<int64_t>((nt + NB_WAVES - 1) / NB_WAVES, 256);
            const size_t lds = (size_t)NB_SLOTS * NB_NDMA * NB_WAVES * 1024;
            if (big_ks == 5) {
                (void)hipFuncSetAttribute((const void *)k_native_blocks_mfma_big<5, NB_SLOTS, NB_NDMA, NB_WAVES>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                LAUNCH(ctx, s, "k_native_blocks", (k_native_blocks_mfma_big<5, NB_SLOTS, NB_NDMA, NB_WAVES>), dim3(g1),
                       dim3(64 * NB_WAVES), lds, s, a, af, init, mt, big_bs);
            } else {
                (void)hipFuncSetAttribute((const void *)k_native_blocks_mfma_big<10, NB_SLOTS, NB_NDMA, NB_WAVES>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                LAUNCH(ctx, s, "k_native_blocks", (k_native_blocks_mfma_big<10, NB_SLOTS, NB_NDMA, NB_WAVES>), dim3(g1),
                       dim3(64 * NB_WAVES), lds, s, a, af, init, mt, big_bs);
            }
        } else if (use_dma) {
            a.total = foff[F] * P->channels;                 /* int16 elements */
            const unsigned g1 = (unsigned)std::min<int64_t>((nt + ND_WAVES - 1) / ND_WAVES, 256);
            const int ndma = nd_ndma(ds);
            const size_t lds = nd_lds_bytes(ds);
            if (P->channels == 2) {
                (void)hipFuncSetAttribute((const void *)k_native_blocks_dma<2>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                LAUNCH(ctx, s, "k_native_blocks", k_native_blocks_dma<2>, dim3(g1), dim3(64 * ND_WAVES), lds, s, a, ndma);
            } else {
                (void)hipFuncSetAttribute((const void *)k_native_blocks_dma<1>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                LAUNCH(ctx, s, "k_native_blocks", k_native_blocks_dma<1>, dim3(g1), dim3(64 * ND_WAVES), lds, s, a, ndma);
            }
        } else if (fast) {
            LAUNCH(ctx, s, "k_native_blocks", k_native_blocks_i16, dim3(grid), dim3(64), 0, s, a,
                   (const double *)(d_tab + TB_COEF));
        } else {
#define NAT_GEN(DT)                                                                                        \
    if (P->channels > 1) LAUNCH(ctx, s, "k_native_blocks", (k_native_blocks_gen<DT, true>), dim3((unsigned)nt), \
                                dim3(64), 0, s, a);                                                          \
    else LAUNCH(ctx, s, "k_native_blocks", (k_native_blocks_gen<DT, false>), dim3((unsigned)nt), dim3(64), 0, s, a);
            switch (P->dtype) {
            case BPMX_DT_U8: NAT_GEN(BPMX_DT_U8) break;
            case BPMX_DT_I16: NAT_GEN(BPMX_DT_I16) break;
            case BPMX_DT_I32: NAT_GEN(BPMX_DT_I32) break;
            case BPMX_DT_F32: NAT_GEN(BPMX_DT_F32) break;
            default: NAT_GEN(BPMX_DT_F64) break;
            }
#undef NAT_GEN
        }
    }
    {
        NatCarryArgs a;
        a.pcm = B->pcm; a.foff = d_foff; a.doff = d_doff; a.boff = d_geo; a.toff = d_geo + F + 1;
        a.active = d_active; a.n_files = F; a.dtype = P->dtype; a.channels = P->channels; a.ds = ds; a.bt = bt;
        a.tab = d_tab; a.tt = d_tt; a.agg = agg; a.part = part; a.carry = carry; a.yd = yd;
        if (io) a.io = *io;
        else a.io = InitOutArgs{};
        SosStep ss;
        for (int i = 0; i < 12; ++i) ss.s[i] = P->sos[i];
        /* the tail tables (rebuilt when the coefficients change): row m holds
         * C A^m, A^m B, A^m zi and h_m of SosStep's recursion, in long double */
        std::vector<double> key2(P->sos, P->sos + 12);
        key2.insert(key2.end(), ctx->nat_tab.begin() + TB_ZI, ctx->nat_tab.begin() + TB_ZI + 4);
        if (key2 != ctx->nat_tkey2) {
            typedef long double LD;
            LD c[12];
            for (int i = 0; i < 12; ++i) c[i] = (LD)P->sos[i];
            auto step = [&](LD z[4], LD u) -> LD {                /* SosStep::step */
                const LD x1 = c[0] * u + z[0];
                const LD z00 = c[1] * u - c[4] * x1 + z[1];
                const LD z01 = c[2] * u - c[5] * x1;
                const LD y = c[6] * x1 + z[2];
                const LD z10 = c[7] * x1 - c[10] * y + z[3];
                const LD z11 = c[8] * x1 - c[11] * y;
                z[0] = z00; z[1] = z01; z[2] = z10; z[3] = z11;
                return y;
            };
            LD Am[4][4], Bv[4], Cv[4], Dv;
            for (int i = 0; i < 4; ++i) {
                LD z[4] = {0, 0, 0, 0};
                z[i] = 1;
                Cv[i] = step(z, 0);
                for (int r = 0; r < 4; ++r) Am[r][i] = z[r];
            }
            {
                LD z[4] = {0, 0, 0, 0};
                Dv = step(z, 1);
                for (int r = 0; r < 4; ++r) Bv[r] = z[r];
            }
            LD ca[4], g[4], az[4];
            for (int i = 0; i < 4; ++i) { ca[i] = Cv[i]; g[i] = Bv[i]; az[i] = (LD)ctx->nat_tab[TB_ZI + i]; }
            std::vector<double> &tt2 = ctx->nat_ttab;
            tt2.assign((size_t)NAT_TT_ROWS * 16, 0.0);
            LD hprev = Dv;
            for (int m = 0; m < NAT_TT_ROWS; ++m) {
                double *row = tt2.data() + (size_t)m * 16;
                for (int i = 0; i < 4; ++i) { row[i] = (double)ca[i]; row[4 + i] = (double)g[i]; row[8 + i] = (double)az[i]; }
                row[12] = (double)hprev;                     /* h_m: D, then C A^(m-1) B */
                LD hn = 0;
                for (int i = 0; i < 4; ++i) hn += ca[i] * Bv[i];
                hprev = hn;
                LD ca2[4], g2[4], az2[4];
                for (int j = 0; j < 4; ++j) {
                    ca2[j] = 0; g2[j] = 0; az2[j] = 0;
                    for (int i = 0; i < 4; ++i) { ca2[j] += ca[i] * Am[i][j]; g2[j] += Am[j][i] * g[i]; az2[j] += Am[j][i] * az[i]; }
                }
                for (int j = 0; j < 4; ++j) { ca[j] = ca2[j]; g[j] = g2[j]; az[j] = az2[j]; }
            }
            ctx->nat_tkey2 = key2;
            ctx->nat_ttab_dirty = true;
        }
        bool grew2 = false;
        double *d_tt2 = (double *)ctx->buf("nat_ttab", (size_t)NAT_TT_ROWS * 16 * 8, &rc, &grew2);
        if (rc != BPMX_OK) return rc;
        if (grew2) ctx->nat_ttab_dirty = true;
        if (ctx->nat_ttab_dirty) {
            HIP_TRY(hipMemcpyAsync(d_tt2, ctx->nat_ttab.data(), ctx->nat_ttab.size() * 8, hipMemcpyHostToDevice, s));
            ctx->nat_ttab_dirty = false;
        }
        /* BPMX_CARRY_SERIAL (A/B diagnostic: the serial tail recursion) is read
         * once per process, not on every run's launch path */
        static const bool carry_serial = std::getenv("BPMX_CARRY_SERIAL") != nullptr;
        a.ttab = carry_serial ? nullptr : d_tt2;
        LAUNCH(ctx, s, "k_native_carry", k_native_carry, dim3(F), dim3(64), 0, s, a, ss);
    }
    /* k_hilbert_env makes yd of the full tiles itself (HilbArgs::fy) for every
     * run of recordings it takes, when the tiles hold an even number of blocks
     * and yd is not an output; k_native_yd then covers only the other
     * recordings' tiles (a skip list), and is not launched when none is left */
    static const bool no_fy = std::getenv("BPMX_NO_FY") != nullptr;   /* A/B diagnostic, read once */
    const bool fy_ok = !O->y && bt % 2 == 0 && bt <= 64 && !(P->options & BPMX_OPT_HILBERT_ROCFFT) && !no_fy;
    std::vector<int32_t> &fyrec = ctx->nat_fyrec;
    fyrec.assign(F, 0);
    bool any_fy = false, all_fy = true;
    for (int f0 = 0; f0 < F;) {
        const int64_t nd = doff[f0 + 1] - doff[f0];
        int f1 = f0 + 1;
        while (f1 < F && doff[f1 + 1] - doff[f1] == nd) ++f1;
        if (nd > 15) {
            HilbPlan hp;
            size_t hlds = 0;
            const bool plan = fy_ok && hb_tables(ctx, nd, P->env_window, &hp, &hlds, s, &rc) != nullptr;
            if (rc != BPMX_OK) return rc;
            for (int f = f0; f < f1; ++f) fyrec[f] = plan ? 1 : 0;
            any_fy |= plan;
            all_fy &= plan;
        }
        f0 = f1;
    }
    double *ys = any_fy ? (double *)ctx->buf("nat_ys", (size_t)(doff[F] + 32 * (int64_t)F + 16) * 8, &rc) : nullptr;
    int32_t *d_fyrec = any_fy ? (int32_t *)ctx->buf("nat_fyrec", (size_t)F * 4, &rc) : nullptr;
    if (rc != BPMX_OK) return rc;
    if (any_fy && !all_fy) HIP_TRY(hipMemcpyAsync(d_fyrec, fyrec.data(), (size_t)F * 4, hipMemcpyHostToDevice, s));
    if (nt > 0 && !all_fy) {
        NatYdArgs a;
        a.tiles = d_tiles; a.skip = any_fy ? d_fyrec : nullptr; a.bt = bt; a.tt = d_tt; a.carry = carry; a.gam = gam;
        a.yd = yd;
        LAUNCH(ctx, s, "k_native_yd", k_native_yd, dim3((unsigned)nt), dim3(64), 0, s, a);
    }
    /* Hilbert + envelope: runs of equal Nd share a plan.  The fused LDS kernel
     * (k_hilbert.hip) takes every run whose Nd factors into small primes and
     * fits; the rest go through rocFFT + k_hilbert_rotate + k_native_env. */
    if (P->env_window > 2 * 1024) return fail(BPMX_E_LIMIT, "envelope window too large for k_native_env");
    bool need_env = false;
    std::vector<int32_t> &fused = ctx->nat_fused;
    fused.assign(F, 0);
    bool side_used[bpmx_ctx::NSIDE] = {};
    bool forked = false;
    std::vector<int32_t> blu;
    int f0 = 0;
    while (f0 < F) {
        const int64_t nd = doff[f0 + 1] - doff[f0];
        int f1 = f0 + 1;
        while (f1 < F && doff[f1 + 1] - doff[f1] == nd) ++f1;
        HilbPlan hp;
        size_t hlds = 0;
        HbTables *ht = nullptr;
        if (nd > 15 && !(P->options & BPMX_OPT_HILBERT_ROCFFT) &&
            (ht = hb_tables(ctx, nd, P->env_window, &hp, &hlds, s, &rc)) != nullptr) {
            if (rc != BPMX_OK) return rc;
            {                                                    /* any decimated offset (k_hilbert_env's loads) */
                HilbArgs a;
                a.yd = yd; a.doff = d_doff; a.active = d_active; a.f_begin = f0; a.f_end = f1;
                a.tabs = ht->dev; a.env = O->env; a.stamps = nullptr;
                a.fy = fyrec[f0]; a.bt = bt; a.gstr = (int32_t)gstr; a.gam = gam; a.car = carry;
                a.al = d_tt + TT_ALPHA; a.be = d_tt + TT_BETA;
                a.toff = d_geo + F + 1; a.ys = ys;
                a.q = QuantArgs{};
                if (qa) {
                    a.q = *qa;                                   /* the select's scratch is the stage region */
                    hlds = std::max(hlds, sizeof(QrShared));
                }
                (void)hipFuncSetAttribute((const void *)k_hilbert_env, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)hlds);
                LAUNCH(ctx, s, "k_hilbert_env", k_hilbert_env, dim3((unsigned)(f1 - f0)), dim3(HB_T), hlds, s, a, hp);
                for (int f = f0; f < f1; ++f) fused[f] = 1;
                f0 = f1;
                continue;
            }
        }
        if (rc != BPMX_OK) return rc;
        if (nd > 15 && !(P->options & BPMX_OPT_HILBERT_R2C)) {   /* batched Bluestein, after the loop */
            need_env = true;
            for (int f = f0; f < f1; ++f) blu.push_back(f);
        } else if (nd > 15) {
            need_env = true;
            FftPlans *pl = nullptr;
            if ((rc = get_plans(ctx->device, nd, f1 - f0, &pl)) != BPMX_OK) return rc;
            /* each run on a side stream chosen by Nd (a plan never runs on two
             * streams at once), its own work buffer; joined back into s below */
            if (!forked) {
                if (!ctx->side_ready()) return fail(BPMX_E_HIP, "side stream creation failed");
                HIP_TRY(hipEventRecord(ctx->side_fork, s));
                forked = true;
            }
            const int si = (int)(nd % bpmx_ctx::NSIDE);
            hipStream_t ss = ctx->side[si];
            if (!side_used[si]) {
                HIP_TRY(hipStreamWaitEvent(ss, ctx->side_fork, 0));
                side_used[si] = true;
            }
            void *work = pl->work ? ctx->buf("nat_fft_work" + std::to_string(si), pl->work, &rc) : nullptr;
            if (rc != BPMX_OK) return rc;
            rocfft_execution_info info = nullptr;
            rocfft_execution_info_create(&info);
            rocfft_execution_info_set_stream(info, ss);
            if (work) rocfft_execution_info_set_work_buffer(info, work, pl->work);
            void *in[1] = {yd + doff[f0]};
            void *out[1] = {z + doff[f0]};
            {
                Launch l(ctx, ss, "rocfft_r2c");
                rocfft_status st = rocfft_execute(pl->fwd, in, out, info);
                if (st != rocfft_status_success) { rocfft_execution_info_destroy(info); return fft_fail("rocfft_execute(r2c)", st); }
                if ((rc = l.done()) != BPMX_OK) { rocfft_execution_info_destroy(info); return rc; }
            }
            LAUNCH(ctx, ss, "k_hilbert_rotate", k_hilbert_rotate, dim3((unsigned)((nd / 2 + 256) / 256), f1 - f0),
                   dim3(256), 0, ss, z, d_doff, d_active, f0, f1);
            {
                Launch l(ctx, ss, "rocfft_c2r");
                void *hout[1] = {hb + doff[f0]};
                rocfft_status st = rocfft_execute(pl->inv, out, hout, info);
                if (st != rocfft_status_success) { rocfft_execution_info_destroy(info); return fft_fail("rocfft_execute(c2r)", st); }
                if ((rc = l.done()) != BPMX_OK) { rocfft_execution_info_destroy(info); return rc; }
            }
            rocfft_execution_info_destroy(info);
        }
        f0 = f1;
    }
    /* long recordings: exact-length four-step DFTs (k_longfft.hip) for every
     * length that factors for them, rocFFT Bluestein for the rest (or all of
     * them with BPMX_OPT_HILBERT_BLUESTEIN) */
    std::vector<int32_t> lf;
    if (!(P->options & BPMX_OPT_HILBERT_BLUESTEIN)) {
        std::vector<int32_t> rest;
        for (int32_t f : blu) (longfft_supported(doff[f + 1] - doff[f]) ? lf : rest).push_back(f);
        blu.swap(rest);
    }
    if ((rc = longfft_hilbert(ctx, s, yd, hb, doff, lf)) != BPMX_OK) return rc;
    if ((rc = bluestein_hilbert(ctx, s, yd, hb, doff, d_doff, blu)) != BPMX_OK) return rc;
    for (int i = 0; i < bpmx_ctx::NSIDE; ++i)       /* join the side streams back into s */
        if (side_used[i]) {
            HIP_TRY(hipEventRecord(ctx->side_join[i], ctx->side[i]));
            HIP_TRY(hipStreamWaitEvent(s, ctx->side_join[i], 0));
        }
    if (need_env) {                                   /* the rocFFT runs (fused runs are skipped) */
        int32_t *d_fused = (int32_t *)ctx->buf("nat_fused", (size_t)F * 4, &rc);
        if (rc != BPMX_OK) return rc;
        HIP_TRY(hipMemcpyAsync(d_fused, fused.data(), (size_t)F * 4, hipMemcpyHostToDevice, s));
        NatEnvArgs a;
        a.y = yd; a.h = hb; a.doff = d_doff; a.active = d_active; a.n_files = F; a.window = P->env_window;
        a.env = O->env; a.skip = d_fused;
        LAUNCH(ctx, s, "k_native_env", k_native_env, dim3((unsigned)((maxnd + NE_T - 1) / NE_T), F), dim3(NE_T), 0,
               s, a);
    }
    return BPMX_OK;
}

}  // namespace bpmx
