/*
 * k_envelope_native.hip — native mode envelope (north_star ordering):
 *   sosfiltfilt(butter(2,[20,150],'band',fs,'sos'), x) at the native rate
 *   -> y[::ds] -> |hilbert| -> centred rolling mean (window sr//10)
 * oracle: scipy/signal/_signaltools.py:4718-4829 (sosfiltfilt), :2318 (hilbert),
 * composed as SURVEY.md §8(a) A13 defines; tolerance 1e-9 relative on env.
 *
 * sosfiltfilt is linear and time-invariant, so the per-sample recursion over
 * one decimation block of ds samples collapses to 8 dot products (the block's
 * forward-state increment u_j and backward-state increment v_j; tables from
 * bpm_analysis_amd/native_tables.py).  That turns the HBM-bound part into a
 * fully parallel, coalesced streaming kernel:
 *
 *   k_native_blocks  every PCM sample read once from HBM (a tile of 128
 *                    blocks staged in LDS), 8 f64 FMA per sample,
 *                    64 B of (u_j, v_j) written per block.
 *   k_native_scan    one wave per recording: affine scans over blocks (lane
 *                    segments + a Kogge-Stone combine of 4x4 affine maps) for
 *                    the forward states S_j and backward states Q_j, the exact
 *                    per-sample recursion over the 15-sample head pad and the
 *                    <= ds+15-sample tail, and the decimated output
 *                    yd_j = C Q_j + D (C S_j + D x[j*ds]).
 *   rocFFT           R2C + C2C inverse (Hilbert), one plan per (Nd, batch).
 *   k_hilbert_weights  the analytic-signal weights h (1, 2, ..., 1, 0, ...).
 *   k_native_env     |z|/Nd and the centred rolling mean, LDS-tiled.
 */
#include <rocfft/rocfft.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <tuple>
#include <vector>

#include "bpmx_common.h"
#include "bpmx_kernels.h"
#include "bpmx_native.h"

namespace bpmx {

/* table layout (native_tables.pack) */
enum { TB_A = 0, TB_B = 16, TB_C = 20, TB_D = 24, TB_M = 25, TB_P = 41, TB_ZI = 57, TB_COEF = 64 };

struct NatTile;
struct NatBlockArgs {
    const void *pcm;
    const int64_t *foff, *boff;   /* frame offsets, block offsets (blocks = Nd-1 per file) */
    const int64_t *boffp;         /* padded per-file block storage: 64 * ceil(nb/64) entries */
    const struct NatTile *tiles;  /* int16 mono path: tile list */
    int64_t n_tiles, total;       /* tiles; samples in pcm */
    int bt;                       /* blocks per tile */
    const int32_t *active;
    int32_t n_files, channels, ds;
    const double *tab;
    double *uv;                    /* [sum blocks][8] */
};

struct NatScanArgs {
    const void *pcm;
    const int64_t *foff, *doff, *boff, *boffp;
    const int32_t *active;
    int32_t n_files, dtype, channels, ds;
    const double *tab;
    const double *uv;
    double *S;                     /* [sum blocks][4] forward block-start states */
    double *tail;                  /* [F][ds+16] */
    double *yd;                    /* [sumNd] decimated filtered signal */
};

struct NatEnvArgs {
    const double2 *z;              /* [sumNd] analytic signal (unnormalised) */
    const int64_t *doff;
    const int32_t *active;
    int32_t n_files, window;
    double *env;
};

/* ---------------------------------------------------------------------- */
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

/* int16 mono fast path.  Persistent single-wave workgroups walk a list of
 * tiles (up to 64 consecutive blocks of one file).  A tile's samples arrive
 * with coalesced 16-byte loads into registers — issued one tile AHEAD, so
 * HBM latency hides behind the current tile's FMAs — then go through LDS,
 * where lane b reads block b's ds+1 samples (lane stride ds/2 dwords: odd for
 * the usual ds, conflict-free).  The 8 coefficients of each sample are
 * wave-uniform scalar loads. */
constexpr int NB_RCH = 20;              /* 16-byte chunks per lane per tile: <= 10240 samples */
struct NatTile {
    int64_t s0;                         /* first sample of the tile (index into pcm) */
    int64_t ebase;                      /* boffp[f] */
    int32_t j0, nb;                     /* first block, blocks of the file */
};

__device__ __forceinline__ double nat_lo16(uint32_t w) { return (double)(int)(int16_t)(w & 0xFFFFu); }
__device__ __forceinline__ double nat_hi16(uint32_t w) { return (double)((int)w >> 16); }

typedef uint32_t nat_u4 __attribute__((ext_vector_type(4)));
/* `coef` is passed separately as __restrict__ so its loads become scalar
 * (wave-uniform) loads: the compiler must know the uv stores cannot alias it */
__global__ __launch_bounds__(64) void k_native_blocks_i16(NatBlockArgs A, const double *__restrict__ coef) {
    typedef nat_u4 u4;
    __shared__ u4 tile[NB_RCH * 64];
    const int lane = threadIdx.x;
    const int16_t *pcm = (const int16_t *)A.pcm;
    const int64_t total = A.total;
    const int ds = A.ds, bt = A.bt;
    const int nch = (7 + bt * ds + 1 + 7) >> 3;           /* chunks a tile may touch */
    auto issue = [&](int64_t t, u4 *reg, int &off) {
        const int64_t s0 = A.tiles[t].s0;
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
        const NatTile tl = A.tiles[t];
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
        if (lane < bt && j < tl.nb) {
            const int base = coff + lane * ds;                        /* halfword index in the tile */
            const uint32_t *wp = (const uint32_t *)tile + (base >> 1);
            const uint32_t sh = (base & 1) ? 16u : 0u;
            double u0 = 0, u1 = 0, u2 = 0, u3 = 0, v0 = 0, v1 = 0, v2 = 0, v3 = 0;
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
            const uint32_t R = ((uint32_t)tl.nb + 63u) >> 6;
            const int64_t e = tl.ebase + (int64_t)((uint32_t)j % R) * 64 + (uint32_t)j / R;
            double2 *o = (double2 *)(A.uv + e * 8);
            o[0] = make_double2(u0, u1); o[1] = make_double2(u2, u3);
            o[2] = make_double2(v0, v1); o[3] = make_double2(v2, v3);
        }
        __syncthreads();
        t = tn;
    }
}

/* generic path (other sample formats, multi-channel): f64 tile, 32 blocks per group */
template <int DT, bool MULTI>
__global__ __launch_bounds__(64) void k_native_blocks_gen(NatBlockArgs A) {
    constexpr int NBG = 32;
    extern __shared__ __align__(16) double tile_d[];   /* 32*ds + 1 */
    double *tile = tile_d;
    const int f = blockIdx.y;
    if (f >= A.n_files || !A.active[f]) return;
    const int64_t nb = A.boff[f + 1] - A.boff[f];
    const int64_t j0 = (int64_t)blockIdx.x * NBG;
    if (j0 >= nb) return;
    const int ds = A.ds, tid = threadIdx.x;
    const int64_t nblk = nb - j0 < NBG ? nb - j0 : NBG;
    const int64_t nsamp = nblk * ds + 1;
    const int64_t fb = A.foff[f] + j0 * ds;
    for (int64_t i = tid; i < nsamp; i += 64) tile[i] = nat_frame<DT, MULTI>(A.pcm, A.channels, fb + i);
    __syncthreads();
    if (tid >= nblk) return;
    const double *__restrict__ coef = A.tab + TB_COEF;
    const double *x = tile + tid * ds;
    double u0 = 0, u1 = 0, u2 = 0, u3 = 0, v0 = 0, v1 = 0, v2 = 0, v3 = 0;
    for (int i = 0; i < ds; ++i) {
        const double xv = x[i];
        const double *c = coef + i * 8;
        u0 = __builtin_fma(c[0], xv, u0); u1 = __builtin_fma(c[1], xv, u1);
        u2 = __builtin_fma(c[2], xv, u2); u3 = __builtin_fma(c[3], xv, u3);
        v0 = __builtin_fma(c[4], xv, v0); v1 = __builtin_fma(c[5], xv, v1);
        v2 = __builtin_fma(c[6], xv, v2); v3 = __builtin_fma(c[7], xv, v3);
    }
    {
        const double xv = x[ds];
        const double *c = coef + ds * 8;
        v0 = __builtin_fma(c[4], xv, v0); v1 = __builtin_fma(c[5], xv, v1);
        v2 = __builtin_fma(c[6], xv, v2); v3 = __builtin_fma(c[7], xv, v3);
    }
    const int64_t j = j0 + tid, R = (nb + 63) >> 6;
    double2 *o = (double2 *)(A.uv + (A.boffp[f] + (j % R) * 64 + j / R) * 8);
    o[0] = make_double2(u0, u1); o[1] = make_double2(u2, u3);
    o[2] = make_double2(v0, v1); o[3] = make_double2(v2, v3);
}

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
__device__ __forceinline__ V4 add4(const V4 &x, const V4 &y) { return V4{x.a + y.a, x.b + y.b, x.c + y.c, x.d + y.d}; }
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

/* One wave per recording.  Block j of the file is held by lane j / R at step
 * t = j % R (R = ceil(nb/64)); per-block data lives at [t][lane], so each step
 * of the lane loops is one coalesced 4-KiB access, prefetched one step ahead. */
__global__ __launch_bounds__(64) void k_native_scan(NatScanArgs A, SosStep SS) {
    const int f = blockIdx.x;
    if (f >= A.n_files || !A.active[f]) return;
    const int lane = threadIdx.x;
    const int64_t nd = A.doff[f + 1] - A.doff[f];
    const int64_t nb = nd - 1;
    const int64_t n = A.foff[f + 1] - A.foff[f];
    const int64_t fb = A.foff[f];
    const int ds = A.ds;
    const int wdt = work_dtype(A.dtype, A.channels);
    const double *tb = A.tab;
    M4 Mm, Pm;
#pragma unroll
    for (int i = 0; i < 16; ++i) { Mm.m[i] = tb[TB_M + i]; Pm.m[i] = tb[TB_P + i]; }
    const V4 Cv{tb[TB_C], tb[TB_C + 1], tb[TB_C + 2], tb[TB_C + 3]};
    const double Dd = tb[TB_D];
    const V4 zi{tb[TB_ZI], tb[TB_ZI + 1], tb[TB_ZI + 2], tb[TB_ZI + 3]};
    auto x = [&](int64_t k) { return frame_value(A.pcm, A.dtype, A.channels, fb + k); };
    const double4 *uv = (const double4 *)(A.uv + A.boffp[f] * 8);   /* entry e: uv[2e] = u, uv[2e+1] = v */
    double4 *S = (double4 *)(A.S + A.boffp[f] * 4);
    double *yd = A.yd + A.doff[f];

    /* (a) head: 15 padded samples, exact recursion (redundant in every lane) */
    V4 s0;
    {
        const double x0 = x(0);
        const double e0 = odd_ext(wdt, x0, x(15));
        V4 z{zi.a * e0, zi.b * e0, zi.c * e0, zi.d * e0};
        for (int k = 0; k < 15; ++k) (void)SS.step(z, odd_ext(wdt, x0, x(15 - k)));
        s0 = z;
    }
    const int64_t R = (nb + 63) >> 6;
    const int64_t lo = lane * R < nb ? lane * R : nb;
    const int64_t len = (lo + R < nb ? lo + R : nb) - lo;
    auto U = [&](int64_t t) { const double4 w = uv[2 * (t * 64 + lane)]; return V4{w.x, w.y, w.z, w.w}; };
    auto Vv = [&](int64_t t) { const double4 w = uv[2 * (t * 64 + lane) + 1]; return V4{w.x, w.y, w.z, w.w}; };

    /* (b) forward: segment map a = sum M^.. u, then Kogge-Stone across lanes */
    V4 a{0, 0, 0, 0};
    {
        V4 un = R > 0 ? U(0) : V4{0, 0, 0, 0};
        for (int64_t t = 0; t < R; ++t) {
            const V4 uc = un;
            if (t + 1 < R) un = U(t + 1);
            if (t < len) a = add4(mv(Mm, a), uc);
        }
    }
    const M4 Tl = mpow(Mm, len);
    M4 T = Tl;
    for (int d = 1; d < 64; d <<= 1) {
        const M4 To = shfl_up_m(T, d);
        const V4 ao = shfl_up_v(a, d);
        if (lane >= d) { a = add4(mv(T, ao), a); T = mm(T, To); }
    }
    M4 Te = shfl_up_m(T, 1);
    V4 ae = shfl_up_v(a, 1);
    if (lane == 0) { Te = eye4(); ae = V4{0, 0, 0, 0}; }
    V4 st = add4(mv(Te, s0), ae);
    {
        V4 un = R > 0 ? U(0) : V4{0, 0, 0, 0};
        for (int64_t t = 0; t < R; ++t) {
            const V4 uc = un;
            if (t + 1 < R) un = U(t + 1);
            if (t < len) {
                S[t * 64 + lane] = make_double4(st.a, st.b, st.c, st.d);
                st = add4(mv(Mm, st), uc);
            }
        }
    }
    const int last_lane = nb > 0 ? (int)((nb - 1) / R) : 0;
    V4 slast = shfl_v(st, last_lane);
    if (nb == 0) slast = s0;

    /* (c) tail [c_{nd-1}, ne): exact forward then backward recursion, lane 0 */
    __shared__ double s_q[4];
    if (lane == 0) {
        double *tl = A.tail + (int64_t)f * (ds + 16);
        const int64_t base = (nd - 1) * ds;     /* x index of c_{nd-1} */
        const int64_t nt = n - base + 15;         /* tail length incl. right pad */
        const double xl = x(n - 1);
        V4 z = slast;
        for (int64_t k = 0; k < nt; ++k) {
            const int64_t xi = base + k;
            const double u = xi < n ? x(xi) : odd_ext(wdt, xl, x(n - 2 - (xi - n)));
            tl[k] = SS.step(z, u);
        }
        const double y0 = tl[nt - 1];
        V4 q{zi.a * y0, zi.b * y0, zi.c * y0, zi.d * y0};
        for (int64_t k = nt - 1; k >= 1; --k) (void)SS.step(q, tl[k]);
        s_q[0] = q.a; s_q[1] = q.b; s_q[2] = q.c; s_q[3] = q.d;
        yd[nd - 1] = Cv.a * q.a + Cv.b * q.b + Cv.c * q.c + Cv.d * q.d + Dd * tl[0];
    }
    __syncthreads();
    const V4 qlast{s_q[0], s_q[1], s_q[2], s_q[3]};

    /* (d) backward: Q_j = M Q_{j+1} + P S_j + v_j from Q_{nb} = qlast */
    auto Sv = [&](int64_t t) { const double4 w = S[t * 64 + lane]; return V4{w.x, w.y, w.z, w.w}; };
    V4 b{0, 0, 0, 0};
    {
        V4 sn = R > 0 ? Sv(R - 1) : V4{0, 0, 0, 0}, vn = R > 0 ? Vv(R - 1) : V4{0, 0, 0, 0};
        for (int64_t t = R - 1; t >= 0; --t) {
            const V4 sc = sn, vc = vn;
            if (t > 0) { sn = Sv(t - 1); vn = Vv(t - 1); }
            if (t < len) b = add4(mv(Mm, b), add4(mv(Pm, sc), vc));
        }
    }
    T = Tl;
    for (int d = 1; d < 64; d <<= 1) {
        const M4 To = shfl_down_m(T, d);
        const V4 bo = shfl_down_v(b, d);
        if (lane + d < 64) { b = add4(mv(T, bo), b); T = mm(T, To); }
    }
    Te = shfl_down_m(T, 1);
    V4 be = shfl_down_v(b, 1);
    if (lane == 63) { Te = eye4(); be = V4{0, 0, 0, 0}; }
    V4 q = add4(mv(Te, qlast), be);
    {
        V4 sn = R > 0 ? Sv(R - 1) : V4{0, 0, 0, 0}, vn = R > 0 ? Vv(R - 1) : V4{0, 0, 0, 0};
        double xn = len > 0 ? x((lo + (R - 1 < len - 1 ? R - 1 : len - 1)) * ds) : 0.0;
        for (int64_t t = R - 1; t >= 0; --t) {
            const V4 sc = sn, vc = vn;
            const double xc = xn;
            if (t > 0) {
                sn = Sv(t - 1); vn = Vv(t - 1);
                const int64_t tt = t - 1 < len - 1 ? t - 1 : (len > 0 ? len - 1 : 0);
                xn = x((lo + tt) * ds);
            }
            if (t < len) {
                q = add4(mv(Mm, q), add4(mv(Pm, sc), vc));
                const double yf = Cv.a * sc.a + Cv.b * sc.b + Cv.c * sc.c + Cv.d * sc.d + Dd * xc;
                yd[lo + t] = Cv.a * q.a + Cv.b * q.b + Cv.c * q.c + Cv.d * q.d + Dd * yf;
            }
        }
    }
}

/* ---------------------------------------------------------------------- */
/* analytic-signal weights on the R2C half spectrum, written as a full-length
 * complex spectrum in place (slot of Nd complex values per file) */
__global__ __launch_bounds__(256) void k_hilbert_weights(double2 *z, const int64_t *doff, const int32_t *active,
                                                         int f_begin, int f_end) {
    const int f = f_begin + blockIdx.y;
    if (f >= f_end || !active[f]) return;
    const int64_t n = doff[f + 1] - doff[f];
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    double2 *zf = z + doff[f];
    double w;
    if (k == 0) w = 1.0;
    else if ((n % 2 == 0) && k == n / 2) w = 1.0;
    else if (k < (n + 1) / 2) w = 2.0;
    else w = 0.0;
    if (w == 0.0) zf[k] = make_double2(0.0, 0.0);
    else if (w == 2.0) { double2 c = zf[k]; zf[k] = make_double2(2.0 * c.x, 2.0 * c.y); }
}

/* |z|/Nd and the centred rolling mean (window w, min_periods 1) */
constexpr int NE_T = 256;
__global__ __launch_bounds__(NE_T) void k_native_env(NatEnvArgs A) {
    __shared__ double mag[NE_T + 2 * 1024];
    const int f = blockIdx.y;
    if (f >= A.n_files || !A.active[f]) return;
    const int64_t n = A.doff[f + 1] - A.doff[f];
    const int64_t i0 = (int64_t)blockIdx.x * NE_T;
    if (i0 >= n) return;
    const int64_t w = A.window, off = (w - 1) / 2;
    const int64_t lo = i0 + 1 + off - w < 0 ? 0 : i0 + 1 + off - w;
    const int64_t hiE = i0 + NE_T + off < n ? i0 + NE_T + off : n;   /* exclusive */
    const double2 *z = A.z + A.doff[f];
    const double inv = 1.0 / (double)n;
    for (int64_t p = lo + threadIdx.x; p < hiE; p += NE_T) {
        const double2 c = z[p];
        mag[p - lo] = sqrt(c.x * c.x + c.y * c.y) * inv;
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
std::map<std::tuple<int, int64_t, int64_t>, FftPlans> g_plans;   /* (device, nd, batch) */
bool g_fft_setup = false;

int fft_fail(const char *what, rocfft_status st) {
    return fail(BPMX_E_HIP, std::string(what) + " failed (rocfft status " + std::to_string((int)st) + ")");
}

int get_plans(int dev, int64_t nd, int64_t batch, FftPlans **out) {
    if (!g_fft_setup) {
        rocfft_status st = rocfft_setup();
        if (st != rocfft_status_success) return fft_fail("rocfft_setup", st);
        g_fft_setup = true;
    }
    auto key = std::make_tuple(dev, nd, batch);
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
    st = rocfft_plan_description_set_data_layout(d2, rocfft_array_type_complex_interleaved,
                                                 rocfft_array_type_complex_interleaved, nullptr, nullptr, 1, nullptr,
                                                 len, 1, nullptr, len);
    if (st != rocfft_status_success) return fft_fail("set_data_layout(c2c)", st);
    st = rocfft_plan_create(&p.inv, rocfft_placement_inplace, rocfft_transform_type_complex_inverse,
                            rocfft_precision_double, 1, &len, (size_t)batch, d2);
    if (st != rocfft_status_success) return fft_fail("plan_create(c2c)", st);
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

std::vector<double> build_tables(const double *sos, const double *sos_zi, int L) {
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
    std::vector<double> out(64 + 8 * (size_t)(L + 1), 0.0);
    for (int i = 0; i < 16; ++i) out[TB_A + i] = (double)A.m[i];
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
    }
    return out;
}
}  // namespace

int native_envelope(bpmx_ctx *ctx, const bpmx_params *P, const bpmx_batch *B, const bpmx_out *O, hipStream_t s,
                    int F, const std::vector<int64_t> &foff, const std::vector<int64_t> &doff, int64_t maxnd,
                    const int64_t *d_foff, const int64_t *d_doff, const int32_t *d_active) {
    const int ds = P->ds;
    if (ds > 300) return fail(BPMX_E_LIMIT, "native mode supports ds <= 300");
    int rc = BPMX_OK;
    /* tables (cached on the host key; uploaded when they change) */
    /* tables and block offsets: rebuilt / re-uploaded only when they change (the
     * host copies live in the context, so the async upload never outlives them) */
    std::vector<int64_t> key(15);
    for (int i = 0; i < 12; ++i) std::memcpy(&key[i], &P->sos[i], 8);
    key[12] = ds;
    std::memcpy(&key[13], &P->sos_zi[0], 8);
    std::memcpy(&key[14], &P->sos_zi[2], 8);
    if (key != ctx->nat_key) {
        ctx->nat_tab = build_tables(P->sos, P->sos_zi, ds);
        ctx->nat_key = key;
        ctx->nat_tab_dirty = true;
    }
    bool grew = false;
    double *d_tab = (double *)ctx->buf("nat_tab", ctx->nat_tab.size() * 8, &rc, &grew);
    if (grew) ctx->nat_tab_dirty = true;
    std::vector<int64_t> boff(F + 1, 0);
    for (int f = 0; f < F; ++f) {
        const int64_t nd = doff[f + 1] - doff[f];
        boff[f + 1] = boff[f] + (nd > 1 ? nd - 1 : 0);
    }
    std::vector<int64_t> boffp(F + 1, 0);
    for (int f = 0; f < F; ++f) boffp[f + 1] = boffp[f] + ((boff[f + 1] - boff[f] + 63) / 64) * 64;
    const int64_t sum_blocks = boffp[F];
    int64_t *d_boff2 = (int64_t *)ctx->buf("nat_boff", (size_t)(F + 1) * 16, &rc, &grew);
    if (grew) ctx->nat_boff.clear();
    if (rc != BPMX_OK) return rc;
    if (ctx->nat_tab_dirty) {
        HIP_TRY(hipMemcpyAsync(d_tab, ctx->nat_tab.data(), ctx->nat_tab.size() * 8, hipMemcpyHostToDevice, s));
        ctx->nat_tab_dirty = false;
    }
    std::vector<int64_t> both(boff);
    both.insert(both.end(), boffp.begin(), boffp.end());
    if (both != ctx->nat_boff) {
        ctx->nat_boff = both;
        HIP_TRY(hipMemcpyAsync(d_boff2, ctx->nat_boff.data(), (size_t)(F + 1) * 16, hipMemcpyHostToDevice, s));
    }
    const int64_t *d_boffp = d_boff2 + F + 1;
    double *uv = (double *)ctx->buf("nat_uv", (size_t)std::max<int64_t>(sum_blocks, 1) * 64, &rc);
    double *S = (double *)ctx->buf("nat_S", (size_t)std::max<int64_t>(sum_blocks, 1) * 32, &rc);
    double *tail = (double *)ctx->buf("nat_tail", (size_t)F * (ds + 16) * 8, &rc);
    double *yd = O->y ? O->y : (double *)ctx->buf("nat_yd", (size_t)doff[F] * 8, &rc);
    double2 *z = (double2 *)ctx->buf("nat_z", (size_t)doff[F] * 16, &rc);
    if (rc != BPMX_OK) return rc;
    int64_t maxnb = 0;
    for (int f = 0; f < F; ++f) maxnb = std::max<int64_t>(maxnb, doff[f + 1] - doff[f] - 1);
    {
        NatBlockArgs a;
        a.pcm = B->pcm; a.foff = d_foff; a.boff = d_boff2; a.boffp = d_boffp; a.active = d_active; a.n_files = F;
        a.channels = P->channels; a.ds = ds; a.tab = d_tab; a.uv = uv;
        const bool fast = P->dtype == BPMX_DT_I16 && P->channels == 1 && ((uintptr_t)B->pcm & 15) == 0;
        if (maxnb > 0) {
            if (fast) {
                const int bt = std::min(64, (NB_RCH * 512 - 16) / ds);
                std::vector<int64_t> tk(3 + F);
                tk[0] = bt; tk[1] = F; tk[2] = foff[F];
                for (int f = 0; f < F; ++f) tk[3 + f] = foff[f];
                if (tk != ctx->nat_tkey || doff != ctx->nat_tdoff) {
                    std::vector<NatTile> tv;
                    for (int f = 0; f < F; ++f) {
                        const int64_t nd = doff[f + 1] - doff[f];
                        if (nd <= 15) continue;                      /* inactive (filtfilt would raise) */
                        const int64_t nb = nd - 1;
                        for (int64_t j0 = 0; j0 < nb; j0 += bt)
                            tv.push_back(NatTile{foff[f] + j0 * ds, boffp[f], (int32_t)j0, (int32_t)nb});
                    }
                    ctx->nat_tiles.resize(tv.size() * sizeof(NatTile));
                    std::memcpy(ctx->nat_tiles.data(), tv.data(), ctx->nat_tiles.size());
                    ctx->nat_tkey = tk;
                    ctx->nat_tdoff = doff;
                    ctx->nat_tiles_dirty = true;
                }
                const int64_t nt = (int64_t)(ctx->nat_tiles.size() / sizeof(NatTile));
                NatTile *d_tiles =
                    (NatTile *)ctx->buf("nat_tiles", std::max<size_t>(ctx->nat_tiles.size(), 64), &rc, &grew);
                if (rc != BPMX_OK) return rc;
                if (grew) ctx->nat_tiles_dirty = true;
                if (ctx->nat_tiles_dirty) {
                    HIP_TRY(hipMemcpyAsync(d_tiles, ctx->nat_tiles.data(), ctx->nat_tiles.size(),
                                           hipMemcpyHostToDevice, s));
                    ctx->nat_tiles_dirty = false;
                }
                a.tiles = d_tiles; a.n_tiles = nt; a.total = foff[F]; a.bt = bt;
                const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>(nt, 1), 256 * 8);
                if (nt > 0) LAUNCH(ctx, s, "k_native_blocks", k_native_blocks_i16, dim3(grid), dim3(64), 0, s, a,
                                   (const double *)(d_tab + TB_COEF));
            } else {
                const dim3 g((unsigned)((maxnb + 31) / 32), F), b(64);
                const size_t lds = ((size_t)32 * ds + 1) * 8;
#define NAT_GEN(DT)                                                                                        \
    if (P->channels > 1) {                                                                                 \
        (void)hipFuncSetAttribute((const void *)k_native_blocks_gen<DT, true>,                             \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                   \
        LAUNCH(ctx, s, "k_native_blocks", (k_native_blocks_gen<DT, true>), g, b, lds, s, a);               \
    } else {                                                                                               \
        (void)hipFuncSetAttribute((const void *)k_native_blocks_gen<DT, false>,                            \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                   \
        LAUNCH(ctx, s, "k_native_blocks", (k_native_blocks_gen<DT, false>), g, b, lds, s, a);              \
    }
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
    }
    {
        NatScanArgs a;
        a.pcm = B->pcm; a.foff = d_foff; a.doff = d_doff; a.boff = d_boff2; a.boffp = d_boffp; a.active = d_active;
        a.n_files = F;
        a.dtype = P->dtype; a.channels = P->channels; a.ds = ds; a.tab = d_tab; a.uv = uv; a.S = S; a.tail = tail;
        a.yd = yd;
        SosStep ss;
        for (int i = 0; i < 12; ++i) ss.s[i] = P->sos[i];
        LAUNCH(ctx, s, "k_native_scan", k_native_scan, dim3(F), dim3(64), 0, s, a, ss);
    }
    /* Hilbert: runs of equal Nd share one batched plan */
    int f0 = 0;
    while (f0 < F) {
        const int64_t nd = doff[f0 + 1] - doff[f0];
        int f1 = f0 + 1;
        while (f1 < F && doff[f1 + 1] - doff[f1] == nd) ++f1;
        if (nd > 15) {
            FftPlans *pl = nullptr;
            if ((rc = get_plans(ctx->device, nd, f1 - f0, &pl)) != BPMX_OK) return rc;
            void *work = pl->work ? ctx->buf("nat_fft_work", pl->work, &rc) : nullptr;
            if (rc != BPMX_OK) return rc;
            rocfft_execution_info info = nullptr;
            rocfft_execution_info_create(&info);
            rocfft_execution_info_set_stream(info, s);
            if (work) rocfft_execution_info_set_work_buffer(info, work, pl->work);
            void *in[1] = {yd + doff[f0]};
            void *out[1] = {z + doff[f0]};
            {
                Launch l(ctx, s, "rocfft_r2c");
                rocfft_status st = rocfft_execute(pl->fwd, in, out, info);
                if (st != rocfft_status_success) { rocfft_execution_info_destroy(info); return fft_fail("rocfft_execute(r2c)", st); }
                if ((rc = l.done()) != BPMX_OK) { rocfft_execution_info_destroy(info); return rc; }
            }
            LAUNCH(ctx, s, "k_hilbert_weights", k_hilbert_weights, dim3((unsigned)((nd + 255) / 256), f1 - f0),
                   dim3(256), 0, s, z, d_doff, d_active, f0, f1);
            {
                Launch l(ctx, s, "rocfft_c2c_inv");
                rocfft_status st = rocfft_execute(pl->inv, out, nullptr, info);
                if (st != rocfft_status_success) { rocfft_execution_info_destroy(info); return fft_fail("rocfft_execute(c2c)", st); }
                if ((rc = l.done()) != BPMX_OK) { rocfft_execution_info_destroy(info); return rc; }
            }
            rocfft_execution_info_destroy(info);
        }
        f0 = f1;
    }
    {
        if (P->env_window > 2 * 1024) return fail(BPMX_E_LIMIT, "envelope window too large for k_native_env");
        NatEnvArgs a;
        a.z = z; a.doff = d_doff; a.active = d_active; a.n_files = F; a.window = P->env_window; a.env = O->env;
        LAUNCH(ctx, s, "k_native_env", k_native_env, dim3((unsigned)((maxnd + NE_T - 1) / NE_T), F), dim3(NE_T), 0,
               s, a);
    }
    return BPMX_OK;
}

}  // namespace bpmx
