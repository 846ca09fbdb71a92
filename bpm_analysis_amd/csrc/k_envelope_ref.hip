/*
 * k_envelope_ref.hip — reference-mode envelope, bit-exact.
 *
 * Restates bpm_analysis.py:1031-1054 for a batch of recordings:
 *   x[::ds] (no anti-alias, :1033) -> filtfilt(b, a) at the decimated rate
 *   (:1044-1045; scipy _signaltools.py:4523-4557, odd pad of 15 in the input
 *   dtype, DF-II-transposed recursion of _sigtools._linear_filter) -> |y| ->
 *   pandas centred rolling mean, Kahan add/remove (:1052-1054).
 *
 * Bit-exactness forces a strictly sequential recursion per recording, so the
 * parallelism is across recordings: one lane per file, 64 files per wave.
 * What remains is a latency problem, and the kernel is built around it:
 *  - the forward output is parked in an interleaved scratch [step][file] so
 *    the 64 lanes of a wave touch one contiguous 512-B row per step;
 *  - every sequential stream (the stride-ds PCM gather, the scratch read of
 *    the backward pass, the add and remove streams of the rolling mean) is
 *    software-pipelined one 16-step block ahead in registers, so a block's
 *    loads are in flight while the previous block's f64 recursion runs;
 *  - env / y rows are transposed through LDS and written 512 B per
 *    instruction instead of 64 scattered 8-B stores.
 * Roofline: the f64 dependency chain (~3 dependent ops per step, ~17 ops
 * issued per step by one wave) — neither HBM nor VALU throughput.
 *
 * The rolling mean splits into its chain and the rest ("chain mode", waves
 * whose |y| has no NaN): only the Kahan add/remove recursion on sum_x is
 * sequential, so the pass keeps just that (8 f64 ops per step, the running sum
 * stored per step), and k_ref_env_mean forms every output in parallel from
 * it — nobs from the window bounds, the run of equal added values and the
 * last added value from |y| itself, then calc_mean's division and tests with
 * the same rounded operations (pandas aggregations.pyx roll_mean).
 */
#include "bpmx_common.h"
#include "bpmx_kernels.h"
#include "bpmx_stamps.h"

namespace bpmx {

/* ---- compile-time PCM loaders (frame value after the channel mean) ---- */
template <int DT>
struct Pcm;
template <> struct Pcm<BPMX_DT_U8> { typedef uint8_t T; };
template <> struct Pcm<BPMX_DT_I16> { typedef int16_t T; };
template <> struct Pcm<BPMX_DT_I32> { typedef int32_t T; };
template <> struct Pcm<BPMX_DT_F32> { typedef float T; };
template <> struct Pcm<BPMX_DT_F64> { typedef double T; };

template <int DT, bool MULTI>
__device__ __forceinline__ double frame_at(const void *__restrict__ pcm, int ch, int64_t frame) {
    typedef typename Pcm<DT>::T T;
    const T *p = (const T *)pcm;
    if (!MULTI) return (double)p[frame];
    if (DT == BPMX_DT_F32) {
        const float *q = (const float *)pcm + frame * ch;
        float s = q[0];
        for (int c = 1; c < ch; ++c) s = s + q[c];
        return (double)(s / (float)ch);
    }
    double s = (double)p[frame * ch];
    for (int c = 1; c < ch; ++c) s = s + (double)p[frame * ch + c];
    return s / (double)ch;
}

struct Df2t {
    double b0, b1, b2, b3, b4, a1, a2, a3, a4;
    double z0, z1, z2, z3;
    /* scipy DOUBLE filt loop: y = Z0 + b0*x; Z_k = Z_{k+1} + x*b_{k+1} - y*a_{k+1}.
     * ZB: the butter band-pass form b = k (1, 0, -2, 0, 1) exactly (its
     * numerator is k (z^2 - 1)^2; the host checks b1 = b3 = 0, b4 = b0 and
     * b2 = -2 b0 bit for bit) and a finite input (integer PCM):
     *  - x*0 is a zero and z + (+-0) == z, so those two products and sums are
     *    skipped — equal values (at most the sign of an exact zero differs,
     *    inside all-zero stretches; |y| and the envelope are unchanged);
     *  - x*b4 is b0*x, and x*b2 = -2 (b0*x) exactly (|b0 x| is 0 or far above
     *    the subnormals for integer x), so z2 + x*b2 is one FMA of the exact
     *    product -2 (b0 x): 13 -> 11 f64 instructions per step */
    template <bool ZB = false>
    __device__ __forceinline__ double step(double xn) {
        /* the same rounded operations, the x-only ones first: only
         * z0 + b0 x -> y a1 -> (z1 + x b1) - y a1 is on the chain to the next y */
        const double bx0 = b0 * xn;
        const double bx2 = ZB ? 0.0 : xn * b2, bx4 = ZB ? bx0 : xn * b4;
        const double bx1 = ZB ? 0.0 : xn * b1, bx3 = ZB ? 0.0 : xn * b3;
        const double p1 = ZB ? z1 : z1 + bx1, p3 = ZB ? z3 : z3 + bx3;
        const double p2 = ZB ? __builtin_fma(-2.0, bx0, z2) : z2 + bx2;
        const double yn = z0 + bx0;
        z0 = p1 - yn * a1;
        z1 = p2 - yn * a2;
        z2 = p3 - yn * a3;
        z3 = bx4 - yn * a4;
        return yn;
    }
    __device__ __forceinline__ void init(const double *zi, double x0) {
        z0 = zi[0] * x0; z1 = zi[1] * x0; z2 = zi[2] * x0; z3 = zi[3] * x0;
    }
};

/* pandas roll_mean state (aggregations.pyx add_mean / remove_mean / calc_mean) */
struct RollMean {
    double sum = 0, cadd = 0, crem = 0, prev = 0;
    int32_t nobs = 0, neg = 0, same = 0;   /* <= recording length (< 2^31, host-checked) */
    /* exact copies across the launches of a chunked pass: 6 doubles */
    __device__ __forceinline__ void save(double *z) const {
        z[0] = sum; z[1] = cadd; z[2] = crem; z[3] = prev;
        z[4] = __longlong_as_double(((long long)nobs << 32) | (unsigned)neg); z[5] = __longlong_as_double(same);
    }
    __device__ __forceinline__ void load(const double *z) {
        sum = z[0]; cadd = z[1]; crem = z[2]; prev = z[3];
        const long long a = __double_as_longlong(z[4]);
        nobs = (int32_t)(a >> 32); neg = (int32_t)(unsigned)(a & 0xFFFFFFFFll); same = (int32_t)__double_as_longlong(z[5]);
    }
    __device__ __forceinline__ void add(double v) {
        if (v == v) {
            nobs++;
            double y = v - cadd, t = sum + y;
            cadd = t - sum - y;
            sum = t;
            if (__signbit(v)) neg++;
            if (v == prev) same++; else same = 1;
            prev = v;
        }
    }
    __device__ __forceinline__ void remove(double v) {
        if (v == v) {
            nobs--;
            double y = -v - crem, t = sum + y;
            crem = t - sum - y;
            sum = t;
            if (__signbit(v)) neg--;
        }
    }
    /* branch-free forms (selects instead of the NaN / tie branches), the same
     * rounded operations when they apply: one basic block per prefetch block */
    __device__ __forceinline__ void add_sel(double v) {
        const bool ok = v == v;
        const double y = v - cadd, t = sum + y;
        cadd = ok ? (t - sum) - y : cadd;
        sum = ok ? t : sum;
        nobs += ok ? 1 : 0;
        neg += (ok && __signbit(v)) ? 1 : 0;
        int32_t sn = v == prev ? same + 1 : 1;
        __asm__ volatile("" : "+v"(sn));          /* keep it a select, not a branch */
        same = ok ? sn : same;
        prev = ok ? v : prev;
    }
    __device__ __forceinline__ void remove_sel(double v) {
        const bool ok = v == v;
        const double y = -v - crem, t = sum + y;
        crem = ok ? (t - sum) - y : crem;
        sum = ok ? t : sum;
        nobs -= ok ? 1 : 0;
        neg -= (ok && __signbit(v)) ? 1 : 0;
    }
    __device__ __forceinline__ double mean_sel() const {
        double r = sum / (double)nobs;
        __asm__ volatile("" : "+v"(r));           /* divide every step (its latency overlaps), no branch */
        r = same >= nobs ? prev : ((neg == 0 && r < 0) || (neg == nobs && r > 0) ? 0.0 : r);
        return nobs >= 1 ? r : __builtin_nan("");
    }
    __device__ __forceinline__ double mean() const {
        if (nobs >= 1) {
            double r = sum / (double)nobs;
            if (same >= nobs) r = prev;
            else if (neg == 0 && r < 0) r = 0;
            else if (neg == nobs && r > 0) r = 0;
            return r;
        }
        return __builtin_nan("");
    }
};

#ifndef BPMX_REF_PFB
#define BPMX_REF_PFB 64
#endif
#ifndef BPMX_REF_PF
#define BPMX_REF_PF 32
#endif
constexpr int PF = BPMX_REF_PF;   /* prefetch block (steps), rolling-mean phase */
constexpr int PFB = BPMX_REF_PFB;   /* prefetch block of the two filter passes */
constexpr int STG = 64;  /* LDS staging rows */

/* write the staged rows [base, base+rows) of every file in the wave, 512 B per store */
__device__ __forceinline__ void flush_rows(double (*stage)[65], double *__restrict__ dst, int64_t base, int rows,
                                           int64_t my_d0, int64_t my_nd) {
    const int lane = lane_id();
    for (int fl = 0; fl < 64; ++fl) {
        const int64_t d0 = __shfl(my_d0, fl);
        const int64_t nd = __shfl(my_nd, fl);
        const int64_t i = base + lane;
        if (lane < rows && i < nd) dst[d0 + i] = stage[lane][fl];
    }
}

/* The odd-extended decimated input of filtfilt (x[::ds], 15 padded samples
 * each side in the input dtype) gathered for every recording into the scratch
 * rows [0, Nd + 30) that the forward pass then filters in place.  The stride-ds
 * picks touch one cache line each; gathered here by many waves at once, with
 * one recording's consecutive picks per wave (neighbouring pages), and
 * transposed through LDS into [row][recording] rows, instead of inside the
 * sequential pass, where 64 scattered picks per step (one per lane, 5 MB
 * apart) cost ~440 cycles per step (tools/chainbench). */
template <int DT, bool MULTI>
__global__ __launch_bounds__(256) void k_ref_pick(EnvRefArgs A) {
    __shared__ double tile[64][65];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t r0 = A.pick_r0 + (int64_t)blockIdx.x * 64, f0 = (int64_t)blockIdx.y * 64;
    const int64_t S = A.n_files, ds = A.ds;
    const int ch = A.channels, wdt = work_dtype(DT, MULTI ? 2 : 1);
    for (int fi = wv; fi < 64; fi += 4) {
        const int64_t f = f0 + fi;
        double v = 0.0;
        if (f < S) {
            const int64_t nd = A.doff[f + 1] - A.doff[f], r = r0 + lane;
            if (nd > 15 && A.active[f] && r < nd + 30) {
                const int64_t fb = A.foff[f], last = nd - 1;
                auto xd = [&](int64_t j) { return frame_at<DT, MULTI>(A.pcm, ch, fb + j * ds); };
                if (r < 15) v = odd_ext(wdt, xd(0), xd(15 - r));
                else if (r < 15 + nd) v = xd(r - 15);
                else v = odd_ext(wdt, xd(last), xd(last - 1 - (r - 15 - nd)));
            }
        }
        tile[lane][fi] = v;
    }
    __syncthreads();
    for (int ri = wv; ri < 64; ri += 4) {
        const int64_t r = r0 + ri, f = f0 + lane;
        if (f < S) A.scratch[r * S + f] = tile[ri][lane];
    }
}

/* The rolling mean's Kahan add/remove recursion on sum_x alone (chain mode),
 * storing the running sum of every step as pair rows [i / 2][file][2]: one
 * 16-B store per two steps (tools/lanebench: 161 -> 87 cycles per step with
 * the remove stream below).  The value removed at step i is the one added at
 * step i - w, so for the usual windows (w = sr // 10 = 30..32, W > 0) it
 * comes from the add stream's registers of this block or the previous one
 * instead of a second load stream; W = 0 loads it (any window). */
template <int W>
__device__ __forceinline__ void kahan_chain(RollMean &R, const double *__restrict__ y, double *__restrict__ ps,
                                            int64_t S, int64_t off, int64_t w, int64_t nd, int64_t ndmax,
                                            int64_t ndmin, bool run, int64_t last, int64_t ib = 0,
                                            int64_t ie = INT64_MAX) {
    static_assert(W <= PF, "the remove value must lie within the previous block");
    auto ldy = [&](int64_t i) -> double {
        i = i < 0 ? 0 : (i > last ? last : i);
        return fabs(y[i * S]);
    };
    typedef double dv2 __attribute__((ext_vector_type(2)));
    auto put = [&](int64_t i, double v) { ps[(i >> 1) * S * 2 + (i & 1)] = v; };
    /* steps [ib, ie) (ib a multiple of PF): the pass in row chunks, R carried between them */
    ps += (ib >> 1) * S * 2;
    const double *pa = y + (ib + off) * S, *pr = y + (ib + off - w) * S;   /* rows i0 + off, i0 + off - w */
    const int64_t SP = (int64_t)PF * S;
    double ca[PF], na[PF], cp[PF], cr[W == 0 ? PF : 1], nr[W == 0 ? PF : 1];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
        ca[u] = ldy(ib + u + off);
        cp[u] = ldy(ib + u + off - PF);
        if (W == 0) cr[u] = ldy(ib + u + off - w);
    }
    const int64_t iend = ie < ndmax ? ie : ndmax;
    for (int64_t i0 = ib; i0 < iend; i0 += PF, ps += SP, pa += SP, pr += SP) {
        if (i0 + PF + off - w >= 0 && i0 + 2 * PF + off <= ndmin) {
#pragma unroll
            for (int u = 0; u < PF; ++u) {
                na[u] = fabs(pa[SP + u * S]);
                if (W == 0) nr[u] = fabs(pr[SP + u * S]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < PF; ++u) {
                const int64_t i = i0 + PF + u;
                na[u] = ldy(i + off);
                if (W == 0) nr[u] = ldy(i + off - w);
            }
        }
        /* removed value of step i0 + u: |y[i0 + u + off - w]| */
        auto rem = [&](int u) -> double {
            if (W == 0) return cr[u];
            return u >= W ? ca[u - W] : cp[u - W + PF];
        };
        if (i0 >= w - off && i0 + PF + off <= ndmin) {
            /* steady state, no NaN in the wave: pandas remove_mean / add_mean's sum_x updates */
            double sum = R.sum, cad = R.cadd, crm = R.crem;
            double sv[PF];
#pragma unroll
            for (int u = 0; u < PF; ++u) {
                const double yr = -rem(u) - crm, tr = sum + yr;
                crm = (tr - sum) - yr;
                sum = tr;
                const double ya = ca[u] - cad, ta = sum + ya;
                cad = (ta - sum) - ya;
                sum = ta;
                sv[u] = sum;
            }
            if (run) {
#pragma unroll
                for (int u = 0; u < PF; u += 2) *(dv2 *)(ps + (u >> 1) * S * 2) = dv2{sv[u], sv[u + 1]};
            }
            R.sum = sum; R.cadd = cad; R.crem = crm;
        } else {
#pragma unroll
            for (int u = 0; u < PF; ++u) {
                const int64_t i = i0 + u;
                if (run && i < nd) {
                    if (i > 0) {
                        const int64_t s = i + 1 + off - w;
                        if (s > 0 && s <= nd) R.remove(rem(u));
                        if (i + off < nd) R.add(ca[u]);
                    }
                    put(u, R.sum);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            cp[u] = ca[u];
            ca[u] = na[u];
            if (W == 0) cr[u] = nr[u];
        }
    }
}


/* The forward pass alone over rows [fwd_rb, fwd_re) (a multiple of PFB), the
 * DF2T state carried between launches in fwd_z: the host runs it chunk by chunk
 * while k_ref_pick gathers the next chunks on a side stream, so the gather
 * (HBM sector bound, many waves) overlaps the sequential pass (16 waves). */
template <bool ZB>
__global__ __launch_bounds__(64) void k_ref_fwd(EnvRefArgs A) {
    const int lane = threadIdx.x;
    const int f = blockIdx.x * 64 + lane;
    const bool have = f < A.n_files;
    int64_t nd = have ? A.doff[f + 1] - A.doff[f] : 0;
    const bool run = have && nd > 15 && A.active[f];
    if (!run) nd = 0;
    const int64_t S = A.n_files;
    double *__restrict__ scr = A.scratch + (have ? f : 0);
    int64_t ndmax = nd;
    for (int o = 32; o > 0; o >>= 1) { int64_t t = __shfl_xor(ndmax, o); ndmax = t > ndmax ? t : ndmax; }
    if (ndmax == 0) return;
    int64_t ndmin = run ? nd : INT64_MAX;
    for (int o = 32; o > 0; o >>= 1) { int64_t t = __shfl_xor(ndmin, o); ndmin = t < ndmin ? t : ndmin; }
    Df2t D;
    D.b0 = A.b[0]; D.b1 = A.b[1]; D.b2 = A.b[2]; D.b3 = A.b[3]; D.b4 = A.b[4];
    D.a1 = A.a[1]; D.a2 = A.a[2]; D.a3 = A.a[3]; D.a4 = A.a[4];
    const int64_t SB = (int64_t)PFB * S;
    const int64_t nemax = ndmax + 30;
    const int64_t ne = run ? nd + 30 : nemax;
    const int64_t nemin = ndmin == INT64_MAX ? nemax : ndmin + 30;
    const int64_t rb = A.fwd_rb, re = A.fwd_re < nemax ? A.fwd_re : nemax;
    if (rb >= re) return;
    auto ldc = [&](int64_t r) -> double { return scr[(r < ne ? r : ne - 1) * S]; };
    double cur[PFB], nxt[PFB];
#pragma unroll
    for (int u = 0; u < PFB; ++u) cur[u] = ldc(rb + u);
    double *zs = A.fwd_z + (have ? (int64_t)f * 4 : 0);
    if (run) {
        if (rb == 0) D.init(A.zi, cur[0]);
        else { D.z0 = zs[0]; D.z1 = zs[1]; D.z2 = zs[2]; D.z3 = zs[3]; }
    }
    double *p = scr + rb * S;
    for (int64_t r0 = rb; r0 < re; r0 += PFB, p += SB) {
        /* the next block: rows past re may not be gathered yet; they are
         * read but never used (the next launch loads its own first block) */
        if (r0 + 2 * PFB <= nemin) {
#pragma unroll
            for (int u = 0; u < PFB; ++u) nxt[u] = p[SB + u * S];
        } else {
#pragma unroll
            for (int u = 0; u < PFB; ++u) nxt[u] = ldc(r0 + PFB + u);
        }
        if (r0 + PFB <= nemin) {
            if (run) {
#pragma unroll
                for (int u = 0; u < PFB; ++u) p[u * S] = D.step<ZB>(cur[u]);
            }
        } else if (run) {
#pragma unroll
            for (int u = 0; u < PFB; ++u)
                if (r0 + u < ne) p[u * S] = D.step<ZB>(cur[u]);
        }
#pragma unroll
        for (int u = 0; u < PFB; ++u) cur[u] = nxt[u];
    }
    if (run) { zs[0] = D.z0; zs[1] = D.z1; zs[2] = D.z2; zs[3] = D.z3; }
}
template __global__ void k_ref_fwd<false>(EnvRefArgs);
template __global__ void k_ref_fwd<true>(EnvRefArgs);

/* The rolling mean's Kahan recursion over steps [kahan_ib, kahan_ie) of the
 * chain mode, R carried in kahan_z: the pass runs in row chunks so that
 * k_ref_env_mean forms the finished chunks' means on a side stream meanwhile.
 * Waves whose recordings left chain mode (a NaN in |y|) did their whole pass
 * in k_envelope_ref_t. */
__global__ __launch_bounds__(64) void k_ref_kahan(EnvRefArgs A) {
    const int lane = threadIdx.x;
    const int f = blockIdx.x * 64 + lane;
    const bool have = f < A.n_files;
    int64_t nd = have ? A.doff[f + 1] - A.doff[f] : 0;
    const bool run = have && nd > 15 && A.active[f];
    if (!run) nd = 0;
    if (!__ballot(have && A.chain[f])) return;              /* not chain mode, or nothing to run */
    int64_t ndmax = nd;
    for (int o = 32; o > 0; o >>= 1) { int64_t t = __shfl_xor(ndmax, o); ndmax = t > ndmax ? t : ndmax; }
    int64_t ndmin = run ? nd : INT64_MAX;
    for (int o = 32; o > 0; o >>= 1) { int64_t t = __shfl_xor(ndmin, o); ndmin = t < ndmin ? t : ndmin; }
    const int64_t S = A.n_files, w = A.env_window, off = (w - 1) / 2;
    const int64_t last = nd > 0 ? nd - 1 : 0;
    const double *__restrict__ y = A.scratch + (have ? f : 0) + 15 * S;
    double *__restrict__ ps = A.sums + (have ? (int64_t)f * 2 : 0);
    RollMean R;
    if (have) R.load(A.kahan_z + (int64_t)f * 6);
    const int64_t ib = A.kahan_ib, ie = A.kahan_ie;
    switch (w) {
    case 30: kahan_chain<30>(R, y, ps, S, off, w, nd, ndmax, ndmin, run, last, ib, ie); break;
    case 31: kahan_chain<31>(R, y, ps, S, off, w, nd, ndmax, ndmin, run, last, ib, ie); break;
    case 32: kahan_chain<32>(R, y, ps, S, off, w, nd, ndmax, ndmin, run, last, ib, ie); break;
    default: kahan_chain<0>(R, y, ps, S, off, w, nd, ndmax, ndmin, run, last, ib, ie); break;
    }
    if (have) R.save(A.kahan_z + (int64_t)f * 6);
}

template <int DT, bool MULTI, bool ZB>
__global__ __launch_bounds__(64) void k_envelope_ref_t(EnvRefArgs A) {
    __shared__ double st_env[STG][65];
    __shared__ double st_y[STG][65];
    const int lane = threadIdx.x;
    const int f = blockIdx.x * 64 + lane;
    const bool have = f < A.n_files;
    int64_t nd = have ? A.doff[f + 1] - A.doff[f] : 0;
    const bool run = have && nd > 15 && A.active[f];
    if (!run) nd = 0;
    const int64_t d0 = have ? A.doff[f] : 0;
    const int64_t S = A.n_files;
    double *__restrict__ scr = A.scratch + (have ? f : 0);
    /* wave-uniform trip counts (ragged files: lanes past their end are masked) */
    int64_t ndmax = nd;
    for (int o = 32; o > 0; o >>= 1) { int64_t t = __shfl_xor(ndmax, o); ndmax = t > ndmax ? t : ndmax; }
    if (have && A.chain) A.chain[f] = 0;
    if (ndmax == 0) return;
    /* shortest running file of the wave: blocks below it need no per-step
     * predicate, so a block's steps form one basic block the scheduler can
     * interleave (the x-only products of later steps fill the latency of the
     * y-dependent chain) */
    int64_t ndmin = run ? nd : INT64_MAX;
    for (int o = 32; o > 0; o >>= 1) { int64_t t = __shfl_xor(ndmin, o); ndmin = t < ndmin ? t : ndmin; }

    Df2t D;
    D.b0 = A.b[0]; D.b1 = A.b[1]; D.b2 = A.b[2]; D.b3 = A.b[3]; D.b4 = A.b[4];
    D.a1 = A.a[1]; D.a2 = A.a[2]; D.a3 = A.a[3]; D.a4 = A.a[4];
    const int64_t last = nd > 0 ? nd - 1 : 0;
    STAMP_DECL

    /* Row addresses: every lane walks its own column with a pointer that
     * advances by PFB rows per block; inside blocks that no lane can run past
     * (the common case) the offsets u * S are loop-invariant, so a load or a
     * store is one instruction with no clamping or 64-bit index arithmetic. */
    const int64_t SB = (int64_t)PFB * S;
    const int64_t nemax = ndmax + 30;
    /* lanes that do not run address a full-length column (they only load, never store) */
    const int64_t ne = run ? nd + 30 : nemax;
    const int64_t nemin = ndmin == INT64_MAX ? nemax : ndmin + 30;   /* shortest running column */
    /* ---------------- forward pass, in place over the gathered rows ---------------- */
    if (!A.fwd_z) {                                          /* else k_ref_fwd ran it in row chunks */
        auto ldc = [&](int64_t r) -> double { return scr[(r < ne ? r : ne - 1) * S]; };   /* clamped */
        double cur[PFB], nxt[PFB];
#pragma unroll
        for (int u = 0; u < PFB; ++u) cur[u] = ldc(u);
        if (run) D.init(A.zi, cur[0]);
        double *p = scr;                                     /* row r0 */
        for (int64_t r0 = 0; r0 < nemax; r0 += PFB, p += SB) {
            if (r0 + 2 * PFB <= nemin) {
#pragma unroll
                for (int u = 0; u < PFB; ++u) nxt[u] = p[SB + u * S];
            } else {
#pragma unroll
                for (int u = 0; u < PFB; ++u) nxt[u] = ldc(r0 + PFB + u);
            }
            if (r0 + PFB <= nemin) {
                if (run) {
#pragma unroll
                    for (int u = 0; u < PFB; ++u) p[u * S] = D.step<ZB>(cur[u]);
                }
            } else if (run) {
#pragma unroll
                for (int u = 0; u < PFB; ++u)
                    if (r0 + u < ne) p[u * S] = D.step<ZB>(cur[u]);
            }
#pragma unroll
            for (int u = 0; u < PFB; ++u) cur[u] = nxt[u];
        }
    }
    STAMP(0);
    /* ---------------- backward pass, in place ---------------- */
    bool nanseen = false;
    {
        /* reversed index r -> row ne - 1 - r (clamped at 0 past the column's start) */
        auto ldc = [&](int64_t r) -> double {
            int64_t row = ne - 1 - r;
            row = row < 0 ? 0 : row;
            return scr[row * S];
        };
        double cur[PFB], nxt[PFB];
#pragma unroll
        for (int u = 0; u < PFB; ++u) cur[u] = ldc(u);
        if (run) D.init(A.zi, cur[0]);
        double *p = scr + (ne - 1) * S;                      /* row ne - 1 - r0 */
        for (int64_t r0 = 0; r0 < nemax; r0 += PFB, p -= SB) {
            if (r0 + 2 * PFB <= nemin) {
#pragma unroll
                for (int u = 0; u < PFB; ++u) nxt[u] = p[-SB - u * S];
            } else {
#pragma unroll
                for (int u = 0; u < PFB; ++u) nxt[u] = ldc(r0 + PFB + u);
            }
            if (r0 + PFB <= nemin) {
                if (run) {
#pragma unroll
                    for (int u = 0; u < PFB; ++u) {
                        const double yv = D.step<ZB>(cur[u]);
                        nanseen |= yv != yv;
                        p[-u * S] = yv;
                    }
                }
            } else if (run) {
#pragma unroll
                for (int u = 0; u < PFB; ++u)
                    if (r0 + u < ne) {
                        const double yv = D.step<ZB>(cur[u]);
                        nanseen |= yv != yv;
                        p[-u * S] = yv;
                    }
            }
#pragma unroll
            for (int u = 0; u < PFB; ++u) cur[u] = nxt[u];
        }
    }
    STAMP(1);
    /* ---------------- |y| centred rolling mean over rows [15, 15+nd) ---------------- */
    {
        const double *__restrict__ y = scr + 15 * S;
        const int64_t w = A.env_window;
        const int64_t off = (w - 1) / 2;
        double *__restrict__ env = A.env;
        double *__restrict__ yout = A.y;
        auto ldy = [&](int64_t i) -> double {
            i = i < 0 ? 0 : (i > last ? last : i);
            return fabs(y[i * S]);
        };
        RollMean R;
        /* i = 0: setup window [0, e0) */
        const int64_t e0 = (1 + off) < nd ? (1 + off) : nd;
        if (run) {
            R.prev = ldy(0);
            for (int64_t j = 0; j < e0; ++j) R.add(ldy(j));
        }
        const bool chain = A.sums && w > 1 && !__ballot(nanseen);   /* wave-uniform */
        if (have && A.chain) A.chain[f] = chain && run ? 1 : 0;
        if (chain) {
            /* only the Kahan recursion; k_ref_env_mean forms the means */
            double *__restrict__ ps = A.sums + (have ? (int64_t)f * 2 : 0);   /* pair rows [i / 2][file][2] */
            const int64_t ie = A.kahan_z ? A.kahan_ie : INT64_MAX;   /* chunked: the first chunk here */
            switch (w) {
            case 30: kahan_chain<30>(R, y, ps, S, off, w, nd, ndmax, ndmin, run, last, 0, ie); break;
            case 31: kahan_chain<31>(R, y, ps, S, off, w, nd, ndmax, ndmin, run, last, 0, ie); break;
            case 32: kahan_chain<32>(R, y, ps, S, off, w, nd, ndmax, ndmin, run, last, 0, ie); break;
            default: kahan_chain<0>(R, y, ps, S, off, w, nd, ndmax, ndmin, run, last, 0, ie); break;
            }
            if (A.kahan_z && have) R.save(A.kahan_z + (int64_t)f * 6);
            STAMP(2);
            STAMP_FLUSH(A.stamps);
            return;
        }
        double ca[PF], cr[PF], na[PF], nr[PF], cy[PF], ny[PF];
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            ca[u] = ldy(u + off); cr[u] = ldy(u + off - w);
            cy[u] = yout ? y[(u < last ? u : last) * S] : 0.0;
        }
        for (int64_t i0 = 0; i0 < ndmax; i0 += PF) {
#pragma unroll
            for (int u = 0; u < PF; ++u) {
                const int64_t i = i0 + PF + u;
                na[u] = ldy(i + off);
                nr[u] = ldy(i + off - w);
                if (yout) ny[u] = y[(i < last ? i : last) * S];
            }
            if (w > 1 && i0 >= w - off && i0 + PF + off <= ndmin) {
                /* every running lane removes and adds one sample per step here
                 * (lanes that do not run compute values nobody stores) */
#pragma unroll
                for (int u = 0; u < PF; ++u) {
                    R.remove_sel(cr[u]);
                    R.add_sel(ca[u]);
                    st_env[(i0 + u) & (STG - 1)][lane] = R.mean_sel();
                    st_y[(i0 + u) & (STG - 1)][lane] = cy[u];      /* flushed only when yout */
                }
            } else
#pragma unroll
            for (int u = 0; u < PF; ++u) {
                const int64_t i = i0 + u;
                double ev = 0.0;
                if (run && i < nd) {
                    if (w == 1) {
                        R = RollMean();
                        R.prev = ca[u];
                        R.add(ca[u]);
                    } else if (i > 0) {
                        const int64_t s = i + 1 + off - w;      /* unclipped start; remove when it advances */
                        if (s > 0 && s <= nd) R.remove(cr[u]);
                        if (i + off < nd) R.add(ca[u]);
                    }
                    ev = R.mean();
                }
                st_env[(i0 + u) & (STG - 1)][lane] = ev;
                if (yout) st_y[(i0 + u) & (STG - 1)][lane] = cy[u];
            }
            if (((i0 + PF) & (STG - 1)) == 0 || i0 + PF >= ndmax) {
                const int64_t base = (i0 + PF - 1) & ~(int64_t)(STG - 1);
                const int rows = (int)(i0 + PF - base);
                __syncthreads();
                flush_rows(st_env, env, base, rows, d0, nd);
                if (yout) flush_rows(st_y, yout, base, rows, d0, nd);
                __syncthreads();
            }
#pragma unroll
            for (int u = 0; u < PF; ++u) { ca[u] = na[u]; cr[u] = nr[u]; cy[u] = ny[u]; }
        }
    }
}

/* chain mode's outputs: env[i] = calc_mean(minp 1, nobs, neg, sum_x, same,
 * prev) for every (recording, step) in parallel.  In chain mode |y| has no
 * NaN, so nobs is the clipped window length and neg is 0 (|y| never has its
 * sign bit set); the last added value is |y[min(i + off, n - 1)]| and the run
 * of equal added values ending there is counted back (it only matters up to
 * nobs).  A tile of 64 steps x 64 recordings, transposed through LDS so the
 * stores are contiguous; the y output (when requested) rides along. */
template <bool WANT_Y>
__global__ __launch_bounds__(256) void k_ref_env_mean(EnvRefArgs A) {
    /* without the y output the staging is half the LDS: four workgroups per CU */
    __shared__ double st_env[STG][65];
    __shared__ double st_y[WANT_Y ? STG : 1][65];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int f = blockIdx.y * 64 + lane;
    const bool have = f < A.n_files;
    const bool mine = have && A.chain[f];
    const int64_t nd = have ? A.doff[f + 1] - A.doff[f] : 0;
    const int64_t d0 = have ? A.doff[f] : 0;
    const int64_t S = A.n_files, w = A.env_window, off = (w - 1) / 2;
    const int64_t i00 = A.mean_r0 + (int64_t)blockIdx.x * STG;
    if (!__syncthreads_or(mine && i00 < nd)) return;
    const double *__restrict__ y = A.scratch + 15 * S + (have ? f : 0);
    const double *__restrict__ sums = A.sums + (have ? (int64_t)f * 2 : 0);     /* pair rows [i / 2][file][2] */
    /* this wave's 16 rows: every load issued first, then the arithmetic */
    constexpr int R = STG / 4;
    const int64_t ib = i00 + wv * R;
    const int64_t lastr = nd > 0 ? nd - 1 : 0;
    double sm[R], ya[R], yb[R], yi[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t i = ib + r;
        const bool ok = mine && i < nd;
        const int64_t ic = ok ? i : 0;
        const int64_t a = ic + off < lastr ? ic + off : lastr;            /* last added index */
        sm[r] = ok ? sums[(ic >> 1) * S * 2 + (ic & 1)] : 0.0;
        ya[r] = ok ? y[a * S] : 0.0;
        yb[r] = ok && a > 0 ? y[(a - 1) * S] : 0.0;
        yi[r] = WANT_Y && ok ? y[ic * S] : 0.0;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t i = ib + r;
        double ev = 0.0;
        if (mine && i < nd) {
            int64_t s, e;
            win_bounds(i, nd, w, s, e);
            const int64_t nobs = e - s;
            const int64_t a = i + off < lastr ? i + off : lastr;
            const double prev = fabs(ya[r]);
            int64_t same = 1;
            if (a > 0 && same < nobs && fabs(yb[r]) == prev) {   /* rare: a run of equal values */
                ++same;
                for (int64_t j = a - 2; j >= 0 && same < nobs && fabs(y[j * S]) == prev; --j) ++same;
            }
            double res = sm[r] / (double)nobs;
            if (same >= nobs) res = prev;
            else if (res < 0) res = 0.0;                 /* neg_ct == 0 and result < 0 */
            ev = nobs >= 1 ? res : __builtin_nan("");
        }
        st_env[wv * R + r][lane] = ev;
        if (WANT_Y) st_y[wv * R + r][lane] = yi[r];
    }
    __syncthreads();
    for (int fl = wv; fl < 64; fl += 4) {
        if (!__shfl((int)mine, fl)) continue;
        const int64_t fd0 = __shfl(d0, fl), fnd = __shfl(nd, fl);
        const int64_t i = i00 + lane;
        if (i < fnd) {
            A.env[fd0 + i] = st_env[lane][fl];
            if (WANT_Y) A.y[fd0 + i] = st_y[lane][fl];
        }
    }
}

template __global__ void k_ref_env_mean<true>(EnvRefArgs);
template __global__ void k_ref_env_mean<false>(EnvRefArgs);
template __global__ void k_ref_pick<BPMX_DT_U8, false>(EnvRefArgs);
template __global__ void k_ref_pick<BPMX_DT_I16, false>(EnvRefArgs);
template __global__ void k_ref_pick<BPMX_DT_I32, false>(EnvRefArgs);
template __global__ void k_ref_pick<BPMX_DT_F32, false>(EnvRefArgs);
template __global__ void k_ref_pick<BPMX_DT_F64, false>(EnvRefArgs);
template __global__ void k_ref_pick<BPMX_DT_U8, true>(EnvRefArgs);
template __global__ void k_ref_pick<BPMX_DT_I16, true>(EnvRefArgs);
template __global__ void k_ref_pick<BPMX_DT_I32, true>(EnvRefArgs);
template __global__ void k_ref_pick<BPMX_DT_F32, true>(EnvRefArgs);
template __global__ void k_ref_pick<BPMX_DT_F64, true>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_U8, false, false>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_U8, true, false>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_I16, false, false>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_I16, true, false>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_I32, false, false>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_I32, true, false>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_F32, false, false>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_F32, true, false>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_F64, false, false>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_F64, true, false>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_U8, false, true>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_U8, true, true>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_I16, false, true>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_I16, true, true>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_I32, false, true>(EnvRefArgs);
template __global__ void k_envelope_ref_t<BPMX_DT_I32, true, true>(EnvRefArgs);

}  // namespace bpmx
