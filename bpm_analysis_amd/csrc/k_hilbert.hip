/*
 * k_hilbert.hip — native-mode envelope after the filter, fused in LDS:
 *   env = centred rolling mean (window sr//10) of |scipy.signal.hilbert(yd)|
 * oracle: scipy/signal/_signaltools.py:2318 (hilbert: ifft(fft(x) * h),
 * h = 1, 2, ..., 2, 1, 0, ...), oracle/oracle.py hilbert_abs + rolling_mean.
 *
 * One workgroup per recording; the recording's whole transform stays in LDS.
 * The real signal y (Nd = N = 2M samples) is read as M complex points
 * z_m = y_2m + i y_2m+1 (its natural memory layout), then
 *   1. forward mixed-radix DIF over M: natural order in, digit-reversed out,
 *      in place (no permutation pass);
 *   2. one pointwise pass over the pairs (k, M - k) turns Z = DFT_M(z) into
 *      X_k = conj(w) S - w D  (w = e^(-2 pi i k / N), S = Z_k + conj(Z_(M-k)),
 *      D = Z_k - conj(Z_(M-k)), X_0 = 0): the half-length spectrum whose
 *      inverse DFT is c_2m + i c_2m+1, with c = N * Im(analytic signal) — the
 *      "-i on the positive half spectrum, zero DC and Nyquist" of hilbert,
 *      folded together with the real-FFT split and merge;
 *   3. inverse mixed-radix DIT: digit-reversed in, natural order out;
 *   4. |analytic| = sqrt(y^2 + (c/N)^2) in place, then the rolling mean.
 * Radix 2 butterflies are plain; odd primes p use the pair-symmetric direct
 * DFT X_k = x_0 + sum_n (x_n + x_(p-n)) cos(2 pi n k/p) -/+ i (x_n - x_(p-n))
 * sin(2 pi n k/p) (a quarter of the multiplies of the plain DFT), with the
 * cos/sin advanced by rotation and re-seeded from the exact table every 16
 * steps.  Twiddles W_N^e = hi[e >> 7] * lo[e & 127] (tables in LDS).
 * Recordings whose M does not factor into primes <= HB_PMAX or does not fit
 * in LDS take the rocFFT path (k_envelope_native.hip).
 */
#include "bpmx_common.h"
#include "bpmx_hilbert.h"
#include "bpmx_qsel.h"
#include "bpmx_stamps.h"
#include "bpmx_dft_consts.h"

namespace bpmx {

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(__builtin_fma(a.x, b.x, -a.y * b.y), __builtin_fma(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ double2 cmulc(double2 a, double2 b) {          /* a * conj(b) */
    return make_double2(__builtin_fma(a.x, b.x, a.y * b.y), __builtin_fma(a.y, b.x, -a.x * b.y));
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }

struct HbLds {
    double2 *x, *twh, *twl, *pt;
    __device__ __forceinline__ double2 tw(int e) const { return cmul(twh[e >> 7], twl[e & 127]); }   /* W_N^e */
};

/* radix-2 stage: DIF (twiddle after) or DIT inverse (conjugate twiddle before) */
template <bool INV>
__device__ __forceinline__ void hb_radix2(const HbLds &S, const HilbPlan &P, int si) {
    const int M = P.M, B = P.B[si], L = P.L[si];
    const uint64_t dL = P.dL[si];
    const int nb = M / 2, step = P.N / B;
    for (int t = threadIdx.x; t < nb; t += HB_T) {
        const int blk = hb_div(t, dL), n2 = t - blk * L, base = blk * B + n2;
        double2 a = S.x[base], b = S.x[base + L];
        if (!INV) {
            const double2 d = csub(a, b);
            S.x[base] = cadd(a, b);
            S.x[base + L] = n2 ? cmul(d, S.tw(step * n2)) : d;
        } else {
            if (n2) b = cmulc(b, S.tw(step * n2));
            S.x[base] = cadd(a, b);
            S.x[base + L] = csub(a, b);
        }
    }
    __syncthreads();
}

/* odd prime radix p, pair-symmetric direct DFT */
template <bool INV>
__device__ __forceinline__ void hb_radixp(const HbLds &S, const HilbPlan &P, int si, const double2 *ct) {
    const int M = P.M, B = P.B[si], L = P.L[si], p = P.rad[si];
    const uint64_t dL = P.dL[si], dP = P.dP[si], dH = P.dH[si], dG = P.dG[si];
    const int h = (p - 1) >> 1, nbf = M / p, step = P.N / B;
    /* pre-pass: (DIT: conjugate twiddles, then) x_n, x_(p-n) -> a_n = x_n + x_(p-n), b_n = x_n - x_(p-n) */
    for (int t = threadIdx.x; t < nbf * h; t += HB_T) {
        const int bf = hb_div(t, dH), n = t - bf * h + 1;
        const int blk = hb_div(bf, dL), n2 = bf - blk * L, base = blk * B + n2;
        double2 u = S.x[base + n * L], v = S.x[base + (p - n) * L];
        if (INV && n2) {
            u = cmulc(u, S.tw(step * n2 * n));
            v = cmulc(v, S.tw(step * n2 * (p - n)));
        }
        S.x[base + n * L] = cadd(u, v);
        S.x[base + (p - n) * L] = csub(u, v);
    }
    __syncthreads();
    /* Outputs k and p - k of every butterfly, HB_KB consecutive k per task so
     * one pair of LDS reads (a_n, b_n) feeds HB_KB frequencies; kept in
     * registers until every task of the stage has read its inputs.  cos and
     * sin of n k (2 pi / p) advance by the two-term recurrence
     * c_(n+1) = 2 cos(k 2pi/p) c_n - c_(n-1) (one FMA each), re-seeded from
     * the exact table every 16 steps. */
    const int ng = (h + HB_KB) / HB_KB;                       /* k groups: k = 0 .. h */
    const int ntask = nbf * ng;
    double2 r0[HB_MAXT][HB_KB], r1[HB_MAXT][HB_KB];
#pragma unroll
    for (int i = 0; i < HB_MAXT; ++i) {
        const int t = threadIdx.x + i * HB_T;
        if (t < ntask) {
            const int bf = hb_div(t, dG), k0 = (t - bf * ng) * HB_KB;
            const int blk = hb_div(bf, dL), n2 = bf - blk * L, base = blk * B + n2;
            const double2 x0 = S.x[base];
            double ax[HB_KB], ay[HB_KB], bx[HB_KB], by[HB_KB], c[HB_KB], cp[HB_KB], sn[HB_KB], sp[HB_KB], c2[HB_KB];
            int idx[HB_KB];
#pragma unroll
            for (int j = 0; j < HB_KB; ++j) {
                ax[j] = ay[j] = bx[j] = by[j] = 0.0;
                c[j] = sn[j] = cp[j] = sp[j] = 0.0;
                idx[j] = 0;
                const int k = k0 + j <= h ? k0 + j : 0;
                c2[j] = 2.0 * ct[k].x;
            }
            for (int n0 = 1; n0 <= h; n0 += 16) {
                /* seed: (c, s) at n0 - 1 and n0 for every k of the group */
#pragma unroll
                for (int j = 0; j < HB_KB; ++j) {
                    const int k = k0 + j <= h ? k0 + j : 0;
                    int i1 = idx[j] + k;                           /* (n0 k) mod p; idx = ((n0 - 1) k) mod p */
                    if (i1 >= p) i1 -= p;
                    const double2 e0 = ct[idx[j]], e1 = ct[i1];
                    cp[j] = e0.x; sp[j] = e0.y; c[j] = e1.x; sn[j] = e1.y;
                    int i16 = i1 + 15 * k;                         /* ((n0 + 15) k) mod p */
                    i16 -= hb_div(i16, dP) * p;
                    idx[j] = i16;
                }
                const int n1 = n0 + 16 <= h + 1 ? n0 + 16 : h + 1;
                /* two steps per trip: the recurrence alternates between (c, cp)
                 * and (cp, c), so no register rotation moves */
                int n = n0;
                for (; n + 1 < n1; n += 2) {
                    const double2 a0 = S.x[base + n * L], b0 = S.x[base + (p - n) * L];
                    const double2 a1 = S.x[base + (n + 1) * L], b1 = S.x[base + (p - n - 1) * L];
#pragma unroll
                    for (int j = 0; j < HB_KB; ++j) {
                        ax[j] = __builtin_fma(a0.x, c[j], ax[j]); ay[j] = __builtin_fma(a0.y, c[j], ay[j]);
                        bx[j] = __builtin_fma(b0.x, sn[j], bx[j]); by[j] = __builtin_fma(b0.y, sn[j], by[j]);
                        cp[j] = __builtin_fma(c2[j], c[j], -cp[j]);       /* cos (n+1) k */
                        sp[j] = __builtin_fma(c2[j], sn[j], -sp[j]);
                        ax[j] = __builtin_fma(a1.x, cp[j], ax[j]); ay[j] = __builtin_fma(a1.y, cp[j], ay[j]);
                        bx[j] = __builtin_fma(b1.x, sp[j], bx[j]); by[j] = __builtin_fma(b1.y, sp[j], by[j]);
                        c[j] = __builtin_fma(c2[j], cp[j], -c[j]);        /* cos (n+2) k */
                        sn[j] = __builtin_fma(c2[j], sp[j], -sn[j]);
                    }
                }
                if (n < n1) {
                    const double2 a0 = S.x[base + n * L], b0 = S.x[base + (p - n) * L];
#pragma unroll
                    for (int j = 0; j < HB_KB; ++j) {
                        ax[j] = __builtin_fma(a0.x, c[j], ax[j]); ay[j] = __builtin_fma(a0.y, c[j], ay[j]);
                        bx[j] = __builtin_fma(b0.x, sn[j], bx[j]); by[j] = __builtin_fma(b0.y, sn[j], by[j]);
                    }
                }
            }
            /* forward: X_k = x0 + A - iB, X_(p-k) = x0 + A + iB; inverse: signs swapped */
#pragma unroll
            for (int j = 0; j < HB_KB; ++j) {
                const double2 xa = make_double2(x0.x + ax[j], x0.y + ay[j]);
                const double2 mib = INV ? make_double2(-by[j], bx[j]) : make_double2(by[j], -bx[j]);   /* -+ iB */
                r0[i][j] = cadd(xa, mib);
                r1[i][j] = csub(xa, mib);
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < HB_MAXT; ++i) {
        const int t = threadIdx.x + i * HB_T;
        if (t < ntask) {
            const int bf = hb_div(t, dG), k0 = (t - bf * ng) * HB_KB;
            const int blk = hb_div(bf, dL), n2 = bf - blk * L, base = blk * B + n2;
#pragma unroll
            for (int j = 0; j < HB_KB; ++j) {
                const int k = k0 + j;
                if (k > h) break;
                if (!INV && n2) {
                    S.x[base + k * L] = k ? cmul(r0[i][j], S.tw(step * n2 * k)) : r0[i][j];
                    if (k) S.x[base + (p - k) * L] = cmul(r1[i][j], S.tw(step * n2 * (p - k)));
                } else {
                    S.x[base + k * L] = r0[i][j];
                    if (k) S.x[base + (p - k) * L] = r1[i][j];
                }
            }
        }
    }
    __syncthreads();
}

/* Small odd-prime stages (p <= 29, hb_cp_off(p) >= 0) from exact constants
 * (bpmx_dft_consts.h: correctly rounded cos / sin, laid out per frequency
 * group and n in constant memory, so each step's row comes by scalar loads):
 * no recurrence, no separate (a_n, b_n) pass.  Frequencies k = 0 .. h split
 * into ng = ceil((h + 1) / HB_CP_G) groups; a wave takes one group
 * (wave-uniform) for 64 butterflies, each lane one butterfly: per n it reads
 * x_n, x_(p-n) (with the DIT's conjugate twiddles first), forms a_n, b_n in
 * registers and accumulates A_k = sum a_n cos(2 pi n k / p),
 * B_k = sum b_n sin(2 pi n k / p) over the group's k.  Results wait in
 * registers for the barrier, then go back in place (with the DIF's
 * twiddles).  One round of waves: the plan takes this form only when
 * ng ceil((M / p) / 64) <= HB_T / 64. */
#ifndef HB_CP_UNROLL
#define HB_CP_UNROLL 2   /* (r06 tools/hbench: 1 -> 2 made the radix-23 stage 20.2 K -> 19.7 K cycles) */
#endif
__host__ __device__ constexpr int hb_cp_ng(int p) { return ((p + 1) / 2 + HB_CP_G - 1) / HB_CP_G; }

template <bool INV>
__device__ __forceinline__ void hb_radixp_const(const HbLds &S, const HilbPlan &PL, int si) {
    constexpr int G = HB_CP_G;
    const int M = PL.M, B = PL.B[si], L = PL.L[si], p = PL.rad[si], h = (p - 1) >> 1;
    const uint64_t dL = PL.dL[si];
    const int nbf = hb_div(M, PL.dP[si]), step = PL.N / B, nbw = (nbf + 63) >> 6;
    const int wv = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    const int g = __builtin_amdgcn_readfirstlane(wv / nbw);                 /* wave-uniform group */
    const int bf = (wv - g * nbw) * 64 + lane;
    const bool act = g < PL.cp[si] && bf < nbf;                           /* cp[si] = ng */
    double2 r0[G], r1[G];
    int base = 0, n2 = 0;
    if (act) {
        const int blk = hb_div(bf, dL);
        n2 = bf - blk * L;
        base = blk * B + n2;
        double ax[G], ay[G], bx[G], by[G];
#pragma unroll
        for (int j = 0; j < G; ++j) ax[j] = ay[j] = bx[j] = by[j] = 0.0;
        const double *row = HB_CP + PL.cpo[si] + g * (h * 2 * G);
        /* the DIT's input twiddles w^(e n) and w^(e (p - n)), e = step n2, by
         * products from two table values: t_n = t_(n-1) w^e, t_(p-n) =
         * w^(e p) conj(t_n) (lanes' table indices step n2 k are strided, so
         * every per-output table read was a bank-conflicted pair of LDS reads) */
        const double2 w1 = (INV && n2) ? S.tw(step * n2) : make_double2(1.0, 0.0);
        const double2 wp = (INV && n2) ? S.tw(step * n2 * p) : make_double2(1.0, 0.0);
        double2 tn = w1;
#pragma unroll HB_CP_UNROLL
        for (int n = 1; n <= h; ++n, row += 2 * G) {
            double2 u = S.x[base + n * L], v = S.x[base + (p - n) * L];
            if (INV && n2) {
                u = cmulc(u, tn);
                v = cmulc(v, cmulc(wp, tn));
                tn = cmul(tn, w1);
            }
            const double2 a = cadd(u, v), b = csub(u, v);
#ifdef HB_CP_NOFMA                                           /* tools/hbench timing diagnostic (wrong outputs) */
            ax[0] += a.x + row[0]; ay[0] += a.y; bx[0] += b.x; by[0] += b.y;
            if (false)
#endif
#pragma unroll
            for (int j = 0; j < G; ++j) {
#ifdef HB_CP_NOROW                                            /* tools/hbench timing diagnostic (wrong outputs) */
                const double c = 0.5 + j, sn = 0.25 - j;
#else
                const double c = row[j], sn = row[G + j];
#endif
                ax[j] = __builtin_fma(a.x, c, ax[j]);
                ay[j] = __builtin_fma(a.y, c, ay[j]);
                bx[j] = __builtin_fma(b.x, sn, bx[j]);
                by[j] = __builtin_fma(b.y, sn, by[j]);
            }
        }
        const double2 x0 = S.x[base];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            /* forward: X_k = x0 + A - iB, X_(p-k) = x0 + A + iB; inverse: signs swapped */
            const double2 xa = make_double2(x0.x + ax[j], x0.y + ay[j]);
            const double2 mib = INV ? make_double2(-by[j], bx[j]) : make_double2(by[j], -bx[j]);
            r0[j] = cadd(xa, mib);
            r1[j] = csub(xa, mib);
        }
    }
    /* the DIF's output twiddles likewise: t_k from w^(e k0) by products with
     * w^e, t_(p-k) = w^(e p) conj(t_k) */
    double2 w1 = make_double2(1.0, 0.0), wp = w1, tk = w1;
    if (!INV && act && n2) {
        w1 = S.tw(step * n2);
        wp = S.tw(step * n2 * p);
        tk = S.tw(step * n2 * g * G);
    }
    __syncthreads();
#ifdef HB_CP_NOWRITE                                          /* tools/hbench timing diagnostic (wrong outputs) */
    if (act && r0[0].x == 1.2345e300) S.x[base] = r1[G - 1];
    if (false)
#endif
    if (act) {
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int k = g * G + j;
            if (k > h) break;
            if (!INV && n2) {
                S.x[base + k * L] = k ? cmul(r0[j], tk) : r0[j];
                if (k) S.x[base + (p - k) * L] = cmul(r1[j], cmulc(wp, tk));
                tk = cmul(tk, w1);
            } else {
                S.x[base + k * L] = r0[j];
                if (k) S.x[base + (p - k) * L] = r1[j];
            }
        }
    }
    __syncthreads();
}

/* The same odd-prime stage as a GEMM on the matrix cores: nbf = M / p
 * butterflies, butterfly (blk, n2) holding x_n at blk B + n2 + n L.  After the
 * (a_n, b_n) pre-pass (with the DIT's conjugate twiddles first) the
 * pair-symmetric DFT is four real products over n = 1..h:
 *   Are = sum a_n.re c_nk,  Aim = sum a_n.im c_nk,  Bre = sum b_n.re s_nk,  Bim = sum b_n.im s_nk
 * with c_nk, s_nk = cos, sin(2 pi (n k mod p) / p) from the exact table, i.e.
 * [butterflies x n] x [n x k] GEMMs: v_mfma_f64_16x16x4_f64 (A: lane l = row
 * l & 15, k-index l >> 4; B: k-index l >> 4, column l & 15; D: column l & 15,
 * row (l >> 4) + 4 reg).  One 16-B LDS read each of a_n, b_n and (c, s) feeds
 * the four MFMAs of a K step.  A wave owns HB_MF_UNITS (16 butterflies x 16
 * frequencies) output tiles; results stay in registers until every wave has
 * read, then the DIF twiddles are applied on the way out. */
typedef double hb_d4 __attribute__((ext_vector_type(4)));
template <bool INV, bool CONTIG>
__device__ __forceinline__ void hb_radixp_mfma(const HbLds &S, const HilbPlan &P, int si, const double2 *ct) {
    const int M = P.M, B = P.B[si], p = P.rad[si];
    const int L = CONTIG ? 1 : P.L[si];                        /* contiguous stage: no index divisions */
    const uint64_t dL = P.dL[si], dP = P.dP[si], dH = P.dH[si], dT = P.dT[si];
    const int h = (p - 1) >> 1, nbf = M / p, step = P.N / B;
    for (int t = threadIdx.x; t < nbf * h; t += HB_T) {
        const int bf = hb_div(t, dH), n = t - bf * h + 1;
        const int blk = CONTIG ? bf : hb_div(bf, dL), n2 = CONTIG ? 0 : bf - blk * L, base = CONTIG ? bf * p : blk * B + n2;
        double2 u = S.x[base + n * L], v = S.x[base + (p - n) * L];
        if (INV && n2) {
            u = cmulc(u, S.tw(step * n2 * n));
            v = cmulc(v, S.tw(step * n2 * (p - n)));
        }
        S.x[base + n * L] = cadd(u, v);
        S.x[base + (p - n) * L] = csub(u, v);
    }
    __syncthreads();
    const int ntl = (h + 16) >> 4, ks = (h + 3) >> 2, units = ((nbf + 15) >> 4) * ntl;
    /* thread-derived values recomputed here from an opaque copy: hoisted to
     * the kernel's entry they stayed live across every stage and spilled */
    int tx = (int)threadIdx.x;
    asm volatile("" : "+v"(tx));
    const int lane = tx & 63, wv = __builtin_amdgcn_readfirstlane(tx >> 6), r16 = lane & 15, kq = lane >> 4;
    auto base_of = [&](int bf) {
        if (CONTIG) return bf * p;
        const int blk = hb_div(bf, dL);
        return blk * B + (bf - blk * L);
    };
    hb_d4 acc[HB_MF_UNITS][4];
    double2 x0[HB_MF_UNITS][4];
#pragma unroll
    for (int u = 0; u < HB_MF_UNITS; ++u) {
        const int unit = wv + u * (HB_T / 64);
        if (unit < units) {                                    /* wave-uniform */
            const int m = hb_div(unit, dT), nt = unit - m * ntl;
            const int dA = 16 * m + r16, kB = 16 * nt + r16;
            const bool rowok = dA < nbf;
            const double2 *xa = S.x + base_of(rowok ? dA : 0);
            hb_d4 c0 = {0.0, 0.0, 0.0, 0.0}, c1 = c0, c2 = c0, c3 = c0;
            int idx = (kq + 1) * kB;                           /* (n k) mod p, n = 4 s + kq + 1 */
            idx -= hb_div(idx, dP) * p;
            const int st4 = 4 * kB - hb_div(4 * kB, dP) * p;
            for (int s = 0; s < ks; ++s) {
                const int n = 4 * s + kq + 1;
                const bool ok = rowok && n <= h;
                const double2 a = ok ? xa[n * L] : make_double2(0.0, 0.0);
                const double2 b = ok ? xa[(p - n) * L] : make_double2(0.0, 0.0);
                const double2 cs = ct[idx];
                c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, cs.x, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, cs.x, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(b.x, cs.y, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b.y, cs.y, c3, 0, 0, 0);
                idx += st4;
                if (idx >= p) idx -= p;
            }
            acc[u][0] = c0; acc[u][1] = c1; acc[u][2] = c2; acc[u][3] = c3;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int d = 16 * m + kq + 4 * r;
                x0[u][r] = d < nbf ? S.x[base_of(d)] : make_double2(0.0, 0.0);
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < HB_MF_UNITS; ++u) {
        const int unit = wv + u * (HB_T / 64);
        if (unit < units) {
            const int m = hb_div(unit, dT), nt = unit - m * ntl, k = 16 * nt + r16;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int d = 16 * m + kq + 4 * r;
                if (d < nbf && k <= h) {
                    const int blk = CONTIG ? d : hb_div(d, dL), n2 = CONTIG ? 0 : d - blk * L, base = CONTIG ? d * p : blk * B + n2;
                    const double are = acc[u][0][r], aim = acc[u][1][r], bre = acc[u][2][r], bim = acc[u][3][r];
                    const double2 xa = make_double2(x0[u][r].x + are, x0[u][r].y + aim);
                    /* forward: X_k = x0 + A - iB, X_(p-k) = x0 + A + iB; inverse: signs swapped */
                    const double2 mib = INV ? make_double2(-bim, bre) : make_double2(bim, -bre);
                    const double2 r0 = cadd(xa, mib), r1 = csub(xa, mib);
                    if (!INV && n2) {
                        S.x[base + k * L] = k ? cmul(r0, S.tw(step * n2 * k)) : r0;
                        if (k) S.x[base + (p - k) * L] = cmul(r1, S.tw(step * n2 * (p - k)));
                    } else {
                        S.x[base + k * L] = r0;
                        if (k) S.x[base + (p - k) * L] = r1;
                    }
                }
            }
        }
    }
    __syncthreads();
}

/* 7-point DFT in registers, pair-symmetric (forward e^(-2 pi i nk/7); INV: e^(+...)) */
template <bool INV>
__device__ __forceinline__ void hb_dft7(double2 (&x)[7]) {
    constexpr double c1 = 0.6234898018587335, c2 = -0.2225209339563144, c3 = -0.9009688679024191;
    constexpr double s1 = 0.7818314824680298, s2 = 0.9749279121818236, s3 = 0.4338837391175581;
    const double2 a1 = cadd(x[1], x[6]), a2 = cadd(x[2], x[5]), a3 = cadd(x[3], x[4]);
    const double2 b1 = csub(x[1], x[6]), b2 = csub(x[2], x[5]), b3 = csub(x[3], x[4]);
    const double2 x0 = x[0];
    auto A = [&](double ca, double cb, double cc) {
        return make_double2(__builtin_fma(cc, a3.x, __builtin_fma(cb, a2.x, __builtin_fma(ca, a1.x, x0.x))),
                            __builtin_fma(cc, a3.y, __builtin_fma(cb, a2.y, __builtin_fma(ca, a1.y, x0.y))));
    };
    auto Bs = [&](double sa, double sb, double sc) {
        return make_double2(__builtin_fma(sc, b3.x, __builtin_fma(sb, b2.x, sa * b1.x)),
                            __builtin_fma(sc, b3.y, __builtin_fma(sb, b2.y, sa * b1.y)));
    };
    /* cos / sin (2 pi n k / 7) for n = 1, 2, 3 at k = 1, 2, 3 */
    const double2 A1 = A(c1, c2, c3), A2 = A(c2, c3, c1), A3 = A(c3, c1, c2);
    const double2 B1 = Bs(s1, s2, s3), B2 = Bs(s2, -s3, -s1), B3 = Bs(s3, -s1, s2);
    x[0] = make_double2(x0.x + a1.x + a2.x + a3.x, x0.y + a1.y + a2.y + a3.y);
    auto put = [&](int k, double2 Ak, double2 Bk) {
        /* forward: X_k = A - iB, X_(7-k) = A + iB; inverse: the other way */
        const double2 mi = make_double2(Ak.x + Bk.y, Ak.y - Bk.x), pl = make_double2(Ak.x - Bk.y, Ak.y + Bk.x);
        x[k] = INV ? pl : mi;
        x[7 - k] = INV ? mi : pl;
    };
    put(1, A1, B1);
    put(2, A2, B2);
    put(3, A3, B3);
}

/* 14-point DFT in registers as the 2 x 7 prime-factor (Good-Thomas) split:
 * input n = (7 n1 + 2 n2) mod 14, output k = (7 k1 + 8 k2) mod 14, no twiddles */
template <bool INV>
__device__ __forceinline__ void hb_dft14(double2 (&v)[14]) {
    double2 u0[7], u1[7];
#pragma unroll
    for (int n2 = 0; n2 < 7; ++n2) {
        const double2 a = v[(2 * n2) % 14], b = v[(7 + 2 * n2) % 14];
        u0[n2] = cadd(a, b);
        u1[n2] = csub(a, b);
    }
    hb_dft7<INV>(u0);
    hb_dft7<INV>(u1);
#pragma unroll
    for (int k2 = 0; k2 < 7; ++k2) {
        v[(8 * k2) % 14] = u0[k2];
        v[(7 + 8 * k2) % 14] = u1[k2];
    }
}

/* Rader's algorithm for the contiguous (L = 1, twiddle-free) radix-197 stage.
 * With g = 2 a generator mod 197 and w = e^(-2 pi i / 197),
 *   X_0 = sum_n x_n,  X_(g^-m) = x_0 + sum_q a_q b_(m-q)   (a_q = x_(g^q), b_j = w^(g^-j)),
 * a 196-point cyclic convolution: IDFT_196(DFT_196(a) . DFT_196(b) / 196), the
 * last factor a host table.  Each 196-point DFT is 14 x 14: thread (butterfly,
 * column c) holds 14 points in registers, a 14-point DFT, the W_196 twiddles,
 * one LDS exchange (row c), a 14-point DFT; the pointwise product and the
 * inverse's first 14-point DFT follow in the same registers, then the second
 * exchange and the last 14-point DFT.  The inverse stage (DIT, first in the
 * inverse pass, also twiddle-free) is conj(DFT(conj x)).  About a quarter of
 * the f64 operations of the pair-symmetric direct DFT. */
template <bool INV>
__device__ __forceinline__ void hb_rader197(const HbLds &S, const HilbPlan &P, const double2 *rt) {
    constexpr int R = 14, PR = HB_RD_P;
    const double2 *Bh = rt, *W = rt + (PR - 1);
    const int nbf = P.M / PR, ntask = nbf * R;
    auto cj = [](double2 z) { return INV ? make_double2(z.x, -z.y) : z; };
    for (int t0 = 0; t0 < ntask; t0 += HB_T) {               /* uniform trip count: barriers inside */
        const int t = t0 + (int)threadIdx.x;
        const bool act = t < ntask;
        const int f = act ? t / R : 0, c = act ? t - f * R : 0;
        double2 *blk = S.x + f * PR;
        double2 v[R], x0 = make_double2(0.0, 0.0), X0 = x0;
        int gc = 1, gic = 1;                                 /* 2^c, 99^c = 2^-c mod 197 */
        for (int j = 0; j < c; ++j) { gc = (gc * 2) % PR; gic = (gic * 99) % PR; }
        if (act) {
            x0 = cj(blk[0]);
            int e = gc;                                      /* a_(14 n1 + c) = x_(2^c 33^n1) */
#pragma unroll
            for (int n1 = 0; n1 < R; ++n1) {
                v[n1] = cj(blk[e]);
                e = (e * 33) % PR;
            }
            hb_dft14<false>(v);
            /* W_196^(c k1) as powers of W_196^c (lanes' table indices c k1 are
             * strided: the per-k1 reads were bank-conflicted) */
            const double2 wc = W[c];
            double2 tw = wc;
#pragma unroll
            for (int k1 = 1; k1 < R; ++k1) {
                v[k1] = cmul(v[k1], tw);
                tw = cmul(tw, wc);
            }
        }
        __syncthreads();
        if (act) {
#pragma unroll
            for (int k1 = 0; k1 < R; ++k1) blk[1 + k1 * R + c] = v[k1];
        }
        __syncthreads();
        if (act) {                                           /* this thread is row k1 = c */
#pragma unroll
            for (int n2 = 0; n2 < R; ++n2) v[n2] = blk[1 + c * R + n2];
            hb_dft14<false>(v);                              /* v[k2] = DFT(a)[c + 14 k2] */
            X0 = cadd(x0, v[0]);                             /* used by c == 0 only */
#pragma unroll
            for (int k2 = 0; k2 < R; ++k2) v[k2] = cmul(v[k2], Bh[c + R * k2]);
            hb_dft14<true>(v);                               /* over k2 -> m2 */
            const double2 wc = W[c];
            double2 tw = wc;
#pragma unroll
            for (int m2 = 1; m2 < R; ++m2) {
                v[m2] = cmulc(v[m2], tw);
                tw = cmul(tw, wc);
            }
        }
        __syncthreads();
        if (act) {
#pragma unroll
            for (int m2 = 0; m2 < R; ++m2) blk[1 + m2 * R + c] = v[m2];
        }
        __syncthreads();
        if (act) {                                           /* this thread is column m2 = c */
#pragma unroll
            for (int k1 = 0; k1 < R; ++k1) v[k1] = blk[1 + c * R + k1];
            hb_dft14<true>(v);                               /* v[m1] = conv[c + 14 m1] */
        }
        __syncthreads();
        if (act) {
            int e = gic;                                     /* X_(2^-(c + 14 m1)) = x_0 + conv */
#pragma unroll
            for (int m1 = 0; m1 < R; ++m1) {
                blk[e] = cj(cadd(x0, v[m1]));
                e = (e * 6) % PR;                            /* 99^14 = 6 mod 197 */
            }
            if (c == 0) blk[0] = cj(X0);
        }
        __syncthreads();
    }
}

__device__ __forceinline__ int hb_pos(const HilbPlan &P, int k) {     /* position of frequency k after the DIF */
    int pos = 0;
    for (int i = 0; i < P.ns; ++i) {
        const int r = P.rad[i], q = hb_div(k, P.dP[i]);
        pos += (k - q * r) * P.L[i];
        k = q;
    }
    return pos;
}

static_assert(HB_T == QR_T, "k_hilbert_env runs qr_select with its own threads");
#ifndef BPMX_HB_YT
#define BPMX_HB_YT 8   /* fused yd: tiles per wave per round trip (8, 16, 24 measured alike; 24 spilled SGPRs) */
#endif

__global__ __launch_bounds__(HB_T) void k_hilbert_env(HilbArgs A, HilbPlan P) {
    const int f = A.f_begin + blockIdx.x;
    if (f >= A.f_end || !A.active[f]) return;
    extern __shared__ __align__(16) double2 hb_smem[];
    const int M = P.M, N = P.N;
    HbLds S;
    S.x = hb_smem;
    S.twh = S.x + M;
    S.twl = S.twh + P.ntwh;
    S.pt = S.twl + 128;
    const int64_t d0 = A.doff[f];
    /* yd as complex pairs: 16-byte loads when the recording starts at an even
     * decimated offset, two 8-byte loads otherwise (same values, so a
     * recording's envelope does not depend on its place in the batch) */
    const bool odd = (d0 & 1) != 0;
    const double2 *y2a = (const double2 *)(A.yd + (d0 & ~(int64_t)1));
    const double *y1 = A.yd + d0;
    auto y2 = [&](int m) -> double2 {
        return odd ? make_double2(y1[2 * m], y1[2 * m + 1]) : y2a[m];
    };
    /* a leading radix-2 stage over the whole transform (B = M) is fused into
     * the load, a trailing one of the inverse into the magnitude */
    const bool r2 = P.rad[0] == 2 && P.B[0] == M;
    const int H = M / 2;
    for (int i = threadIdx.x; i < P.ntwh + 128 + P.nptab + P.nrtab; i += HB_T) S.twh[i] = A.tabs[i];
    const bool fy = A.fy != 0;
    if (fy) {
        /* yd of the full tiles, one tile per wave step (lane = block b): the
         * tile's carries by one scalar load, gamma by one coalesced row read;
         * the real array y fills S.x as the complex pairs the transform packs */
        double *xr = (double *)S.x;
        double *ydw = A.ys + hb_ys_off(d0, f);
        const int lane = (int)(threadIdx.x & 63), wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
        const int64_t tf0 = A.toff[f];
        const int btv = A.bt, ntf = (N - 1) / btv;             /* full tiles: (Nd - 1) / bt */
        const bool on = lane < btv;
        double al[4], be[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) { al[k] = on ? A.al[4 * lane + k] : 0.0; be[k] = on ? A.be[4 * lane + k] : 0.0; }
        /* eight tiles per round trip: lane l loads carry word l % 8 of the
         * round's tile l / 8 (one instruction for all eight), each tile's gamma
         * row is one load, all issued before any use; a tile's carries then
         * come out by readlane (wave-uniform) */
        constexpr int HB_YT = BPMX_HB_YT, HB_YC = (HB_YT + 7) / 8;
        for (int t0 = wv; t0 < ntf; t0 += HB_YT * (HB_T / 64)) {
            double cvs[HB_YC];
#pragma unroll
            for (int q = 0; q < HB_YC; ++q) {
                const int tl = t0 + (8 * q + (lane >> 3)) * (HB_T / 64);
                cvs[q] = tl < ntf ? A.car[(tf0 + tl) * 8 + (lane & 7)] : 0.0;
            }
            double g[HB_YT];
#pragma unroll
            for (int u = 0; u < HB_YT; ++u) {
                const int tt = t0 + u * (HB_T / 64);
                g[u] = (on && tt < ntf) ? __builtin_nontemporal_load(A.gam + (tf0 + tt) * A.gstr + lane) : 0.0;
            }
#pragma unroll
            for (int u = 0; u < HB_YT; ++u) {
                const int tt = t0 + u * (HB_T / 64);
                if (tt >= ntf) break;                          /* uniform */
                double c[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const double cv = cvs[u / 8];
                    const int lo = __builtin_amdgcn_readlane(__double2loint(cv), 8 * (u % 8) + k);
                    const int hi = __builtin_amdgcn_readlane(__double2hiint(cv), 8 * (u % 8) + k);
                    c[k] = __hiloint2double(hi, lo);
                }
                if (on) {
                    const double ya = __builtin_fma(al[0], c[4], __builtin_fma(al[1], c[5], __builtin_fma(al[2], c[6], al[3] * c[7])));
                    const double yb = __builtin_fma(be[0], c[0], __builtin_fma(be[1], c[1], __builtin_fma(be[2], c[2], be[3] * c[3])));
                    const double y = ya + yb + g[u];
                    const int j = tt * btv + lane;
                    xr[j] = y;
                    ydw[j] = y;
                }
            }
        }
        for (int j = ntf * btv + (int)threadIdx.x; j < N; j += HB_T) xr[j] = y1[j];   /* k_native_carry's part */
    } else if (!r2) {
        for (int m = threadIdx.x; m < M; m += HB_T) S.x[m] = y2(m);
    }
    __syncthreads();
    STAMP_DECL
    if (r2) {
        for (int t = threadIdx.x; t < H; t += HB_T) {        /* DIF radix 2: L = M / 2, twiddle W_N^(2t) */
            const double2 a = fy ? S.x[t] : y2(t), b = fy ? S.x[t + H] : y2(t + H), d = csub(a, b);
            S.x[t] = cadd(a, b);
            S.x[t + H] = t ? cmul(d, S.tw(2 * t)) : d;
        }
        __syncthreads();
    }
    STAMP(0);
    for (int i = r2 ? 1 : 0; i < P.ns; ++i) {
        if (P.rad[i] == 2) hb_radix2<false>(S, P, i);
        else if (P.rd[i]) hb_rader197<false>(S, P, S.pt + P.nptab);
        else if (P.cp[i]) hb_radixp_const<false>(S, P, i);
        else if (P.mf[i] && P.L[i] == 1) hb_radixp_mfma<false, true>(S, P, i, S.pt + P.ptab[i]);
        else if (P.mf[i]) hb_radixp_mfma<false, false>(S, P, i, S.pt + P.ptab[i]);
        else hb_radixp<false>(S, P, i, S.pt + P.ptab[i]);
        STAMP(i < 3 ? 1 + i : 3);
    }
    /* pointwise: pairs (k, M - k), k = 0 .. M/2 */
    for (int k = threadIdx.x; k <= M / 2; k += HB_T) {
        if (k == 0) {
            S.x[0] = make_double2(0.0, 0.0);                        /* pos(0) = 0: DC and Nyquist of the Hilbert spectrum */
            continue;
        }
        const int km = M - k;
        const int pk = hb_pos(P, k), pm = hb_pos(P, km);
        const double2 zk = S.x[pk], zm = S.x[pm];
        auto xk = [&](double2 za, double2 zb, int kk) {              /* X_kk from Z_kk, Z_(M-kk) */
            const double2 cb = make_double2(zb.x, -zb.y);
            const double2 Sm = cadd(za, cb), D = csub(za, cb), w = S.tw(kk);
            return csub(cmulc(Sm, w), cmul(w, D));
        };
        const double2 xa = xk(zk, zm, k);
        if (km != k) S.x[pm] = xk(zm, zk, km);
        S.x[pk] = xa;
    }
    __syncthreads();
    STAMP(4);
    for (int i = P.ns - 1; i >= (r2 ? 1 : 0); --i) {
        if (P.rad[i] == 2) hb_radix2<true>(S, P, i);
        else if (P.rd[i]) hb_rader197<true>(S, P, S.pt + P.nptab);
        else if (P.cp[i]) hb_radixp_const<true>(S, P, i);
        else if (P.mf[i] && P.L[i] == 1) hb_radixp_mfma<true, true>(S, P, i, S.pt + P.ptab[i]);
        else if (P.mf[i]) hb_radixp_mfma<true, false>(S, P, i, S.pt + P.ptab[i]);
        else hb_radixp<true>(S, P, i, S.pt + P.ptab[i]);
    }
    STAMP(5);
    /* |analytic| = sqrt(y^2 + (c/N)^2), in place (two reals per complex slot) */
    const double inv = 1.0 / (double)N;
    auto mag2 = [&](double2 c, double2 y) {
        const double i0 = c.x * inv, i1 = c.y * inv;
        return make_double2(sqrt(y.x * y.x + i0 * i0), sqrt(y.y * y.y + i1 * i1));
    };
    /* y for |analytic|: the full tiles' pairs from ys (written by this
     * workgroup's first phase: every wave's stores complete, then a barrier),
     * the rest from yd */
    const int jfy = fy ? (N - 1) / A.bt * A.bt : 0;           /* even: bt is */
    const double2 *ys2 = fy ? (const double2 *)(A.ys + hb_ys_off(d0, f)) : nullptr;
    if (fy) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    auto ym = [&](int m) -> double2 { return 2 * m < jfy ? ys2[m] : y2(m); };
    if (r2) {
        for (int t = threadIdx.x; t < H; t += HB_T) {        /* DIT radix 2 (conjugate twiddle before), then |.| */
            const double2 ya = ym(t), yb = ym(t + H);
            const double2 a = S.x[t];
            double2 b = S.x[t + H];
            if (t) b = cmulc(b, S.tw(2 * t));
            S.x[t] = mag2(cadd(a, b), ya);
            S.x[t + H] = mag2(csub(a, b), yb);
        }
    } else {
        for (int m = threadIdx.x; m < M; m += HB_T) S.x[m] = mag2(S.x[m], ym(m));
    }
    __syncthreads();
    STAMP(6);
    /* centred rolling mean (min_periods 1): each thread a contiguous run of
     * outputs, the window sum slid along it (one direct sum per run) */
    const int64_t w = P.window;
    double *env = A.env + d0;
    const int per = P.per;                                 /* ceil(N / HB_T) <= HB_RMPER (host checks) */
    const double *mag = (const double *)S.x;
    const int i0 = threadIdx.x * per, i1 = i0 + per < N ? i0 + per : N;
    double ev[HB_RMPER];
    /* full windows multiply by 1/w (within an ulp of the division; the
     * envelope's tolerance is 1e-9 relative), edge windows divide */
    const double invw = 1.0 / (double)w;
    auto mean = [&](double sum, int64_t cnt) { return cnt == w ? sum * invw : sum / (double)cnt; };
    /* one code path for every run: each output adds the sample entering at the
     * right (none once the window reaches N) and drops the one leaving at the
     * left (none while the window starts at 0); an absent sample adds or
     * drops 0.0, which leaves the sum bit for bit as the sliding sum had it.
     * Every LDS read is issued before the sums.  (A run holding edge windows
     * took a per-output bounds-and-loops path: the first and last threads
     * were the phase's critical path, 18 K cycles against ~5 K.) */
    if (i0 < i1) {
        const int cnt = i1 - i0, offw = (int)((w - 1) / 2) + 1, wi = (int)w;
        /* window of output i: [max(i + offw - w, 0), min(i + offw, N)) */
        auto we = [&](int i) { return min(i + offw, N); };
        auto ws = [&](int i) { return max(i + offw - wi, 0); };
        double sum = 0.0;
        for (int q = ws(i0); q < we(i0); ++q) sum += mag[q];
        ev[0] = mean(sum, we(i0) - ws(i0));
        /* in two halves, each half's reads issued before its sums (all of them
         * at once held 40 more doubles beside ev and spilled) */
        constexpr int HALF = HB_RMPER / 2;
#pragma unroll
        for (int c0 = 1; c0 < HB_RMPER; c0 += HALF) {
            double ad[HALF], sb[HALF];
#pragma unroll
            for (int u = 0; u < HALF; ++u) {
                const int j = c0 + u, i = i0 + j;
                ad[u] = (j < HB_RMPER && j < cnt && we(i) > we(i - 1)) ? mag[we(i) - 1] : 0.0;
                sb[u] = (j < HB_RMPER && j < cnt && ws(i) > ws(i - 1)) ? mag[ws(i - 1)] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < HALF; ++u) {
                const int j = c0 + u;
                if (j < HB_RMPER && j < cnt) {
                    sum += ad[u];
                    sum -= sb[u];
                    ev[j] = mean(sum, we(i0 + j) - ws(i0 + j));
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    STAMP(8);
    /* through LDS, so the global stores are coalesced */
    __syncthreads();
    STAMP(9);
    double *stage = (double *)S.x;
#pragma unroll
    for (int j = 0; j < HB_RMPER; ++j)
        if (i0 + j < i1) stage[i0 + j] = ev[j];
    __syncthreads();
    STAMP(10);
#ifdef HB_DIAG_NOQ                                              /* timing diagnostic: no select (wrong outputs) */
    if (false) {
#else
    if (A.q.n_levels > 0 && N <= QR_MAX) {
#endif
        /* the detection stage's quantiles from the staged envelope, so
         * k_quantile_reg need not reload it; each value read once for its
         * global store and its key.  (The stores after the select instead,
         * from the keys, made the kernel slower: 0.34 -> 0.356 ms; issued
         * first they drain during the select.) */
        uint64_t key[QR_IT];
#pragma unroll
        for (int it = 0; it < QR_IT; ++it) {
            const int i = it * HB_T + (int)threadIdx.x;
            const double v = i < N ? stage[i] : 0.0;
            if (i < N) env[i] = v;
            key[it] = i < N ? f64_key(v) : 0ull;
        }
        STAMP(11);
        __syncthreads();                                    /* the stage becomes the select's scratch */
        qr_select(key, N, A.q, f, *reinterpret_cast<QrShared *>(hb_smem));
    } else {
        for (int i = threadIdx.x; i < N; i += HB_T) env[i] = stage[i];
        STAMP(11);
    }
    __syncthreads();
    STAMP(7);
    STAMP_FLUSH(A.stamps);
}

/* ---------------------------------------------------------------------- */
/* host: plan + tables (long double), cached per N */
int hilbert_plan(int64_t nd, int window, HilbPlan *P, std::vector<double2> *tabs, size_t *lds_bytes, bool mfma,
                 bool rader, bool cprime) {
    if (nd < 4 || (nd & 1)) return 0;
    const int64_t M = nd / 2;
    int rad[HB_MAXS], ns = 0;
    int64_t m = M;
    while (m % 2 == 0) {
        if (ns == HB_MAXS) return 0;
        rad[ns++] = 2;
        m /= 2;
    }
    for (int64_t p = 3; m > 1; p += 2) {
        if (p > HB_PMAX) return 0;
        while (m % p == 0) {
            if (ns == HB_MAXS) return 0;
            rad[ns++] = (int)p;
            m /= p;
        }
    }
    std::memset(P, 0, sizeof(*P));
    P->M = (int32_t)M;
    P->N = (int32_t)nd;
    P->ns = ns;
    P->ntwh = (int32_t)((nd + 127) / 128);
    P->window = window;
    int64_t B = M;
    std::vector<int> primes;
    if (M >= 16384) return 0;                 /* hb_div: dividends < 16 M, divisors <= M */
    for (int i = 0; i < ns; ++i) {
        const int r = rad[i];
        P->rad[i] = r;
        P->B[i] = (int32_t)B;
        P->L[i] = (int32_t)(B / r);
        B /= r;
        const int h = (r - 1) / 2;
        P->dL[i] = hb_magic((uint32_t)P->L[i]);
        P->dP[i] = hb_magic((uint32_t)r);
        P->dH[i] = hb_magic((uint32_t)(h > 0 ? h : 1));
        P->dG[i] = hb_magic((uint32_t)((h + HB_KB) / HB_KB));
        P->dT[i] = hb_magic((uint32_t)((h + 16) / 16));
        if (r > 2) {
            /* matrix-core form: 16 x 16 output tiles within the waves' budget */
            const int64_t units = ((M / r + 15) / 16) * (((r - 1) / 2 + 16) / 16);
            P->mf[i] = mfma && r >= HB_MF_PMIN && units <= (int64_t)(HB_T / 64) * HB_MF_UNITS;
            /* Rader's 197-point DFT on the contiguous, twiddle-free stage */
            P->rd[i] = rader && r == HB_RD_P && P->L[i] == 1;
            if (P->rd[i]) P->mf[i] = 0;
            /* small primes with compile-time constants, one round of waves */
            const bool cp = cprime && hb_cp_off(r) >= 0 && !P->rd[i] &&
                            (int64_t)hb_cp_ng(r) * ((M / r + 63) / 64) <= (int64_t)(HB_T / 64);
            P->cp[i] = cp ? hb_cp_ng(r) : 0;
            P->cpo[i] = cp ? hb_cp_off(r) : 0;
            if (cp) P->mf[i] = 0;
            /* register-held outputs: (M / p) ceil((h + 1) / HB_KB) tasks over HB_T threads */
            if (!P->mf[i] && !P->rd[i] && !P->cp[i] && (M / r) * (((r + 1) / 2 + HB_KB - 1) / HB_KB) > (int64_t)HB_T * HB_MAXT)
                return 0;
            int off = -1, acc = 0;
            for (int q : primes) { if (q == r) off = acc; acc += q; }
            if (off < 0) { off = acc; primes.push_back(r); }
            P->ptab[i] = off;
        } else {
            P->ptab[i] = -1;
        }
    }
    int np = 0;
    for (int q : primes) np += q;
    P->nptab = np;
    bool any_rd = false;
    for (int i = 0; i < ns; ++i) any_rd = any_rd || P->rd[i];
    P->nrtab = any_rd ? 2 * (HB_RD_P - 1) : 0;
    P->per = (int32_t)((nd + HB_T - 1) / HB_T);
    if (P->per > HB_RMPER) return 0;
#ifdef HB_ODDPER
    /* an odd run length: the threads' runs start an odd number of doubles
     * apart, so a wave's LDS reads along the runs conflict at most 2-way */
    if ((P->per & 1) == 0 && P->per + 1 <= HB_RMPER) P->per += 1;
#endif
    *lds_bytes = (size_t)(M + P->ntwh + 128 + np + P->nrtab) * sizeof(double2);
    if (*lds_bytes > HB_LDS_MAX) return 0;
    tabs->resize((size_t)P->ntwh + 128 + np + P->nrtab);
    const long double tp = 6.283185307179586476925286766559005768L;
    for (int j = 0; j < P->ntwh; ++j) {
        const long double a = -tp * (long double)(128LL * j) / (long double)nd;
        (*tabs)[j] = make_double2((double)cosl(a), (double)sinl(a));
    }
    for (int j = 0; j < 128; ++j) {
        const long double a = -tp * (long double)j / (long double)nd;
        (*tabs)[P->ntwh + j] = make_double2((double)cosl(a), (double)sinl(a));
    }
    int o = P->ntwh + 128;
    for (int q : primes)
        for (int j = 0; j < q; ++j, ++o) {
            const long double a = tp * (long double)j / (long double)q;
            (*tabs)[o] = make_double2((double)cosl(a), (double)sinl(a));
        }
    if (any_rd) {
        /* Bh_k = DFT_196(b)_k / 196 with b_j = e^(-2 pi i (2^-j mod 197) / 197); then W_196^e */
        constexpr int Q = HB_RD_P - 1;
        int gi[Q];
        for (int j = 0, e = 1; j < Q; ++j, e = (e * 99) % HB_RD_P) gi[j] = e;   /* 99 = 2^-1 mod 197 */
        for (int k = 0; k < Q; ++k) {
            long double re = 0.0L, im = 0.0L;
            for (int j = 0; j < Q; ++j) {
                const long double a = -tp * ((long double)gi[j] / HB_RD_P + (long double)((j * k) % Q) / Q);
                re += cosl(a);
                im += sinl(a);
            }
            (*tabs)[o + k] = make_double2((double)(re / Q), (double)(im / Q));
        }
        for (int e = 0; e < Q; ++e) {
            const long double a = -tp * (long double)e / Q;
            (*tabs)[o + Q + e] = make_double2((double)cosl(a), (double)sinl(a));
        }
    }
    return 1;
}

}  // namespace bpmx
