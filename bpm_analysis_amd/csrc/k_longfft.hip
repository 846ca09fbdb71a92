/*
 * k_longfft.hip — the Hilbert transform of long recordings (native mode,
 * scipy.signal.hilbert of y[::ds]; scipy/signal/_signaltools.py:2318) by
 * exact-length DFTs, in place of k_bluestein.hip's rocFFT chirp-z for every
 * recording whose length factors as below (all of BASELINE C5's: Nd = 320 s
 * for whole seconds s in [600, 1800]).
 *
 * Even N is packed, z_m = y_2m + i y_2m+1 over M = N / 2 points (odd N:
 * M = N, unpacked), and the M-point DFT runs as a four-step transform in HBM:
 * M = A B, m = b + B a, k = k_a + A k_b,
 *     Z[k_a + A k_b] = sum_b w_M^(b k_a) w_B^(b k_b) sum_a z[b + B a] w_A^(a k_a).
 * Every sub-DFT is a contiguous row held in LDS (the tile transposes between
 * them are coalesced both ways):
 *   T1   z as [A][B] -> [B][A] (reads y in pairs: the packing is free)
 *   R1   B rows of A points, then the twiddle w_M^(b k_a)
 *   T2   [B][A] -> [A][B]
 *   R2   A rows of B points: Z_k at [k mod A][k div A]
 *   mid  real-FFT split, Hilbert multiplier, half-length inverse packing
 *        (k_blu_mid's arithmetic on that layout)
 *   R2'  inverse: A rows of B points, twiddle w_M^(-b q_a)
 *   T2'  [A][B] -> [B][A]
 *   R1'  B rows of A points
 *   T1'  [B][A] -> natural order, written as h (N x Im of the analytic
 *        signal, as the Bluestein path leaves it for k_native_env)
 * A row DFT is a Stockham autosort over mixed radices (2..64) with the n-th
 * roots of unity tabulated in LDS, or, for a prime n > 64 (the large prime
 * factor of a ragged length), Bluestein's chirp-z inside the workgroup: a
 * cyclic convolution of length L >= 2n - 1 (L <= 4096) against
 * FFT_L(b), tabulated once per prime (L the shortest 2^a 3^b 5^c >= 2n - 1).  M's largest prime factor p > 64 takes
 * A = p (p <= 2047) and B = M / p; a smooth M splits near its square root.
 * Rows are at most LF_NMAX points.  Anything else stays on the rocFFT path.
 */
#include <algorithm>
#include <cmath>
#include <map>
#include <vector>

#include "bpmx_common.h"
#include "bpmx_kernels.h"
#include "bpmx_native.h"

namespace bpmx {

constexpr int LF_T = 1024;         /* threads per row workgroup */
constexpr int LF_NMAX = 4608;      /* longest direct row */
constexpr int LF_LMAX = 4096;      /* longest Bluestein convolution */
constexpr int LF_GROUP = 4096;     /* points of short rows gathered into one workgroup */
constexpr int LF_RMAX = 64;        /* largest direct radix */
constexpr int LF_MAXR = 16;
constexpr int LF_TS = 32;          /* transpose tile */

struct LfSub {                     /* an n-point DFT in LDS */
    int32_t n, L, nrad, rpw;       /* L > 0: Bluestein for prime n over L points; rows per workgroup */
    int32_t rad[LF_MAXR];          /* Stockham radices of n (or of L) */
    int64_t fb;                    /* Bluestein: FFT_L(b) at fbt + fb */
    int64_t toff;                  /* tab: roots e^(-2 pi i t / n) (direct) or chirp c_m (Bluestein) */
    int64_t loff;                  /* Bluestein / Rader: tab offset of the roots of L */
    int32_t kind, pad2;            /* 0 direct, 1 Bluestein, 2 Rader (L = n - 1) */
    int64_t ioff;                  /* Rader: itab + ioff: g^q mod n, then g^-q mod n (q < n - 1) */
};
struct LfRec {                     /* one recording */
    int64_t d0, w0;                /* decimated offset (y, h); work offset (double2) */
    int64_t toff;                  /* tab: w_M^t for t < T, then w_M^(u T) for u < ceil(M / T) */
    int32_t N, M, A, B, pack, sa, sb, twT;
};
/* table fill descriptors (once per geometry) */
struct LfTab {
    int64_t off;
    int32_t count, kind, n, T;     /* kind 0: e^(-2 pi i t / n); 1: e^(-i pi t^2 / n); 2: e^(-2 pi i (t T mod n) / n) */
};
struct LfArgs {
    const double *yd;
    double *hb;
    double2 *w1, *w2;
    const double2 *fbt;            /* FFT_L(b) tables */
    const double2 *tab;            /* roots, chirps, four-step twiddles */
    const int32_t *itab;           /* Rader permutations */
    const LfRec *rec;
    const LfSub *sub;
    const int32_t *pre;            /* work-item prefix over the recordings [R + 1] */
    int32_t R;
};

namespace {
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 conj2(double2 a) { return make_double2(a.x, -a.y); }
__device__ __forceinline__ double2 add2(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 sub2(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 scale2(double2 a, double s) { return make_double2(a.x * s, a.y * s); }
/* e^(sign 2 pi i t / n) for 0 <= t < n (t / n exact in sincospi's argument) */
__device__ __forceinline__ double2 root(int64_t t, int64_t n, int sign) {
    double sn, cs;
    sincospi(2.0 * (double)t / (double)n, &sn, &cs);
    return make_double2(cs, sign * sn);
}
/* the work item's recording: last r with pre[r] <= g */
__device__ __forceinline__ int rec_of(const int32_t *pre, int R, int g) {
    int lo = 0, hi = R;
    while (hi - lo > 1) { const int mid = (lo + hi) >> 1; if (pre[mid] <= g) lo = mid; else hi = mid; }
    return lo;
}

/* w_M^t = e^(-2 pi i t / M) from the recording's two-level table (sign +1: conjugate) */
__device__ __forceinline__ double2 twid(const double2 *tab, const LfRec &rc, int64_t t, int sign) {
    const uint32_t hi = (uint32_t)t / (uint32_t)rc.twT, lo = (uint32_t)t - hi * (uint32_t)rc.twT;
    const double2 w = cmul(tab[rc.toff + lo], tab[rc.toff + rc.twT + hi]);
    return sign < 0 ? w : conj2(w);
}

/* x / d for 0 <= x < 2^22 (a float reciprocal, then one correction) */
__device__ __forceinline__ int fdiv(int x, int d, float rcp) {
    int q = (int)((float)x * rcp);
    const int r = x - q * d;
    q += r < 0 ? -1 : (r >= d ? 1 : 0);
    return q;
}

/* One Stockham stage of radix R over nrows rows of n points in LDS (natural
 * order in and out), roots rt[t] = e^(sign 2 pi i t / n).  Butterfly j of a
 * row (j < n / R, jm = j mod Ns): v_r = x[j + r n/R] rt[r jm n/(Ns R)], then
 * out[(j / Ns) Ns R + k Ns + jm] = sum_r v_r w_R^(r k).  A thread keeps its
 * butterflies' outputs in registers between the read and write halves, so one
 * buffer serves every stage. */
template <int R>
__device__ __forceinline__ void lf_stage(double2 *x, const double2 *rt, int n, int nrows, int Ns) {
    constexpr int BPT = (LF_NMAX / R + LF_T - 1) / LF_T;
    const int tid = threadIdx.x;
    const int nR = n / R, NsR = Ns * R, step = n / NsR, nb = nrows * nR;
    const float rnR = 1.0f / (float)nR, rNs = 1.0f / (float)Ns;
    double2 v[BPT][R];
    int dst[BPT];
#pragma unroll
    for (int it = 0; it < BPT; ++it) {
        const int b = tid + it * LF_T;
        dst[it] = -1;
        if (b < nb) {
            const int row = fdiv(b, nR, rnR), j = b - row * nR;
            const int jh = fdiv(j, Ns, rNs), jm = j - jh * Ns;
            const double2 *xr = x + row * n;
            const int t1 = jm * step;                           /* < n */
            int t = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                double2 a = xr[j + r * nR];
                if (r > 0) {
                    t += t1;
                    if (t >= n) t -= n;
                    const double2 w = rt[t];
                    a = cmul(a, w);
                }
                v[it][r] = a;
            }
            /* R-point DFT */
            double2 o[R];
            if (R == 2) {
                o[0] = add2(v[it][0], v[it][1]);
                o[1] = sub2(v[it][0], v[it][1]);
            } else if (R == 4) {
                const double2 w = rt[nR];                       /* e^(sign i pi / 2) = sign * i */
                const double2 s02 = add2(v[it][0], v[it][2]), d02 = sub2(v[it][0], v[it][2]);
                const double2 s13 = add2(v[it][1], v[it][3]), d13 = sub2(v[it][1], v[it][3]);
                const double2 wd = make_double2(-w.y * d13.y, w.y * d13.x);
                o[0] = add2(s02, s13);
                o[2] = sub2(s02, s13);
                o[1] = add2(d02, wd);
                o[3] = sub2(d02, wd);
            } else if (R == 8) {
                /* radix 2 x 4: a_k = v_k + v_(k+4), b_k = (v_k - v_(k+4)) w8^k, then two
                 * 4-point DFTs give the even and the odd outputs; w8 = e^(sign i pi / 4) */
                const double2 w4 = rt[2 * nR];                  /* w8^2 = sign * i */
                const double sg = w4.y, h = 0.70710678118654752440;
                double2 a[4], bb[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    a[k] = add2(v[it][k], v[it][k + 4]);
                    bb[k] = sub2(v[it][k], v[it][k + 4]);
                }
                /* b1 *= (1 + sg i) / sqrt 2, b2 *= sg i, b3 *= (-1 + sg i) / sqrt 2 */
                bb[1] = make_double2(h * (bb[1].x - sg * bb[1].y), h * (bb[1].y + sg * bb[1].x));
                bb[2] = make_double2(-sg * bb[2].y, sg * bb[2].x);
                bb[3] = make_double2(h * (-bb[3].x - sg * bb[3].y), h * (-bb[3].y + sg * bb[3].x));
                auto dft4 = [&](const double2 *x4, double2 *y0, double2 *y1, double2 *y2, double2 *y3) {
                    const double2 s02 = add2(x4[0], x4[2]), d02 = sub2(x4[0], x4[2]);
                    const double2 s13 = add2(x4[1], x4[3]), d13 = sub2(x4[1], x4[3]);
                    const double2 wd = make_double2(-sg * d13.y, sg * d13.x);
                    *y0 = add2(s02, s13);
                    *y2 = sub2(s02, s13);
                    *y1 = add2(d02, wd);
                    *y3 = sub2(d02, wd);
                };
                dft4(a, &o[0], &o[2], &o[4], &o[6]);
                dft4(bb, &o[1], &o[3], &o[5], &o[7]);
            } else {
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    double2 acc = v[it][0];
#pragma unroll
                    for (int r = 1; r < R; ++r) {
                        const double2 w = rt[((r * k) % R) * nR];
                        acc = add2(acc, cmul(v[it][r], w));
                    }
                    o[k] = acc;
                }
            }
#pragma unroll
            for (int k = 0; k < R; ++k) v[it][k] = o[k];
            dst[it] = row * n + jh * NsR + jm;
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < BPT; ++it)
        if (dst[it] >= 0) {
#pragma unroll
            for (int k = 0; k < R; ++k) x[dst[it] + k * Ns] = v[it][k];
        }
    __syncthreads();
}

/* a stage of a larger radix (8 < R <= 64): one output per thread item,
 * out[o] = sum_r x[j + r n/R] rt[r (jm + k Ns) n / (Ns R)] */
__device__ __forceinline__ void lf_stage_gen(double2 *x, const double2 *rt, int n, int nrows, int Ns, int R) {
    constexpr int OPT = (LF_NMAX + LF_T - 1) / LF_T;
    const int tid = threadIdx.x;
    const int nR = n / R, NsR = Ns * R, step = n / NsR, tot = nrows * n;
    const float rn = 1.0f / (float)n, rNs = 1.0f / (float)Ns, rR = 1.0f / (float)R;
    double2 acc[OPT];
    int dst[OPT];
#pragma unroll
    for (int it = 0; it < OPT; ++it) {
        const int e = tid + it * LF_T;
        dst[it] = -1;
        acc[it] = make_double2(0.0, 0.0);
        if (e < tot) {
            const int row = fdiv(e, n, rn), o = e - row * n;
            const int q = fdiv(o, Ns, rNs), jm = o - q * Ns;    /* q = (o / Ns) = jh R + k */
            const int jh = fdiv(q, R, rR), k = q - jh * R;
            const int j = jh * Ns + jm;
            const double2 *xr = x + row * n;
            const int t1 = (jm + k * Ns) * step;                /* < n */
            double2 a = xr[j];
            int t = 0;
            for (int r = 1; r < R; ++r) {
                t += t1;
                if (t >= n) t -= n;
                a = add2(a, cmul(xr[j + r * nR], rt[t]));
            }
            acc[it] = a;
            dst[it] = e;
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < OPT; ++it)
        if (dst[it] >= 0) x[dst[it]] = acc[it];
    __syncthreads();
}

__device__ __forceinline__ void lds_fft(double2 *x, const double2 *rt, int n, int nrows, const int32_t *rad, int nrad) {
    int Ns = 1;
    for (int s = 0; s < nrad; ++s) {
        const int R = rad[s];
        switch (R) {
        case 2: lf_stage<2>(x, rt, n, nrows, Ns); break;
        case 3: lf_stage<3>(x, rt, n, nrows, Ns); break;
        case 4: lf_stage<4>(x, rt, n, nrows, Ns); break;
        case 5: lf_stage<5>(x, rt, n, nrows, Ns); break;
        case 8: lf_stage<8>(x, rt, n, nrows, Ns); break;
        default: lf_stage_gen(x, rt, n, nrows, Ns, R); break;
        }
        Ns *= R;
    }
}
}  // namespace

/* ---- transposes: [rows][cols] -> [cols][rows] per recording, 32 x 32 tiles.
 * MODE 1: input is y as pairs (z_m = y_2m + i y_2m+1, or y_m + 0i unpacked);
 * MODE 2: output is h (pairs, or the real part unpacked).  dir 0: [A][B] ->
 * [B][A]; dir 1: [B][A] -> [A][B]. */
template <int MODE>
__global__ __launch_bounds__(256) void k_lf_tr(LfArgs A, const double2 *__restrict__ in, double2 *__restrict__ out,
                                               int dir) {
    __shared__ double2 tile[LF_TS][LF_TS + 1];
    const int g = blockIdx.x;
    const int r = rec_of(A.pre, A.R, g);
    const LfRec rc = A.rec[r];
    const int rows = dir == 0 ? rc.A : rc.B, cols = dir == 0 ? rc.B : rc.A;
    const int tc = (cols + LF_TS - 1) / LF_TS;
    const int t = g - A.pre[r];
    const int r0 = (t / tc) * LF_TS, c0 = (t % tc) * LF_TS;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int yy = ty; yy < LF_TS; yy += 8) {
        const int ri = r0 + yy, ci = c0 + tx;
        if (ri < rows && ci < cols) {
            const int64_t m = (int64_t)ri * cols + ci;
            double2 v;
            if (MODE == 1) {
                const double *y = A.yd + rc.d0;
                v = rc.pack ? make_double2(y[2 * m], y[2 * m + 1]) : make_double2(y[m], 0.0);
            } else {
                v = in[rc.w0 + m];
            }
            tile[yy][tx] = v;
        }
    }
    __syncthreads();
    for (int yy = ty; yy < LF_TS; yy += 8) {
        const int ci = c0 + yy, ri = r0 + tx;        /* out row ci, column ri */
        if (ri < rows && ci < cols) {
            const int64_t m = (int64_t)ci * rows + ri;
            const double2 v = tile[tx][yy];
            if (MODE == 2) {
                double *h = A.hb + rc.d0;
                if (rc.pack) { h[2 * m] = v.x; h[2 * m + 1] = v.y; }
                else h[m] = v.x;
            } else {
                out[rc.w0 + m] = v;
            }
        }
    }
}

/* ---- row DFTs: one workgroup per group of rpw rows of n = (useA ? A : B)
 * points, in place in buf; rows per recording = M / n.  sign -1 forward, +1
 * inverse.  tw: then multiply element k of row q by e^(sign 2 pi i (q k mod M) / M). */
__global__ __launch_bounds__(LF_T) void k_lf_rows(LfArgs A, double2 *__restrict__ buf, int useA, int sign, int tw) {
    extern __shared__ double2 lds[];
    const int g = blockIdx.x;
    const int r = rec_of(A.pre, A.R, g);
    const LfRec rc = A.rec[r];
    const LfSub *sbp = A.sub + (useA ? rc.sa : rc.sb);        /* radices read from global (scalar cache) */
    const int n = sbp->n, Lb = sbp->L, nrad = sbp->nrad, rpw = sbp->rpw, tid = threadIdx.x;
    const int64_t M = rc.M;
    const int rows = useA ? rc.B : rc.A;
    const int q0 = (g - A.pre[r]) * rpw;
    const int nr = min(rpw, rows - q0);
    double2 *row0 = buf + rc.w0 + (int64_t)q0 * n;
    if (Lb == 0) {
        double2 *x = lds, *rt = lds + (int64_t)rpw * n;
        for (int i = tid; i < nr * n; i += LF_T) x[i] = row0[i];
        for (int i = tid; i < n; i += LF_T) {
            const double2 w = A.tab[sbp->toff + i];
            rt[i] = sign < 0 ? w : conj2(w);
        }
        __syncthreads();
        lds_fft(x, rt, n, nr, sbp->rad, nrad);
        if (!tw) {
            for (int i = tid; i < nr * n; i += LF_T) row0[i] = x[i];
            return;
        }
        /* element k of row q times w_M^(q k): t = q k mod M stepped by q LF_T */
        for (int qq = 0; qq < nr; ++qq) {
            const int64_t q = q0 + qq, d = (q * LF_T) % M;
            int64_t t = (q * tid) % M;
            for (int k = tid; k < n; k += LF_T) {
                row0[(int64_t)qq * n + k] = cmul(x[qq * n + k], twid(A.tab, rc, t, sign));
                t += d;
                if (t >= M) t -= M;
            }
        }
        return;
    }
    if (sbp->kind == 2) {
        /* Rader, prime n with a smooth n - 1 = P (rpw rows per workgroup): with
         * g a primitive root, a_q = x_(g^q), b_q = w_n^(g^-q) (w_n =
         * e^(-2 pi i / n); the inverse transform conjugates), X_(g^-m) = x_0 +
         * (a (*) b)_m, the cyclic convolution by FFT_P; X_0 = x_0 + sum_q a_q =
         * x_0 + FFT_P(a)_0 */
        const int P = Lb;
        double2 *xin = lds, *a = lds + (int64_t)rpw * n, *rt = a + (int64_t)rpw * P;
        __shared__ double2 s_x0[64], s_X0[64];
        const int32_t *perm = A.itab + sbp->ioff, *iperm = perm + P;
        for (int i = tid; i < nr * n; i += LF_T) xin[i] = row0[i];
        for (int i = tid; i < P; i += LF_T) rt[i] = A.tab[sbp->loff + i];
        __syncthreads();
        const float rP = 1.0f / (float)P, rn = 1.0f / (float)n;
        for (int i = tid; i < nr * P; i += LF_T) {
            const int r = fdiv(i, P, rP), q = i - r * P;
            a[i] = xin[r * n + perm[q]];
        }
        __syncthreads();
        lds_fft(a, rt, P, nr, sbp->rad, nrad);
        for (int r = tid; r < nr; r += LF_T) {
            s_x0[r] = xin[r * n];
            s_X0[r] = add2(xin[r * n], a[r * P]);
        }
        __syncthreads();
        const double2 *fb = A.fbt + sbp->fb + (sign < 0 ? 0 : P);
        for (int i = tid; i < nr * P; i += LF_T) a[i] = cmul(a[i], fb[i - fdiv(i, P, rP) * P]);
        for (int i = tid; i < P; i += LF_T) rt[i] = conj2(rt[i]);
        __syncthreads();
        lds_fft(a, rt, P, nr, sbp->rad, nrad);
        /* unpermute into LDS (x_0 is saved), then one coalesced pass with the
         * four-step twiddle */
        const double invP = 1.0 / (double)P;
        for (int i = tid; i < nr * n; i += LF_T) {
            const int r = fdiv(i, n, rn), m = i - r * n;     /* m = P stands for X_0 */
            xin[r * n + (m == P ? 0 : iperm[m])] = m == P ? s_X0[r] : add2(s_x0[r], scale2(a[r * P + m], invP));
        }
        __syncthreads();
        if (!tw) {
            for (int i = tid; i < nr * n; i += LF_T) row0[i] = xin[i];
            return;
        }
        for (int qq = 0; qq < nr; ++qq) {
            const int64_t q = q0 + qq, d = (q * LF_T) % M;
            int64_t t = (q * tid) % M;
            for (int k = tid; k < n; k += LF_T) {
                row0[(int64_t)qq * n + k] = cmul(xin[qq * n + k], twid(A.tab, rc, t, sign));
                t += d;
                if (t >= M) t -= M;
            }
        }
        return;
    }
    /* Bluestein, prime n over L points (one row): X_k = ch_k sum_j (x_j ch_j)
     * conj(ch_(k-j)), ch = c (forward) or conj(c) (inverse), c_m =
     * e^(-i pi m^2 / n); the convolution by FFT_L: kernel FFT_L(b) (forward)
     * or its conjugate */
    const int L = Lb;
    double2 *x = lds, *rt = lds + L;
    const double2 *ch = A.tab + sbp->toff;                  /* c_m = e^(-i pi m^2 / n) */
    auto chirp = [&](int m) -> double2 { const double2 c = ch[m]; return sign < 0 ? c : conj2(c); };
    for (int i = tid; i < L; i += LF_T) {
        x[i] = i < n ? cmul(row0[i], chirp(i)) : make_double2(0.0, 0.0);
        rt[i] = A.tab[sbp->loff + i];
    }
    __syncthreads();
    lds_fft(x, rt, L, 1, sbp->rad, nrad);
    const double2 *fb = A.fbt + sbp->fb;
    for (int i = tid; i < L; i += LF_T) {
        const double2 b = fb[i];
        x[i] = cmul(x[i], sign < 0 ? b : conj2(b));
        rt[i] = conj2(rt[i]);                               /* the inverse's roots */
    }
    __syncthreads();
    lds_fft(x, rt, L, 1, sbp->rad, nrad);
    const double invL = 1.0 / (double)L;
    const int64_t d = ((int64_t)q0 * LF_T) % M;
    int64_t t = ((int64_t)q0 * tid) % M;
    for (int i = tid; i < n; i += LF_T) {
        double2 v = scale2(cmul(x[i], chirp(i)), invL);
        if (tw) v = cmul(v, twid(A.tab, rc, t, sign));
        row0[i] = v;
        t += d;
        if (t >= M) t -= M;
    }
}

/* FFT_L(b) of one Bluestein prime: b_m = conj(c_m) for m < n, b_(L-m) =
 * conj(c_m) for 0 < m < n, else 0 (one workgroup per prime) */
__global__ __launch_bounds__(LF_T) void k_lf_blu_b(const LfSub *sub, const int32_t *which, const double2 *tab,
                                                  double2 *fbt) {
    extern __shared__ double2 lds[];
    const LfSub *sbp = sub + which[blockIdx.x];
    const int n = sbp->n, L = sbp->L, tid = threadIdx.x;
    double2 *x = lds, *rt = lds + L;
    for (int i = tid; i < L; i += LF_T) {
        const int m = i < n ? i : (i > L - n ? L - i : -1);
        x[i] = m >= 0 ? conj2(tab[sbp->toff + m]) : make_double2(0.0, 0.0);
        rt[i] = tab[sbp->loff + i];
    }
    __syncthreads();
    lds_fft(x, rt, L, 1, sbp->rad, sbp->nrad);
    for (int i = tid; i < L; i += LF_T) fbt[sbp->fb + i] = x[i];
}

/* FFT_P(b) and FFT_P(conj b) of one Rader prime, b_q = w_n^(g^-q) */
__global__ __launch_bounds__(LF_T) void k_lf_rader_b(const LfSub *sub, const int32_t *which, const double2 *tab,
                                                    const int32_t *itab, double2 *fbt) {
    extern __shared__ double2 lds[];
    const LfSub *sbp = sub + which[blockIdx.x];
    const int P = sbp->L, tid = threadIdx.x;
    const int32_t *iperm = itab + sbp->ioff + P;
    double2 *x = lds, *rt = lds + P;
    for (int c = 0; c < 2; ++c) {
        for (int i = tid; i < P; i += LF_T) {
            const double2 b = tab[sbp->toff + iperm[i]];
            x[i] = c == 0 ? b : conj2(b);
            rt[i] = tab[sbp->loff + i];
        }
        __syncthreads();
        lds_fft(x, rt, P, 1, sbp->rad, sbp->nrad);
        for (int i = tid; i < P; i += LF_T) fbt[sbp->fb + c * P + i] = x[i];
        __syncthreads();
    }
}

/* the tables: one workgroup row per descriptor, exact arguments for sincospi */
__global__ __launch_bounds__(256) void k_lf_tab(const LfTab *desc, double2 *tab) {
    const LfTab d = desc[blockIdx.y];
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= d.count) return;
    double sn, cs;
    if (d.kind == 1) {
        const int64_t e = (t * t) % (2 * (int64_t)d.n);
        sincospi((double)e / (double)d.n, &sn, &cs);
    } else {
        const int64_t e = d.kind == 2 ? (t * d.T) % d.n : t;
        sincospi(2.0 * (double)e / (double)d.n, &sn, &cs);
    }
    tab[d.off + t] = make_double2(cs, -sn);
}

/* forward DFT Z at [k mod A][k div A]: real-FFT split, Hilbert multiplier,
 * half-length inverse packing (k_blu_mid's arithmetic, no chirps).  Threads
 * walk the storage order (row k_a, column k_b: k = k_a + A k_b), so a row's
 * pairs (k, M - k) read one row forwards and the partner row backwards. */
__global__ __launch_bounds__(256) void k_lf_mid(LfArgs A) {
    const int g = blockIdx.x;
    const int r = rec_of(A.pre, A.R, g);
    const LfRec rc = A.rec[r];
    const int64_t sidx = (int64_t)(g - A.pre[r]) * 256 + threadIdx.x;
    const int64_t M = rc.M, N = rc.N, Aa = rc.A, Bb = rc.B;
    if (sidx >= M) return;
    double2 *z = A.w2 + rc.w0;
    const int64_t ka = sidx / Bb, kb = sidx - ka * Bb;
    const int64_t k = ka + Aa * kb;
    auto pos = [Aa, Bb](int64_t kk) -> int64_t { return (kk % Aa) * Bb + kk / Aa; };
    if (!rc.pack) {                                          /* odd N: V_k = -i X_k (k < N/2), +i X_k (k > N/2) */
        const double2 X = z[sidx];
        z[sidx] = k == 0 ? make_double2(0.0, 0.0) : (2 * k < N ? make_double2(X.y, -X.x) : make_double2(-X.y, X.x));
        return;
    }
    if (2 * k > M) return;                                   /* the pair's other thread */
    const int64_t kp = M - k;                                /* kp == M stands for 0 */
    const double2 Zk = z[sidx];
    const double2 Zp = kp == M ? Zk : z[pos(kp)];
    auto spec = [N](int64_t qq, double2 Zq, double2 Zr) -> double2 {
        double sn, cs;
        sincospi(2.0 * (double)qq / (double)N, &sn, &cs);
        const double2 t = make_double2(cs, -sn);
        const double2 s = add2(Zq, conj2(Zr)), d = sub2(Zq, conj2(Zr));
        const double2 td = cmul(t, d);
        return make_double2(0.5 * (s.x + td.y), 0.5 * (s.y - td.x));
    };
    const double2 Xk = spec(k, Zk, Zp), Xp = spec(kp, Zp, Zk);
    const double2 Wk = k == 0 ? make_double2(0.0, 0.0) : make_double2(Xk.y, -Xk.x);
    const double2 Wp = (kp == M || kp == 0) ? make_double2(0.0, 0.0) : make_double2(Xp.y, -Xp.x);
    auto pack = [N](int64_t qq, double2 Wq, double2 Wr) -> double2 {
        double sn, cs;
        sincospi(2.0 * (double)qq / (double)N, &sn, &cs);
        const double2 e = make_double2(-sn, cs);
        return add2(add2(Wq, conj2(Wr)), cmul(e, sub2(Wq, conj2(Wr))));
    };
    z[sidx] = pack(k, Wk, Wp);
    if (kp < M && kp != k) z[pos(kp)] = pack(kp, Wp, Wk);
}

/* ---------------------------------------------------------------------- */
namespace {
std::vector<int> factorize(int64_t n) {
    std::vector<int> f;
    for (int64_t d = 2; d * d <= n; ++d)
        while (n % d == 0) { f.push_back((int)d); n /= d; }
    if (n > 1) f.push_back((int)n);
    return f;
}
/* Stockham radices of a smooth n (factors <= LF_RMAX): fours first, then the rest */
bool radices(int64_t n, std::vector<int> &out) {
    out.clear();
    std::vector<int> f = factorize(n);
    int twos = 0;
    std::vector<int> odd;
    for (int p : f) {
        if (p > LF_RMAX) return false;
        if (p == 2) ++twos; else odd.push_back(p);
    }
    for (; twos >= 3; twos -= 3) out.push_back(8);
    if (twos == 2) out.push_back(4);
    if (twos == 1) out.push_back(2);
    for (int p : odd) out.push_back(p);
    return (int)out.size() <= LF_MAXR;
}
/* the least primitive root of a prime p, or 0 */
int32_t primitive_root(int64_t p) {
    if (p < 3) return 0;
    std::vector<int> f = factorize(p - 1);
    f.erase(std::unique(f.begin(), f.end()), f.end());
    for (int64_t g = 2; g < p; ++g) {
        bool ok = true;
        for (int q : f) {
            int64_t e = (p - 1) / q, r = 1, b = g;
            while (e) { if (e & 1) r = r * b % p; b = b * b % p; e >>= 1; }
            if (r == 1) { ok = false; break; }
        }
        if (ok) return (int32_t)g;
    }
    return 0;
}
}  // namespace

/* per-context host state: the plan of the last geometry (host copies outlive
 * their async uploads) */
struct LfHost {
    std::vector<int64_t> key;
    std::vector<LfRec> recs;
    std::vector<LfSub> subs;
    std::vector<int32_t> pre, blu, rad, itab;
    std::vector<LfTab> tabs;
    int64_t fbsz = 0, work = 0, tabsz = 0;
    size_t lds = 0;
    bool uploaded = false;
};

void longfft_free(bpmx_ctx *ctx) {
    delete (LfHost *)ctx->lf;
    ctx->lf = nullptr;
}

/* the four-step plan of one length: false when it does not fit */
static bool lf_shape(int64_t M, int32_t *A, int32_t *B) {
    std::vector<int> f = factorize(M);
    const int p = f.empty() ? 1 : f.back();
    if (p > LF_RMAX) {
        if (2 * (int64_t)p - 1 > LF_LMAX || M / p > LF_NMAX) return false;
        std::vector<int> r;
        if (!radices(M / p, r)) return false;
        *A = p;
        *B = (int32_t)(M / p);
        return true;
    }
    int64_t best = 0;
    const double sq = std::sqrt((double)M);
    for (int64_t a = 1; a <= LF_NMAX && a <= M; ++a) {
        if (M % a || M / a > LF_NMAX) continue;
        if (!best || std::fabs((double)a - sq) < std::fabs((double)best - sq)) best = a;
    }
    if (!best) return false;
    *A = (int32_t)best;
    *B = (int32_t)(M / best);
    return true;
}

bool longfft_supported(int64_t N) {
    if (N < 64 || N > 2 * (int64_t)LF_NMAX * LF_NMAX) return false;
    const int64_t M = (N % 2 == 0) ? N / 2 : N;
    int32_t a, b;
    return lf_shape(M, &a, &b);
}

int longfft_hilbert(bpmx_ctx *ctx, hipStream_t s, const double *yd, double *hb, const std::vector<int64_t> &doff,
                    const std::vector<int32_t> &files) {
    if (files.empty()) return BPMX_OK;
    if (!ctx->lf) ctx->lf = new LfHost();
    LfHost &H = *(LfHost *)ctx->lf;
    std::vector<int64_t> key;
    for (int32_t f : files) { key.push_back(f); key.push_back(doff[f + 1] - doff[f]); key.push_back(doff[f]); }
    int rc = BPMX_OK;
    const int R = (int)files.size();
    if (key != H.key) {
        /* plans: recordings, sub-DFTs (one per distinct length), work-item prefixes */
        std::vector<LfRec> recs(R);
        std::vector<LfSub> subs;
        std::map<int32_t, int32_t> sub_of;
        std::map<int32_t, int64_t> root_of;                  /* Bluestein lengths' root tables */
        int64_t fbsz = 0, tabsz = 0;
        std::vector<int32_t> blu, rad, itab;
        std::vector<LfTab> tabs;
        auto get_sub = [&](int32_t n) -> int32_t {
            auto it = sub_of.find(n);
            if (it != sub_of.end()) return it->second;
            LfSub sb{};
            sb.n = n;
            std::vector<int> rd, rp;
            const bool direct = radices(n, rd);
            const bool rader = !direct && radices(n - 1, rp) && primitive_root(n) > 0;
            sb.kind = direct ? 0 : (rader ? 2 : 1);
            sb.toff = tabsz;
            tabs.push_back(LfTab{tabsz, n, sb.kind == 1 ? 1 : 0, n, 0});    /* roots of n, or chirps */
            tabsz += n;
            auto roots_of = [&](int32_t L) -> int64_t {
                auto lt = root_of.find(L);
                if (lt == root_of.end()) {
                    lt = root_of.emplace(L, tabsz).first;
                    tabs.push_back(LfTab{tabsz, L, 0, L, 0});
                    tabsz += L;
                }
                return lt->second;
            };
            if (direct) {
                sb.L = 0;
                sb.rpw = std::max(1, LF_GROUP / n);
            } else if (rader) {
                /* g^q and g^-q mod n; the convolution kernels' spectra at fb (forward, inverse) */
                const int32_t P = n - 1, g = primitive_root(n);
                /* rows per workgroup: LF_GROUP points, within ~144 KB of LDS */
                sb.rpw = std::max(1, std::min({LF_GROUP / P, (9216 - P) / (n + P), 64}));
                sb.L = P;
                rd = rp;
                sb.loff = roots_of(P);
                sb.ioff = (int64_t)itab.size();
                std::vector<int32_t> pw(P);
                int64_t v = 1;
                for (int q = 0; q < P; ++q) { pw[q] = (int32_t)v; v = v * g % n; }
                for (int q = 0; q < P; ++q) itab.push_back(pw[q]);
                for (int q = 0; q < P; ++q) itab.push_back(pw[(P - q) % P]);     /* g^-q = g^(P - q) */
                sb.fb = fbsz;
                fbsz += 2 * P;
                rad.push_back((int32_t)subs.size());
            } else {
                sb.rpw = 1;
                /* the shortest 2^a 3^b 5^c >= 2n - 1 (power-of-two padding would
                 * cost ~40 % more butterflies over C5's lengths) */
                int32_t L = 0;
                for (int64_t p2 = 1; p2 <= LF_LMAX; p2 *= 2)
                    for (int64_t p3 = p2; p3 <= LF_LMAX; p3 *= 3)
                        for (int64_t p5 = p3; p5 <= LF_LMAX; p5 *= 5)
                            if (p5 >= 2 * n - 1 && (L == 0 || p5 < L)) L = (int32_t)p5;
                sb.L = L;
                radices(L, rd);
                sb.loff = roots_of(L);
                sb.fb = fbsz;
                fbsz += L;
                blu.push_back((int32_t)subs.size());
            }
            sb.nrad = (int32_t)rd.size();
            for (int i = 0; i < sb.nrad; ++i) sb.rad[i] = rd[i];
            subs.push_back(sb);
            return sub_of[n] = (int32_t)subs.size() - 1;
        };
        int64_t w = 0;
        size_t lds = 0;
        for (int k = 0; k < R; ++k) {
            const int32_t f = files[k];
            LfRec &r = recs[k];
            r.d0 = doff[f];
            r.N = (int32_t)(doff[f + 1] - doff[f]);
            r.pack = r.N % 2 == 0;
            r.M = r.pack ? r.N / 2 : r.N;
            if (!lf_shape(r.M, &r.A, &r.B)) return fail(BPMX_E_LIMIT, "longfft: unsupported length");
            r.sa = get_sub(r.A);
            r.sb = get_sub(r.B);
            r.w0 = w;
            w += r.M;
            r.twT = (int32_t)std::ceil(std::sqrt((double)r.M));
            const int32_t nhi = (r.M + r.twT - 1) / r.twT;
            r.toff = tabsz;
            tabs.push_back(LfTab{tabsz, r.twT, 0, r.M, 0});
            tabs.push_back(LfTab{tabsz + r.twT, nhi, 2, r.M, r.twT});
            tabsz += r.twT + nhi;
        }
        for (auto &sb : subs)
            lds = std::max(lds, (size_t)(sb.kind == 0 ? (sb.rpw + 1) * sb.n
                                         : sb.kind == 1 ? 2 * sb.L : sb.rpw * (sb.n + sb.L) + sb.L) * sizeof(double2));
        /* prefixes: tiles (T1, T1' over [A][B] / [B][A]: same count), rows of B
         * (R1, R1': B rows of A points), rows of A (R2, R2'), mid groups */
        std::vector<int32_t> pre(4 * (R + 1), 0);
        for (int k = 0; k < R; ++k) {
            const LfRec &r = recs[k];
            const int32_t tiles = ((r.A + LF_TS - 1) / LF_TS) * ((r.B + LF_TS - 1) / LF_TS);
            pre[0 * (R + 1) + k + 1] = pre[0 * (R + 1) + k] + tiles;
            const int32_t ra = subs[r.sa].rpw, rb = subs[r.sb].rpw;   /* rows per workgroup */
            pre[1 * (R + 1) + k + 1] = pre[1 * (R + 1) + k] + (r.B + ra - 1) / ra;
            pre[2 * (R + 1) + k + 1] = pre[2 * (R + 1) + k] + (r.A + rb - 1) / rb;
            pre[3 * (R + 1) + k + 1] = pre[3 * (R + 1) + k] + (int32_t)((r.M + 255) / 256);   /* mid: storage order */
        }
        H.recs = recs;
        H.subs = subs;
        H.pre = pre;
        H.blu = blu;
        H.rad = rad;
        H.itab = itab;
        H.fbsz = fbsz;
        H.tabs = tabs;
        H.tabsz = tabsz;
        H.work = w;
        H.lds = lds;
        H.key = key;
        H.uploaded = false;
    }
    const size_t nrec = H.recs.size() * sizeof(LfRec), nsub = H.subs.size() * sizeof(LfSub);
    const size_t npre = H.pre.size() * 4, nblu = (std::max<size_t>(1, H.blu.size()) * 4 + 15) / 16 * 16;
    const size_t ndesc = H.tabs.size() * sizeof(LfTab);
    bool grew_m = false, grew_w = false, grew_b = false, grew_t = false;
    char *meta = (char *)ctx->buf("lf_meta", nrec + nsub + npre + nblu + ndesc + 64, &rc, &grew_m);
    double2 *tab = (double2 *)ctx->buf("lf_tab", (size_t)H.tabsz * sizeof(double2), &rc, &grew_t);
    bool grew_i = false;
    int32_t *itab = (int32_t *)ctx->buf("lf_itab", std::max<size_t>(1, H.itab.size()) * 4 + (H.rad.size() + 1) * 4,
                                        &rc, &grew_i);
    double2 *w1 = (double2 *)ctx->buf("lf_w", (size_t)H.work * 2 * sizeof(double2), &rc, &grew_w);
    double2 *fbt = (double2 *)ctx->buf("lf_fb", (size_t)std::max<int64_t>(1, H.fbsz) * sizeof(double2), &rc, &grew_b);
    if (rc != BPMX_OK) return rc;
    LfRec *d_rec = (LfRec *)meta;
    LfSub *d_sub = (LfSub *)(meta + nrec);
    int32_t *d_pre = (int32_t *)(meta + nrec + nsub);
    int32_t *d_blu = (int32_t *)(meta + nrec + nsub + npre);
    LfTab *d_desc = (LfTab *)(meta + nrec + nsub + npre + nblu);
    int32_t *d_rad = itab + std::max<size_t>(1, H.itab.size());
    if (!H.uploaded || grew_b || grew_m || grew_t || grew_i) {
        /* host vectors live in the context until the next plan, past these async copies */
        HIP_TRY(hipMemcpyAsync(d_rec, H.recs.data(), nrec, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_sub, H.subs.data(), nsub, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_pre, H.pre.data(), npre, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_desc, H.tabs.data(), ndesc, hipMemcpyHostToDevice, s));
        int32_t tmax = 0;
        for (const LfTab &t : H.tabs) tmax = std::max(tmax, t.count);
        LAUNCH(ctx, s, "k_lf_tab", k_lf_tab, dim3((unsigned)((tmax + 255) / 256), (unsigned)H.tabs.size()), dim3(256), 0,
               s, d_desc, tab);
        if (!H.rad.empty()) {
            HIP_TRY(hipMemcpyAsync(itab, H.itab.data(), H.itab.size() * 4, hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemcpyAsync(d_rad, H.rad.data(), H.rad.size() * 4, hipMemcpyHostToDevice, s));
            size_t bl = 0;
            for (int32_t i : H.rad) bl = std::max(bl, (size_t)2 * H.subs[i].L * sizeof(double2));
            (void)hipFuncSetAttribute((const void *)k_lf_rader_b, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bl);
            LAUNCH(ctx, s, "k_lf_rader_b", k_lf_rader_b, dim3((unsigned)H.rad.size()), dim3(LF_T), bl, s, d_sub, d_rad,
                   tab, itab, fbt);
        }
        if (!H.blu.empty()) {
            HIP_TRY(hipMemcpyAsync(d_blu, H.blu.data(), H.blu.size() * 4, hipMemcpyHostToDevice, s));
            size_t bl = 0;
            for (int32_t i : H.blu) bl = std::max(bl, (size_t)2 * H.subs[i].L * sizeof(double2));
            (void)hipFuncSetAttribute((const void *)k_lf_blu_b, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bl);
            LAUNCH(ctx, s, "k_lf_blu_b", k_lf_blu_b, dim3((unsigned)H.blu.size()), dim3(LF_T), bl, s, d_sub, d_blu, tab,
                   fbt);
        }
        H.uploaded = true;
    }
    LfArgs a;
    a.yd = yd; a.hb = hb; a.w1 = w1; a.w2 = w1 + H.work; a.fbt = fbt; a.tab = tab; a.itab = itab; a.rec = d_rec;
    a.sub = d_sub;
    a.R = R;
    const int32_t *P = H.pre.data();
    const unsigned ntile = (unsigned)P[R];
    const unsigned rows_of_A = (unsigned)P[1 * (R + 1) + R];   /* R1 / R1': B rows of A points */
    const unsigned rows_of_B = (unsigned)P[2 * (R + 1) + R];   /* R2 / R2': A rows of B points */
    const unsigned nmid = (unsigned)P[3 * (R + 1) + R];
    (void)hipFuncSetAttribute((const void *)k_lf_rows, hipFuncAttributeMaxDynamicSharedMemorySize, (int)H.lds);
    LfArgs at = a, ar1 = a, ar2 = a, am = a;
    at.pre = d_pre;
    ar1.pre = d_pre + (R + 1);
    ar2.pre = d_pre + 2 * (R + 1);
    am.pre = d_pre + 3 * (R + 1);
    LAUNCH(ctx, s, "k_lf_tr", k_lf_tr<1>, dim3(ntile), dim3(256), 0, s, at, (const double2 *)nullptr, a.w1, 0);
    LAUNCH(ctx, s, "k_lf_rows[A]", k_lf_rows, dim3(rows_of_A), dim3(LF_T), H.lds, s, ar1, a.w1, 1, -1, 1);
    LAUNCH(ctx, s, "k_lf_tr", k_lf_tr<0>, dim3(ntile), dim3(256), 0, s, at, (const double2 *)a.w1, a.w2, 1);
    LAUNCH(ctx, s, "k_lf_rows[B]", k_lf_rows, dim3(rows_of_B), dim3(LF_T), H.lds, s, ar2, a.w2, 0, -1, 0);
    LAUNCH(ctx, s, "k_lf_mid", k_lf_mid, dim3(nmid), dim3(256), 0, s, am);
    LAUNCH(ctx, s, "k_lf_rows[B]", k_lf_rows, dim3(rows_of_B), dim3(LF_T), H.lds, s, ar2, a.w2, 0, +1, 1);
    LAUNCH(ctx, s, "k_lf_tr", k_lf_tr<0>, dim3(ntile), dim3(256), 0, s, at, (const double2 *)a.w2, a.w1, 0);
    LAUNCH(ctx, s, "k_lf_rows[A]", k_lf_rows, dim3(rows_of_A), dim3(LF_T), H.lds, s, ar1, a.w1, 1, +1, 0);
    LAUNCH(ctx, s, "k_lf_tr", k_lf_tr<2>, dim3(ntile), dim3(256), 0, s, at, (const double2 *)a.w1, (double2 *)nullptr, 1);
    return BPMX_OK;
}

}  // namespace bpmx
