/*
 * k_floor.hip — the dynamic noise floor (bpm_analysis.py:1079-1115).
 *
 *   k_interp            reindex(arange(Nd)).interpolate() of the trough
 *                       samples == numpy arr_interp (slope*(x-x0)+y0), NaN
 *                       before the first trough.
 *   k_rolling_quantile  .rolling(W, min_periods=3, center=True).quantile(q)
 *                       .bfill().ffill() — exact order statistics.
 *   k_sanitize          keep trough t iff draft[t] is not NaN and
 *                       env[t] <= mult*draft[t] (:1090-1097), ordered.
 *   k_floor_final       static / draft / all-NaN fallbacks (:1073-1077,
 *                       :1107-1115).
 *
 * Rolling quantile design (one workgroup per recording, T outputs per step):
 * the union of the T windows of a tile is kept SORTED in LDS.  Moving to the
 * next tile removes the <= T oldest positions and merges the <= T newest
 * (ranked among themselves, then both sides placed by binary search: a
 * parallel merge, no full sort).  Output i of the tile excludes only "edge"
 * samples (left of its own window start or right of its end); those are
 * marked in a bitmap over the sorted order, and each thread walks that bitmap
 * from the low end to turn the window rank k into a sorted index: O(edges
 * below rank k) per output instead of O(W).  The window-validity count makes
 * min_periods / NaN handling exact, and because nobs(i) is unimodal in i the
 * NaN outputs are a prefix and a suffix, which bfill/ffill fill from the first
 * and last valid output.
 */
#include "bpmx_common.h"
#include "bpmx_kernels.h"

namespace bpmx {

__global__ __launch_bounds__(256) void k_interp(InterpArgs A) {
    const int f = blockIdx.y;
    if (f >= A.n_files || !A.run[f]) return;
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (x >= n) return;
    const int64_t *t = A.troughs + d0;
    const double *e = A.env + d0;
    const int m = A.ntr[f];
    double r;
    if (m == 0 || x < t[0]) {
        r = __builtin_nan("");
    } else {
        int lo = 0, hi = m;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (t[mid] <= x) lo = mid + 1; else hi = mid;
        }
        const int j = lo - 1;
        if (j == m - 1 || t[j] == x) {
            r = e[t[j]];
        } else {
            const double y0 = e[t[j]], y1 = e[t[j + 1]];
            const double slope = (y1 - y0) / ((double)t[j + 1] - (double)t[j]);
            r = slope * ((double)x - (double)t[j]) + y0;
            if (r != r) {
                r = slope * ((double)x - (double)t[j + 1]) + y1;
                if (r != r && y0 == y1) r = y0;
            }
        }
    }
    A.dense[d0 + x] = r;
}

/* ------------------------------------------------------------------------ */

__device__ __forceinline__ int lower_bound_lds(const double *a, int n, double v) {
    int lo = 0, hi = n;
    while (lo < hi) { int mid = (lo + hi) >> 1; if (a[mid] < v) lo = mid + 1; else hi = mid; }
    return lo;
}
__device__ __forceinline__ int upper_bound_lds(const double *a, int n, double v) {
    int lo = 0, hi = n;
    while (lo < hi) { int mid = (lo + hi) >> 1; if (a[mid] <= v) lo = mid + 1; else hi = mid; }
    return lo;
}

template <int T>
__global__ __launch_bounds__(T) void k_rolling_quantile(RollqArgs A) {
    const int f = blockIdx.x;
    if (f >= A.n_files || !A.run[f]) return;
    extern __shared__ __align__(16) unsigned char smem[];
    const int cap = A.cap;
    double *Av = (double *)smem;
    double *Bv = Av + cap;
    double *nv = Bv + cap;          /* [T] new values in position order */
    double *nsv = nv + T;           /* [T] new values sorted */
    unsigned long long *ebits = (unsigned long long *)(nsv + T);   /* [cap/64+2] */
    uint16_t *Ap = (uint16_t *)(ebits + cap / 64 + 2);
    uint16_t *Bp = Ap + cap;
    uint16_t *rem = Bp + cap;       /* [cap+1] exclusive prefix of removed flags */
    uint16_t *nsp = rem + cap + 4;  /* [T] positions of sorted new values */
    int *sh = (int *)(nsp + T + 4); /* scan scratch */
    __shared__ int s_first, s_last;

    const int tid = threadIdx.x, lane = lane_id();
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    const double *dense = A.dense + d0;
    double *out = A.out + d0;
    const int64_t W = A.window, minp = A.min_periods;
    const int64_t t0 = A.troughs[d0];
    const double q = A.q;
    if (tid == 0) { s_first = INT_MAX; s_last = -1; }

    int nA = 0;
    int64_t P0prev = 0, P1prev = 0;
    for (int64_t i0 = 0; i0 < n; i0 += T) {
        const int64_t i1 = i0 + T < n ? i0 + T : n;
        int64_t sA, eA, sB, eB;
        win_bounds(i0, n, W, sA, eA);
        win_bounds(i1 - 1, n, W, sB, eB);
        const int64_t P0 = sA > t0 ? sA : t0;
        const int64_t P1 = eB > P0 ? eB : P0;
        /* ---- removal of positions < P0 ---- */
        bool pending_rem = false;
        if (nA > 0 && P0 > P0prev) {
            if (P0 >= P1prev) {
                nA = 0;
            } else {
                pending_rem = true;
                const int cut = (int)(P0 - P0prev);
                const uint16_t b16 = (uint16_t)P0prev;
                const int ch = (nA + T - 1) / T;
                const int j0 = tid * ch, j1 = j0 + ch < nA ? j0 + ch : nA;
                int cnt = 0;
                for (int j = j0; j < j1; ++j) cnt += ((uint16_t)(Ap[j] - b16) < cut) ? 1 : 0;
                int tot;
                int pre = block_scan_int<T>(cnt, sh, &tot);
                for (int j = j0; j < j1; ++j) {
                    rem[j] = (uint16_t)pre;
                    pre += ((uint16_t)(Ap[j] - b16) < cut) ? 1 : 0;
                }
                if (tid == 0) rem[nA] = (uint16_t)tot;
                __syncthreads();
            }
        }
        /* ---- insert new positions [max(P1prev,P0), P1) in chunks of T ---- */
        int64_t a = P1prev > P0 ? P1prev : P0;
        const uint16_t b16 = (uint16_t)P0prev;
        const int cut = (int)(P0 - P0prev);
        do {
            const int64_t b = a + T < P1 ? a + T : P1;
            const int nn = b > a ? (int)(b - a) : 0;
            if (nn == 0 && !pending_rem) break;
            double v = 0;
            if (tid < nn) { v = dense[a + tid]; nv[tid] = v; }
            __syncthreads();
            if (tid < nn) {
                int r = 0;
                for (int u = 0; u < nn; ++u) {
                    const double w = nv[u];
                    r += (w < v || (w == v && u < tid)) ? 1 : 0;
                }
                nsv[r] = v;
                nsp[r] = (uint16_t)(a + tid);
            }
            __syncthreads();
            int kept = nA;
            if (pending_rem) kept = nA - rem[nA];
            for (int j = tid; j < nA; j += T) {
                int kb = j;
                if (pending_rem) {
                    if ((uint16_t)(Ap[j] - b16) < cut) continue;
                    kb = j - rem[j];
                }
                const double ov = Av[j];
                const int dst = kb + lower_bound_lds(nsv, nn, ov);
                Bv[dst] = ov;
                Bp[dst] = Ap[j];
            }
            if (tid < nn) {
                const double w = nsv[tid];
                const int ub = upper_bound_lds(Av, nA, w);
                const int kb = pending_rem ? ub - rem[ub] : ub;
                Bv[tid + kb] = w;
                Bp[tid + kb] = nsp[tid];
            }
            __syncthreads();
            { double *tv = Av; Av = Bv; Bv = tv; uint16_t *tp = Ap; Ap = Bp; Bp = tp; }
            nA = kept + nn;
            pending_rem = false;
            a = b;
        } while (a < P1);
        P0prev = P0;
        P1prev = P1 > P1prev ? P1 : P1prev;

        /* ---- edge bitmap over the sorted union ---- */
        const int64_t LE = sB > t0 ? sB : t0;   /* left edge: positions < LE may be excluded */
        const int64_t RE = eA;                   /* right edge: positions >= RE may be excluded */
        const int relLE = (int)(LE - P0), relRE = (int)(RE - P0);
        const uint16_t p16 = (uint16_t)P0;
        const int nwords = (nA + 63) >> 6;
        for (int w = wave_id(); w < nwords; w += T / 64) {
            const int j = (w << 6) + lane;
            bool bit = false;
            if (j < nA) {
                const int rel = (uint16_t)(Ap[j] - p16);
                bit = rel < relLE || rel >= relRE;
            }
            const unsigned long long word = __ballot(bit);
            if (lane == 0) ebits[w] = word;
        }
        __syncthreads();

        /* ---- one output per thread ---- */
        const int64_t i = i0 + tid;
        if (i < i1) {
            int64_t s, e;
            win_bounds(i, n, W, s, e);
            const int64_t lo = s > t0 ? s : t0;
            const int64_t nobs = e > lo ? e - lo : 0;
            double res = __builtin_nan("");
            if (nobs >= minp && nobs > 0) {
                const int xlo = (int)(lo - P0), xhi = (int)(e - P0);
                int64_t k;
                double idxf = 0;
                bool interp = false;
                if (nobs == 1) {
                    k = 0;
                } else {
                    idxf = q * (double)(nobs - 1);
                    k = (int64_t)idxf;
                    interp = (double)k != idxf;
                }
                /* walk the edge bitmap: first the k-th valid sorted index */
                int qa = (int)k;
                int w = 0;
                unsigned long long bits = nwords > 0 ? ebits[0] : 0ull;
                for (;;) {
                    while (bits == 0ull && w + 1 < nwords) bits = ebits[++w];
                    if (bits == 0ull) break;
                    const int j = (w << 6) + __ffsll((long long)bits) - 1;
                    if (j > qa) break;
                    const int rel = (uint16_t)(Ap[j] - p16);
                    if (rel < xlo || rel >= xhi) qa++;
                    bits &= bits - 1ull;
                }
                const double va = Av[qa];
                if (!interp) {
                    res = va;
                } else {
                    int qb = qa + 1;
                    for (;;) {
                        while (bits == 0ull && w + 1 < nwords) bits = ebits[++w];
                        if (bits == 0ull) break;
                        const int j = (w << 6) + __ffsll((long long)bits) - 1;
                        if (j > qb) break;
                        const int rel = (uint16_t)(Ap[j] - p16);
                        if (j == qb && (rel < xlo || rel >= xhi)) qb++;
                        bits &= bits - 1ull;
                    }
                    const double vb = Av[qb];
                    res = va + (vb - va) * (idxf - (double)k);
                }
                atomicMin(&s_first, (int)i);
                atomicMax(&s_last, (int)i);
            }
            out[i] = res;
        }
        __syncthreads();
    }
    /* ---- .bfill().ffill() ---- */
    const int first = s_first, last = s_last;
    if (last < 0) {
        if (tid == 0) A.allnan[f] = 1;
        return;
    }
    if (tid == 0) A.allnan[f] = 0;
    const double vf = out[first], vl = out[last];
    for (int64_t i = tid; i < first; i += T) out[i] = vf;
    for (int64_t i = last + 1 + tid; i < n; i += T) out[i] = vl;
}

template __global__ void k_rolling_quantile<256>(RollqArgs A);
template __global__ void k_rolling_quantile<128>(RollqArgs A);

/* ------------------------------------------------------------------------ */
__global__ __launch_bounds__(256) void k_sanitize(SanitizeArgs A) {
    const int f = blockIdx.x;
    if (f >= A.n_files || !A.active[f]) return;
    __shared__ int sh[256 / 64 + 1];
    const int64_t d0 = A.doff[f];
    const int64_t *raw = A.raw + d0;
    int64_t *out = A.out + d0;
    const int m = A.nraw[f];
    const int tid = threadIdx.x;
    if (m < 5) {
        for (int j = tid; j < m; j += 256) out[j] = raw[j];
        if (tid == 0) { A.nout[f] = m; A.flags[f] |= BPMX_F_STATIC_FLOOR; A.run2[f] = 0; }
        return;
    }
    const double *env = A.env + d0, *draft = A.draft + d0;
    int w = 0;
    for (int c0 = 0; c0 < m; c0 += 256) {
        const int j = c0 + tid;
        bool keep = false;
        int64_t t = 0;
        if (j < m) {
            t = raw[j];
            const double fl = draft[t];
            keep = (fl == fl) && env[t] <= A.mult * fl;
        }
        int tot;
        const int off = block_scan_flag<256>(keep, sh, &tot);
        if (keep) out[w + off] = t;
        w += tot;
    }
    if (tid == 0) {
        A.nout[f] = w;
        if (w <= 2) A.flags[f] |= BPMX_F_DRAFT_FLOOR;
        A.run2[f] = w > 2 ? 1 : 0;
    }
}

__global__ __launch_bounds__(256) void k_floor_final(FinalArgs A) {
    const int f = blockIdx.y;
    if (f >= A.n_files || !A.active[f]) return;
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int fl = A.flags[f];
    const double *qv = A.qv + (int64_t)f * Q_SLOTS;
    bool nanfb = false;
    double v;
    if (fl & BPMX_F_STATIC_FLOOR) {
        v = qv[Q_NOISE];
    } else if (fl & BPMX_F_DRAFT_FLOOR) {
        nanfb = A.allnan_draft[f] != 0;
        v = nanfb ? qv[Q_FALLBACK] : (i < n ? A.draft[d0 + i] : 0.0);
    } else {
        nanfb = A.allnan_final[f] != 0;
        if (!nanfb) return;   /* floor already written by the second rolling pass */
        v = qv[Q_FALLBACK];
    }
    if (i < n) A.floor[d0 + i] = v;
    if (i == 0 && nanfb) A.flags[f] = fl | BPMX_F_NAN_FLOOR;
}

}  // namespace bpmx
