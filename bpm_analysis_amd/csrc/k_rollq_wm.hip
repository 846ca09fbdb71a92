/*
 * k_rollq_wm.hip — centred rolling quantile by a per-recording wavelet matrix
 * (bpm_analysis.py:1084-1086 / :1104-1106:
 *  .rolling(W, min_periods=3, center=True).quantile(q).bfill().ffill()).
 *
 * One 1024-thread workgroup per recording, everything in LDS:
 *   0. (pruned variant) only samples that can be some window's k-th or
 *      (k+1)-th smallest enter the structure.  Values are put in 64 monotone
 *      bins; per block of 64 outputs, the bin b* holding the (k_max+1)-th
 *      smallest sample of the block's common window (the intersection of its
 *      64 windows, full 64-sample position blocks only) bounds every one of
 *      its windows' (k+1)-th smallest from above.  A sample whose bin exceeds
 *      b* of every block whose windows can contain it is strictly greater than
 *      each such window's (k+1)-th smallest, so dropping it changes no output;
 *      the window's k-th smallest is the k-th smallest of its kept samples.
 *      The lower side likewise: a* = the bin of the k_min-th smallest of the
 *      position blocks covering the block's windows' union bounds every one of
 *      its windows' k-th smallest from below, so a sample below a* of every
 *      block whose windows can contain it ranks before the window's k-th and
 *      (k+1)-th smallest; such samples are only counted (a second mask +
 *      prefix), and the window's k-th smallest is the (k - low count)-th of its
 *      kept samples.
 *      Kept samples are compacted (a per-64 bit mask + prefix maps a position
 *      range to a kept range).  On the metric workload ~19 % are kept (31 %
 *      with the upper bound alone, tools/prune_sim.py).
 *      Recordings keeping more than WM_PMAX take the unpruned variant.
 *   1. ranks: the kept samples are ordered by (value, index) with an LSD radix
 *      sort on order-preserving 64-bit keys, 8-bit digits, digits constant
 *      over the recording skipped.  What moves is only the 16-bit index
 *      (ping-pong in LDS); the current 32-bit key half sits in LDS indexed by
 *      index (low halves for digits 0-3, then high halves).  Slots are
 *      wave-contiguous, so a stable rank is: per-wave digit counter (LDS
 *      atomic, issued in slot order) + peers below in the same round (ballot
 *      match) + one (digit, wave) block scan.
 *   2. outputs, 64 consecutive ones per wave step: a rank cursor moved from
 *      block to block, the block's candidate members collected from it in rank
 *      order until every lane's k-th / (k+1)-th own member is among them, each
 *      lane skipping the few members its window misses (details at the phase).  pandas' linear
 *      interpolation, nobs / min_periods from the window bounds.  NaN outputs
 *      are a prefix and a suffix (nobs is unimodal), filled from the first and
 *      last valid output.  (r01-r03 answered every output by a top-down descent
 *      of a wavelet matrix over the rank sequence; building its levels and the
 *      descents cost more than the whole of this phase.)
 * Recordings longer than WM_MMAX decimated samples take k_rolling_quantile.
 */
#include "bpmx_common.h"
#include "bpmx_kernels.h"
#include "bpmx_stamps.h"
#include "bpmx_qsel.h"

namespace bpmx {

__device__ __forceinline__ uint64_t wm_key(double v) {
    return f64_key(v == 0.0 ? 0.0 : v);      /* -0.0 == +0.0 for the quantile */
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    return (1ull << lane_id()) - 1ull;
}

/* lanes holding the same 8-bit digit as this lane */
__device__ __forceinline__ uint64_t match8(uint32_t dg) {
    uint64_t m = ~0ull;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const uint64_t bal = __ballot((dg >> b) & 1u);
        m &= ((dg >> b) & 1u) ? bal : ~bal;
    }
    return m;
}

/* returns true (uniformly) when a recording the pruned variant cannot take
 * must be redone unpruned */
struct RqShared {
    int jlo, jhi, first, last, wt[WM_T / 64], mk;
    unsigned long long orv[WM_T / 64], andv[WM_T / 64];
    double vmin, vmax;
};

template <bool PRUNE>
__device__ __forceinline__ bool rollq_wm_body(RollqArgs A, uint16_t *pos_scratch, int32_t *full, RqShared &S_) {
    constexpr int NWV = WM_T / 64;
    constexpr int MMAX = PRUNE ? WM_PMAX : WM_MMAX;          /* samples in the structure */
    constexpr int MAXIT = MMAX / WM_T;
    const int f = blockIdx.x;
    if (f >= A.n_files) return false;
    const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
    if (!A.run[f]) {
        if (PRUNE && tid == 0) full[f] = 0;
        return false;
    }
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    const int ntr_all = A.env ? A.ntr[f] : 0;
    /* chunk mode: a long recording's outputs [o0, o1) in workgroup (f, chunk),
     * over the samples [t0, top) their windows reach */
    const bool chunked = PRUNE && A.wm_chunk > 0 && n > WM_MMAX && A.env;
    if (!chunked && blockIdx.y > 0) return false;
    const int64_t W = A.window, minp = A.min_periods;
    int64_t o0 = 0, o1 = n, t0 = 0, top = n;
    int jlo = 0, ntr = ntr_all;                              /* troughs staged: [jlo, jlo + ntr) */
    int &s_jlo = S_.jlo, &s_jhi = S_.jhi;
    if (chunked) {
        if (tid == 0 && blockIdx.y == 0) full[f] = 0;        /* long: never the unpruned variant */
        o0 = (int64_t)blockIdx.y * A.wm_chunk;
        if (o0 >= n) return false;
        o1 = min<int64_t>(n, o0 + A.wm_chunk);
        int64_t s, e;
        win_bounds(o0, n, W, s, e);
        const int64_t *tr = A.troughs + d0;
        t0 = s > tr[0] ? s : tr[0];                          /* every chunk window lies in [t0, top) */
        win_bounds(o1 - 1, n, W, s, e);
        top = e;
        if (tid == 0) {                                      /* last trough <= t0, first trough >= top - 1 */
            int lo = 0, hi = ntr_all;
            while (lo < hi) { const int mid = (lo + hi) >> 1; if (tr[mid] <= t0) lo = mid + 1; else hi = mid; }
            s_jlo = lo > 0 ? lo - 1 : 0;
            lo = 0; hi = ntr_all;
            while (lo < hi) { const int mid = (lo + hi) >> 1; if (tr[mid] < top - 1) lo = mid + 1; else hi = mid; }
            s_jhi = lo < ntr_all ? lo : ntr_all - 1;
        }
        __syncthreads();
        jlo = s_jlo;
        ntr = s_jhi - s_jlo + 1;
        if (top <= t0) {                                     /* no finite sample in reach: NaN outputs */
            for (int64_t i = o0 + tid; i < o1; i += WM_T) A.out[d0 + i] = __builtin_nan("");
            return false;
        }
        if (top - t0 > WM_MMAX || ntr > WM_TRMAX) {
            if (tid == 0) A.wm_fail[f] = 1;
            return false;
        }
    }
    const bool fused = A.env && ntr <= WM_TRMAX;
    if (!chunked && (n > WM_MMAX || n <= 0 || (PRUNE && !fused))) {   /* k_rolling_quantile / the unpruned variant */
        if (PRUNE && tid == 0) full[f] = (n <= WM_MMAX && n > 0) ? 1 : 0;
        return PRUNE && n <= WM_MMAX && n > 0;
    }
    extern __shared__ __align__(16) unsigned char smem[];
    int &s_first = S_.first, &s_last = S_.last, *s_wt = S_.wt, &s_mk = S_.mk;
    unsigned long long *s_or = S_.orv, *s_and = S_.andv;
    double &s_vmin = S_.vmin, &s_vmax = S_.vmax;

    const double *dense = A.dense + d0;
    double *out = A.out + d0;
    (void)pos_scratch;
    if (!chunked) t0 = A.troughs[d0];
    const int mall = (int)(top - t0);                        /* finite samples dense[t0:top) */
    const WmLayout Lay = wm_layout(chunked ? top - t0 : n, PRUNE);
    if (tid == 0) { s_first = INT_MAX; s_last = -1; }
    STAMP_DECL

    /* dense = np.interp of the troughs (k_interp), evaluated here from env at
     * the troughs staged in LDS when there are <= WM_TRMAX of them */
    double *s_tv = (double *)(smem + Lay.tab);
    double *s_sl = s_tv + WM_TRMAX;                          /* per-segment slope (pruned variant) */
    int32_t *s_tp = (int32_t *)(s_sl + (PRUNE ? WM_TRMAX : 0));
    int32_t *s_bj = s_tp + WM_TRMAX;                         /* [(top - xb)/64 + 1]: last trough <= block start */
    const int64_t xb = chunked ? t0 : 0;                     /* block table origin */
    if (fused) {
        const int64_t *tr = A.troughs + d0 + jlo;
        const double *trv = A.tv + d0 + jlo;                 /* env at the troughs, beside them */
        for (int j = tid; j < ntr; j += WM_T) {
            s_tp[j] = (int32_t)tr[j];
            s_tv[j] = trv[j];
        }
        __syncthreads();
        for (int64_t b = tid; b <= ((top - xb) >> 6); b += WM_T) {
            int lo = 0, hi = ntr;
            while (lo < hi) { const int mid = (lo + hi) >> 1; if (s_tp[mid] <= xb + (b << 6)) lo = mid + 1; else hi = mid; }
            s_bj[b] = lo - 1;
        }
        if (PRUNE) {
            /* the same slope interp_at computes, once per segment */
            for (int j = tid; j + 1 < ntr; j += WM_T)
                s_sl[j] = (s_tv[j + 1] - s_tv[j]) / ((double)s_tp[j + 1] - (double)s_tp[j]);
        }
        __syncthreads();
    }
    /* interp_at's arithmetic, with the bracketing trough found from the block
     * table (a staged run that stops before the recording's last trough always
     * reaches past every position asked for) */
    auto dval = [&](int64_t x) -> double {
        if (!fused) {                                        /* > WM_TRMAX troughs: np.interp from global memory */
            if (!A.env) return dense[x];
            const int64_t *trg = A.troughs + d0;
            return interp_at(x, trg, [&](int j) { return A.tv[d0 + j]; }, ntr_all);
        }
        const int xi = (int)x;                               /* positions < 2^31 (host check): 32-bit arithmetic */
        if (ntr == 0 || xi < s_tp[0]) return __builtin_nan("");
        int j = s_bj[(xi - (int)xb) >> 6];
        if (j < 0) j = 0;
        while (j + 1 < ntr && s_tp[j + 1] <= xi) ++j;
        if (j == ntr - 1 || s_tp[j] == xi) return s_tv[j];
        const double y0 = s_tv[j], y1 = s_tv[j + 1];
        const double slope = PRUNE ? s_sl[j] : (y1 - y0) / ((double)s_tp[j + 1] - (double)s_tp[j]);
        double r = slope * ((double)xi - (double)s_tp[j]) + y0;
        if (r != r) {
            r = slope * ((double)xi - (double)s_tp[j + 1]) + y1;
            if (r != r && y0 == y1) r = y0;
        }
        return r;
    };

    const double q = A.q;

    /* ---------------- 0. pruning (PRUNE only) ---------------- */
    const int NPB = (mall + 63) >> 6;                        /* 64-sample position blocks of dense[t0:n) */
    uint64_t *kmask = (uint64_t *)(smem + Lay.meta);         /* [NPB + 1] kept bits */
    int32_t *kpre = (int32_t *)(kmask + (WM_MMAX / 64 + 2)); /* [NPB + 1] kept before the block */
    uint8_t *thr = (uint8_t *)(kpre + (WM_MMAX / 64 + 2));   /* [NPB] highest bin kept */
    uint8_t *bstar = thr + (WM_MMAX / 64 + 2);               /* [9][n/64] per output block, then sparse-table maxima */
    /* the lower side: samples below every reachable window's k-th smallest */
    uint64_t *lmask = (uint64_t *)(smem + Lay.meta + WM_META_LOW);         /* [NPB + 1] low bits */
    int32_t *lpre = (int32_t *)(lmask + (WM_MMAX / 64 + 2)); /* [NPB + 1] low samples before the block */
    uint8_t *lthr = (uint8_t *)(lpre + (WM_MMAX / 64 + 2));  /* [NPB] lowest bin kept */
    uint8_t *astar = lthr + (WM_MMAX / 64 + 2);              /* [9][n/64] per output block, then sparse-table minima */
    uint16_t *kpos = (uint16_t *)(smem + Lay.kpos);          /* kept index -> position - t0 */
    int m = mall;
    if (PRUNE) {
        constexpr int NB = 64;
        STAMP(8);
        /* value range of the curve = range of the trough values (interpolation
         * stays between segment ends up to rounding; the bins clamp) */
        {
            double lo = __builtin_inf(), hi = -__builtin_inf();
            for (int j = tid; j < ntr; j += WM_T) { lo = fmin(lo, s_tv[j]); hi = fmax(hi, s_tv[j]); }
            lo = wave_min(lo);
            hi = wave_max(hi);
            if (lane == 0) { s_or[wid] = (unsigned long long)__double_as_longlong(lo); s_and[wid] = (unsigned long long)__double_as_longlong(hi); }
            __syncthreads();
            if (tid == 0) {
                for (int w = 0; w < NWV; ++w) {
                    lo = fmin(lo, __longlong_as_double((long long)s_or[w]));
                    hi = fmax(hi, __longlong_as_double((long long)s_and[w]));
                }
                s_vmin = lo;
                s_vmax = hi;
            }
        }
        uint16_t *hist = (uint16_t *)(smem + Lay.area);      /* [NPB + 1][NB], then the exclusive prefix over blocks */
        int32_t *hsc = (int32_t *)(hist + (WM_MMAX / 64 + 2) * NB);   /* [NWV][NB] */
        for (int j = tid; j < (NPB + 1) * NB / 2; j += WM_T) ((uint32_t *)hist)[j] = 0u;
        __syncthreads();
        const double vmin = s_vmin, span = s_vmax - s_vmin;
        const bool ok = span == span && span < __builtin_inf();
        if (!ok) {                                           /* non-finite curve: no pruning */
            if (tid == 0) { if (chunked) A.wm_fail[f] = 1; else full[f] = 1; }
            return !chunked;
        }
        const double scale = span > 0.0 ? (double)NB / span : 0.0;
        /* monotone in the value: (v - vmin) * scale rounds monotonically, the
         * truncation and the clamp are monotone */
        auto vbin = [&](double v) -> int {
            const double t = (v - vmin) * scale;
            int b = t > 0.0 ? (int)fmin(t, (double)(NB - 1)) : 0;
            return b;
        };
        uint8_t *bin8 = (uint8_t *)(hsc + NWV * NB);        /* [mall] bin of each sample */
        /* one 64-sample block per wave step: runs of equal bins (the curve is
         * piecewise monotone, so a block has few) each add their length */
        for (int p0 = wid << 6; p0 < mall; p0 += WM_T) {
            const int p = p0 + lane, nv = min(64, mall - p0);
            const int b = p < mall ? vbin(dval(t0 + p)) : -1;
            if (p < mall) bin8[p] = (uint8_t)b;
            const int bprev = wave_shr1_dpp(b, -1);          /* all lanes active here */
            const bool start = b >= 0 && (lane == 0 || bprev != b);
            const uint64_t sm = __ballot(start);
            const uint64_t after = sm & ~((2ull << lane) - 1ull);
            const int nxt = after ? __ffsll((long long)after) - 1 : nv;
            if (start) atomicAdd((uint32_t *)hist + (((p0 >> 6) * NB + b) >> 1), (uint32_t)(nxt - lane) << (16 * (b & 1)));
        }
        __syncthreads();
        STAMP(9);
        /* exclusive prefix over position blocks, per bin: 16 parts of rows */
        {
            const int b = tid & (NB - 1), g = tid >> 6;
            constexpr int RPMAX = (WM_MMAX / 64 + 1 + NWV - 1) / NWV;
            const int rp = (NPB + NWV - 1) / NWV, r0 = g * rp, r1 = min(NPB, r0 + rp);
            int hv[RPMAX], sum = 0;
#pragma unroll
            for (int u = 0; u < RPMAX; ++u) {
                hv[u] = r0 + u < r1 ? (int)hist[(r0 + u) * NB + b] : 0;
                sum += hv[u];
            }
            hsc[g * NB + b] = sum;
            __syncthreads();
            int run = 0;
            for (int h = 0; h < g; ++h) run += hsc[h * NB + b];
#pragma unroll
            for (int u = 0; u < RPMAX; ++u) {
                if (r0 + u < r1) hist[(r0 + u) * NB + b] = (uint16_t)run;
                run += hv[u];
            }
            if (g == NWV - 1) {
                int tot = 0;
                for (int h = 0; h < NWV; ++h) tot += hsc[h * NB + b];
                hist[NPB * NB + b] = (uint16_t)tot;
            }
        }
        __syncthreads();
        STAMP(10);
        /* cumulative over bins too: hist[r][b] = samples of blocks < r with bin <= b */
        for (int r = wid; r <= NPB; r += NWV) {
            const int v = wave_iscan_dpp<false>((int)hist[r * NB + lane]);
            hist[r * NB + lane] = (uint16_t)v;
        }
        __syncthreads();
        /* b* per block of 64 outputs, one thread per block: the lowest bin
         * with >= k_max + 2 samples of the block's common window (full
         * position blocks only) at or below it, by binary search */
        const int NBO = (int)((o1 - o0 + 63) >> 6);
        for (int B = tid; B < NBO; B += WM_T) {
            const int64_t ib = o0 + ((int64_t)B << 6), ie = min<int64_t>(o1, ib + 64) - 1;
            int64_t s0, e0, s1, e1;
            win_bounds(ib, n, W, s0, e0);
            win_bounds(ie, n, W, s1, e1);
            /* every window of the block holds <= min(W, e(ie) - max(s(ib), t0)) samples */
            int64_t nb = e1 - (s0 > t0 ? s0 : t0);
            nb = nb < W ? nb : W;
            const int kq = nb > 1 ? (int)(int64_t)(q * (double)(nb - 1)) : 0;
            const int64_t clo = (s1 > t0 ? s1 : t0) - t0, chi = e0 - t0;   /* common window, relative */
            const int pbs = (int)((clo + 63) >> 6), pbe = chi > 0 ? (int)(chi >> 6) : 0;
            int bs = NB - 1;
            if (pbe > pbs && (int)hist[pbe * NB + NB - 1] - (int)hist[pbs * NB + NB - 1] >= kq + 2) {
                int lo = 0, hi = NB - 1;                     /* count(<= hi) reaches */
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if ((int)hist[pbe * NB + mid] - (int)hist[pbs * NB + mid] >= kq + 2) hi = mid; else lo = mid + 1;
                }
                bs = lo;
            }
            bstar[B] = (uint8_t)bs;
            /* a*: the bin of the k_min-th smallest of the position blocks
             * covering the block's windows' union (a superset of every window,
             * so that sample is at most each window's k-th smallest; k_min from
             * the fewest observations, at an end of the block: nobs is unimodal).
             * A sample in a lower bin is strictly below every such window's k-th
             * smallest: it leaves the structure and is only counted. */
            const int64_t nl = e0 - (s0 > t0 ? s0 : t0), nr = e1 - (s1 > t0 ? s1 : t0);
            const int64_t nmin = nl < nr ? nl : nr;
            const int kmin = nmin > 1 ? (int)(int64_t)(q * (double)(nmin - 1)) : 0;
            const int64_t ulo = (s0 > t0 ? s0 : t0) - t0, uhi = e1 - t0;   /* union, relative */
            const int cbs = ulo > 0 ? (int)(ulo >> 6) : 0;
            const int cbe = uhi > 0 ? min(NPB, (int)((uhi + 63) >> 6)) : 0;
            int as = 0;
            if (cbe > cbs && nmin > 0 && (int)hist[cbe * NB + NB - 1] - (int)hist[cbs * NB + NB - 1] >= kmin + 1) {
                int lo = 0, hi = NB - 1;                     /* count(<= hi) reaches k_min + 1 */
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if ((int)hist[cbe * NB + mid] - (int)hist[cbs * NB + mid] >= kmin + 1) hi = mid; else lo = mid + 1;
                }
                as = lo;
            }
            astar[B] = (uint8_t)as;
        }
        __syncthreads();
        /* sparse table of b* maxima over 2^j consecutive blocks, j = 1 .. 8 */
        for (int j = 1; (1 << j) <= NBO; ++j) {
            const uint8_t *src = bstar + (size_t)(j - 1) * (WM_MMAX / 64 + 2);
            uint8_t *dst = bstar + (size_t)j * (WM_MMAX / 64 + 2);
            for (int B = tid; B + (1 << j) <= NBO; B += WM_T) dst[B] = max(src[B], src[B + (1 << (j - 1))]);
            const uint8_t *asrc = astar + (size_t)(j - 1) * (WM_MMAX / 64 + 2);
            uint8_t *adst = astar + (size_t)j * (WM_MMAX / 64 + 2);
            for (int B = tid; B + (1 << j) <= NBO; B += WM_T) adst[B] = min(asrc[B], asrc[B + (1 << (j - 1))]);
            __syncthreads();
        }
        STAMP(11);
        /* highest b* and lowest a* over the output blocks whose windows can
         * reach a position block */
        const int64_t off = (W - 1) / 2;
        for (int pb = tid; pb < NPB; pb += WM_T) {
            const int64_t a = t0 + ((int64_t)pb << 6);
            int64_t ilo = a - off > 0 ? a - off : 0;
            int64_t ihi = min<int64_t>(n - 1, a + 63 + W - off);
            if (ihi >= n - 1 - off) ihi = n - 1;             /* windows clamped at n are all alike */
            ilo = ilo > o0 ? ilo : o0;                       /* this workgroup's outputs only */
            ihi = ihi < o1 - 1 ? ihi : o1 - 1;
            if (ihi < ilo) { thr[pb] = 0; lthr[pb] = NB; continue; }   /* no window here reaches it */
            const int B0 = (int)((ilo - o0) >> 6), B1 = (int)((ihi - o0) >> 6), len = B1 - B0 + 1;
            const int j = 31 - __clz(len);
            const uint8_t *st = bstar + (size_t)j * (WM_MMAX / 64 + 2);
            thr[pb] = max(st[B0], st[B1 - (1 << j) + 1]);
            const uint8_t *sa = astar + (size_t)j * (WM_MMAX / 64 + 2);
            lthr[pb] = min(sa[B0], sa[B1 - (1 << j) + 1]);
        }
        __syncthreads();
        STAMP(12);
        /* keep and low masks, one 64-sample block per wave step */
        int kc = 0;
        for (int pb = wid; pb < NPB; pb += NWV) {
            const int p = (pb << 6) + lane;
            const int b = p < mall ? (int)bin8[p] : -1;
            const bool low = p < mall && b < (int)lthr[pb];
            const bool keep = p < mall && !low && b <= (int)thr[pb];
            const uint64_t bal = __ballot(keep), lbal = __ballot(low);
            if (lane == 0) { kmask[pb] = bal; lmask[pb] = lbal; }
        }
        if (tid == 0) { kmask[NPB] = 0ull; lmask[NPB] = 0ull; }
        __syncthreads();
        /* exclusive prefixes of kept (wave 0) and low (wave 1) counts over
         * blocks (NPB <= 289) */
        if (wid < 2) {
            const uint64_t *msk = wid ? lmask : kmask;
            int32_t *pre = wid ? lpre : kpre;
            int run = 0;
            for (int base = 0; base < NPB; base += 64) {
                const int pb = base + lane;
                const int v = pb < NPB ? __popcll(msk[pb]) : 0;
                int x = v;
                for (int o = 1; o < 64; o <<= 1) {
                    const int y = __shfl_up(x, o);
                    if (lane >= o) x += y;
                }
                if (pb < NPB) pre[pb] = run + x - v;
                run += __shfl(x, 63);
            }
            if (lane == 0) {
                pre[NPB] = run;
                if (!wid) s_mk = run;
            }
        }
        __syncthreads();
        kc = s_mk;
        STAMP(13);
        if (kc > WM_PMAX) {                                  /* too many kept: the unpruned variant */
            if (tid == 0) { if (chunked) A.wm_fail[f] = 1; else full[f] = 1; }
            return !chunked;
        }
        if (tid == 0 && !chunked) full[f] = 0;
        for (int pb = wid; pb < NPB; pb += NWV) {
            const uint64_t mk = kmask[pb];
            if ((mk >> lane) & 1) kpos[kpre[pb] + __popcll(mk & lanemask_lt())] = (uint16_t)((pb << 6) + lane);
        }
        m = kc;
        __syncthreads();
    }
#ifdef RQ_STOP_PRUNE
    return false;                                            /* tools/rqbench phase-truncated diagnostic builds */
#endif
    /* relative position of the c-th sample in the structure */
    auto spos = [&](int c) -> int { return PRUNE ? (int)kpos[c] : c; };
    /* structure index range of relative positions [0, p) */
    auto kidx = [&](int p) -> int {
        if (!PRUNE) return p;
        const uint64_t mk = kmask[p >> 6];
        return kpre[p >> 6] + __popcll(mk & ((1ull << (p & 63)) - 1ull));
    };
    /* samples below the structure among relative positions [0, p) */
    auto lidx = [&](int p) -> int {
        const uint64_t mk = lmask[p >> 6];
        return lpre[p >> 6] + __popcll(mk & ((1ull << (p & 63)) - 1ull));
    };
    STAMP(7);
#ifdef RQ_DIAG_M
    if (threadIdx.x == 0) _st_acc[13] = (unsigned long long)m;   /* diagnostics: kept samples */
#endif

    /* LDS, sort phase: posA[m8] | posB[m8] | kh[m8] | cnt[NWV][128] (two 16-bit counters per word).
     * Slots >= m are padding: they sort last, so they are neither stored nor counted. */
    const int IT = (m + WM_T - 1) / WM_T;                    /* rounds per wave */
    const int mu = __builtin_amdgcn_readfirstlane(m), ITu = __builtin_amdgcn_readfirstlane(IT);
    const int S = 64 * IT;                                   /* slots per wave */
    const int m8 = (m + 7) & ~7;
    uint16_t *posA = (uint16_t *)(smem + Lay.area);
    uint16_t *posB = posA + m8;
    uint32_t *kh = (uint32_t *)(posB + m8);
    uint32_t *cnt = kh + m8;
    /* per-wave digit bins for the peer masks (lanes with this lane's digit):
     * each valid lane ORs its bit into its digit's bin and reads the bin back
     * (three LDS instructions instead of eight ballots and ~48 VALU per item);
     * past the counters while they fit, else match8 */
    const size_t wbin_off = (size_t)8 * m8 + (size_t)NWV * 128 * 4;
    unsigned long long *wbin_all =
        wbin_off + (size_t)NWV * 256 * 8 <= Lay.total - Lay.area ? (unsigned long long *)(smem + Lay.area + wbin_off) : nullptr;

    /* ---------------- 1. ranks by LSD radix sort ----------------
     * Keys: the order-preserving 64-bit key minus the curve's lowest key,
     * shifted right so that it spans at most 40 bits (five 8-bit digits
     * instead of the seven a span of a few octaves takes).  Distinct values
     * closer than the shift could share a compact key and keep index order;
     * the sorted values are checked afterwards and any descent hands the
     * recording to the unpruned variant (full-width keys), as too many kept
     * samples do. */
    const size_t wsc = ((size_t)4 * m8 + 15) & ~(size_t)15;
    const size_t svl_off = wsc + (size_t)NWV * WM_WSCR * 4;
    double *svl = svl_off + (size_t)8 * m <= Lay.total - Lay.area ? (double *)(smem + Lay.area + svl_off) : nullptr;
    uint64_t kbase = 0;
    int shc = 0;
    if (PRUNE && svl) {
        /* the curve lies between its lowest and highest trough up to rounding;
         * a sample past them clamps to the ends (and the check catches it) */
        kbase = wm_key(s_vmin);
        const uint64_t ktop = wm_key(s_vmax);
        const int nbits = ktop > kbase ? 64 - __clzll((long long)(ktop - kbase)) : 0;
        shc = nbits > 40 ? nbits - 40 : 0;
    }
    {
        auto ckey = [&](int p) -> uint64_t {
            const uint64_t k = wm_key(dval(t0 + spos(p)));
            return shc ? (k > kbase ? k - kbase : 0ull) >> shc : k;
        };
        uint64_t kor = 0, kand = ~0ull;
        for (int p = tid; p < m; p += WM_T) {
            posA[p] = (uint16_t)p;                           /* slot order == index order */
            const uint64_t k = ckey(p);
            kh[p] = (uint32_t)k;
            kor |= k;
            kand &= k;
        }
        for (int o = 32; o > 0; o >>= 1) {
            kor |= (uint64_t)__shfl_xor((long long)kor, o);
            kand &= (uint64_t)__shfl_xor((long long)kand, o);
        }
        if (lane == 0) { s_or[wid] = kor; s_and[wid] = kand; }
        if (wbin_all)
            for (int j = tid; j < NWV * 256; j += WM_T) wbin_all[j] = 0ull;
        __syncthreads();
        uint64_t vary = 0;
        {
            uint64_t o = 0, a = ~0ull;
            for (int w = 0; w < NWV; ++w) { o |= s_or[w]; a &= s_and[w]; }
            vary = o ^ a;                                    /* key bits that differ somewhere */
        }
        STAMP(0);
        uint32_t *wc = cnt + wid * 128;
        for (int d = 0; d < 8; ++d) {
            if (d == 4 && (vary >> 32)) {                    /* high halves, indexed by index */
                for (int p = tid; p < m; p += WM_T) kh[p] = (uint32_t)(ckey(p) >> 32);
                __syncthreads();
            }
            if (((vary >> (8 * d)) & 0xFFull) == 0) continue;   /* uniform: constant digit, order unchanged */
            const int sh = 8 * (d & 3);
            for (int j = lane; j < 128; j += 64) wc[j] = 0;
            /* digits of all this lane's items first (independent LDS reads) */
            uint32_t dg8[(MAXIT + 3) / 4], rk16[(MAXIT + 1) / 2];   /* packed: digit 8 b, rank 16 b */
            /* m and IT opaque per loop: otherwise the per-item masks of the three
             * unrolled loops are hoisted out of the digit loop and live in ~100
             * SGPRs, which spill to VGPR lanes (a readlane per use) */
            int mo = mu, ITo = ITu, sb = wid * S + lane;
            asm volatile("" : "+s"(mo), "+s"(ITo), "+v"(sb));
#pragma unroll
            for (int i = 0; i < MAXIT; ++i) {
                const int slot = sb + i * 64;
                const uint32_t dg = (i < ITo && slot < mo) ? (kh[posA[slot]] >> sh) & 0xFFu : 0u;
                if ((i & 3) == 0) dg8[i >> 2] = dg; else dg8[i >> 2] |= dg << (8 * (i & 3));
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" : "+s"(mo), "+s"(ITo), "+v"(sb));
#pragma unroll
            for (int i = 0; i < MAXIT; ++i) {
                if (i < ITo) {
                    const int slot = sb + i * 64;
                    const bool valid = slot < mo;
                    const uint32_t dg = (dg8[i >> 2] >> (8 * (i & 3))) & 0xFFu;
                    uint64_t peers;
                    if (wbin_all) {                          /* uniform */
                        unsigned long long *bin = wbin_all + wid * 256 + dg;
                        if (valid) atomicOr(bin, 1ull << lane);
                        peers = __hip_atomic_load(bin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else {
                        peers = match8(dg);
                    }
                    peers &= __ballot(valid);
                    const uint64_t below = peers & lanemask_lt();
                    const int leader = valid ? __ffsll((long long)peers) - 1 : lane;
                    uint32_t base = 0;
                    if (valid && below == 0) {   /* LDS atomics of one wave land in issue (= slot) order */
                        base = atomicAdd(&wc[dg >> 1], (uint32_t)__popcll(peers) << (16 * (dg & 1)));
                        if (wbin_all) __hip_atomic_store(wbin_all + wid * 256 + dg, 0ull, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_WORKGROUP);   /* after every peer's read */
                    }
                    base = (uint32_t)__shfl((int)base, leader);
                    const uint32_t rnk = ((base >> (16 * (dg & 1))) & 0xFFFFu) + (uint32_t)__popcll(below);
                    if ((i & 1) == 0) rk16[i >> 1] = rnk; else rk16[i >> 1] |= rnk << 16;
                }
            }
            __syncthreads();
            STAMP(1);
            /* exclusive scan over (digit, wave) order, 4 consecutive entries per thread */
            {
                uint32_t v[4], sm = 0;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int e = tid * 4 + u, dg = e / NWV, w = e % NWV;
                    v[u] = (cnt[w * 128 + (dg >> 1)] >> (16 * (dg & 1))) & 0xFFFFu;
                    sm += v[u];
                }
                uint32_t x = sm;
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(x, o);
                    if (lane >= o) x += y;
                }
                if (lane == 63) s_wt[wid] = (int)x;
                __syncthreads();
                uint32_t run = x - sm;
                for (int w = 0; w < wid; ++w) run += (uint32_t)s_wt[w];
                /* the two halves of a counter word are different threads' entries:
                 * write 16-bit halves */
                uint16_t *c16 = (uint16_t *)cnt;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int e = tid * 4 + u, dg = e / NWV, w = e % NWV;
                    c16[(w * 128 + (dg >> 1)) * 2 + (dg & 1)] = (uint16_t)run;
                    run += v[u];
                }
            }
            __syncthreads();
            STAMP(2);
            const uint16_t *c16 = (const uint16_t *)cnt;
            asm volatile("" : "+s"(mo), "+s"(ITo), "+v"(sb));
#pragma unroll
            for (int i = 0; i < MAXIT; ++i) {
                const int slot = sb + i * 64;
                if (i < ITo && slot < mo) {
                    const uint32_t dg = (dg8[i >> 2] >> (8 * (i & 3))) & 0xFFu;
                    const uint32_t rnk = (rk16[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
                    posB[(int)c16[(wid * 128 + (dg >> 1)) * 2 + (dg & 1)] + (int)rnk] = posA[slot];
                }
            }
            __syncthreads();
            uint16_t *t = posA; posA = posB; posB = t;
            STAMP(3);
        }
    }
    /* posA[r] = structure index of rank r; posB becomes its inverse */
    uint16_t *posR = posA, *rkx = posB;
    for (int r = tid; r < m; r += WM_T) rkx[posR[r]] = (uint16_t)r;
    if (svl)
        for (int r = tid; r < m; r += WM_T) svl[r] = dval(t0 + spos(posR[r]));
    __syncthreads();
    if (shc) {
        bool down = false;                                   /* a compact key hid an order */
        for (int r = tid; r + 1 < m; r += WM_T) down |= svl[r] > svl[r + 1];
        if (__syncthreads_or(down)) {                        /* the full-width variant redoes it */
            if (tid == 0) { if (chunked) A.wm_fail[f] = 1; else full[f] = 1; }
            return !chunked;
        }
    }
    /* per-wave block scratch past the two index arrays: the collected ranks,
     * then the partial members; the sorted values past that when they fit
     * (else each output evaluates its two) */
#ifdef RQ_STOP_SORT
    return false;
#endif
    uint32_t *wl = (uint32_t *)(smem + Lay.area + wsc) + (size_t)wid * WM_WSCR;
    STAMP(5);

    /* ---------------- 2. outputs, a block of 64 at a time per wave ----------------
     * Lane j of a wave takes output i = i0 + j.  Its window's kept samples are
     * the structure indices [plo_j, phi_j); plo and phi do not decrease with j,
     * and within a block each moves by at most 63 (the window moves by one
     * position per output).  U = [plo_first, phi_last) over the block's valid
     * lanes.  Lane j's k-th smallest kept sample is its own t_j-th member in
     * rank order (t_j = k_j - low samples in its window).  A rank cursor rs is
     * kept as U's Tmin-th member (Tmin = min_j t_j), moved from the previous
     * block's (U shifts by at most 64 indices at each end: one ballot per end
     * corrects the count of members below rs; the cursor then walks 64 ranks
     * per step).  From rs the next `need` members of U are collected in rank
     * order.  Lane j has Tmin - (its excluded members below rs) own members
     * before rs, so its k-th and (k+1)-th smallest are its na-th and nb-th own
     * member among the collected ones; `need` bounds how far that can lie,
     * excluded members included.  A collected member at position p belongs to
     * the lanes j with s_j <= p < e_j, i.e. the lane range [p - i0 - off,
     * p - i0 - off + W) (the window bounds' clamps never bind at a kept
     * position); the few members that miss some valid lane ("partial": within
     * 63 positions of U's ends) are listed, and each lane skips the ones it
     * misses while counting to na and nb.  Every step is a wave-wide operation;
     * no workgroup barrier. */
    auto target = [&](int nb, double &idxf, bool &interp) -> int {
        idxf = 0;
        int k = 0;
        if (nb > 1) {
            idxf = q * (double)(nb - 1);
            k = (int)idxf;
        }
        interp = !(nb == 1 || (double)k == idxf);
        return k;
    };
    const uint64_t ltm = lanemask_lt();
    const int off = (int)((W - 1) / 2), Wi = (int)W, ni = (int)n, t0i = (int)t0;
#ifdef RQ_DIAG_Q
    unsigned long long dq[8] = {0};   /* tools/rqbench -DRQ_DIAG_Q, wave 0: blocks, need, partial members, collect trips, cursor trips, collected */
#endif
    int vfirst = INT_MAX, vlast = -1;
#ifdef RQ_DIAG_W
    const unsigned long long tw0 = __builtin_amdgcn_s_memtime();   /* tools/rqbench -DRQ_DIAG_W: per-wave output phase */
#endif
    {
        const int NBLK = (int)((o1 - o0 + 63) >> 6);
        const int NBW = (NBLK + NWV - 1) / NWV;
        const int b0 = wid * NBW, b1 = min(NBLK, b0 + NBW);
        int rs = 0, cU = 0, pPlo = -1, pPhi = -1;            /* wave-uniform cursor */
        for (int bk = b0; bk < b1; ++bk) {
            const int i0 = (int)o0 + (bk << 6), i = i0 + lane;
            bool valid = false;
            int plo = 0, phi = 0, t = 0, nobs = 0, kq = 0;
            double idxq = 0.0;                               /* pandas' quantile index and its interpolation */
            bool intq = false;
            if (i < (int)o1) {
                const int ee = i + 1 + off, ss = ee - Wi;
                const int e = ee < ni ? ee : ni, sc = ss > 0 ? ss : 0;
                const int lo = sc > t0i ? sc : t0i;
                nobs = e > lo ? e - lo : 0;
                if (nobs >= minp && nobs > 0) {
                    valid = true;
                    plo = kidx(lo - t0i);
                    phi = kidx(e - t0i);
                    const int lw = PRUNE ? lidx(e - t0i) - lidx(lo - t0i) : 0;
                    kq = target(nobs, idxq, intq);
                    t = kq - lw;
                }
            }
            const uint64_t vm0 = __ballot(valid);
            if (vm0 == 0) {                                  /* NaN block: the cursor restarts after it */
                if (i < (int)o1) out[i] = __builtin_nan("");
                rs = cU = 0;
                pPlo = -1;
                continue;
            }
            /* a block whose members to collect exceed the scratch runs as four
             * passes of 16 lanes (need <= 15 + 2 * 30 + 2 there; 64 lanes need
             * about 30 on the bench's curves, at most 63 + 2 * 126 + 2) */
            int ja = __ffsll((long long)vm0) - 1, jb = 63 - __clzll((long long)vm0);
            int Plo = __builtin_amdgcn_readlane(plo, ja), PloMax = __builtin_amdgcn_readlane(plo, jb);
            int PhiMin = __builtin_amdgcn_readlane(phi, ja), Phi = __builtin_amdgcn_readlane(phi, jb);
            int Tmin = -wave_max_dpp(valid ? -t : INT_MIN + 1);
            int need = wave_max_dpp(valid ? t - Tmin + (plo - Plo) + (Phi - phi) : 0) + 2;
            const int npass = need > WM_DCAP ? 4 : 1;
#ifdef RQ_DIAG_Q
            dq[0] += 1; dq[1] += (unsigned long long)need;
#endif
#ifdef BPMX_STAMPS
            if (threadIdx.x == 0) _st_acc[12] += 1000000ull * (npass > 1) + (unsigned long long)need;   /* diagnostics: 4-pass blocks, need */
#endif
            const bool valid0 = valid;
            double res = __builtin_nan("");
            for (int pass = 0; pass < npass; ++pass) {
                if (npass > 1) {
                    valid = valid0 && (lane >> 4) == pass;
                    const uint64_t vm = __ballot(valid);
                    if (vm == 0) continue;
                    ja = __ffsll((long long)vm) - 1;
                    jb = 63 - __clzll((long long)vm);
                    Plo = __builtin_amdgcn_readlane(plo, ja); PloMax = __builtin_amdgcn_readlane(plo, jb);
                    PhiMin = __builtin_amdgcn_readlane(phi, ja); Phi = __builtin_amdgcn_readlane(phi, jb);
                    Tmin = -wave_max_dpp(valid ? -t : INT_MIN + 1);
                    need = min(WM_DCAP, wave_max_dpp(valid ? t - Tmin + (plo - Plo) + (Phi - phi) : 0) + 2);
                }
                STAMP(4);
                /* the cursor's count for this U: members dropped on the left, added on the right */
                if (pPlo >= 0) {
                    const int xl = pPlo + lane, xe = pPhi + lane;
                    const bool bl = xl < Plo && (int)rkx[xl] < rs;
                    const bool be = xe < Phi && (int)rkx[xe] < rs;
                    cU += __popcll(__ballot(be)) - __popcll(__ballot(bl));
                } else {
                    rs = cU = 0;
                }
                /* move rs to U's Tmin-th member */
                for (int guard = 0; guard <= m / 64 + 2; ++guard) {
#ifdef RQ_DIAG_Q
                    dq[4] += 1;
#endif
                    if (cU <= Tmin) {                        /* forward, two chunks of ranks per round trip */
                        const int rr = rs + lane;
                        const int x0 = rr < m ? (int)posR[rr] : -1;
                        const int x1 = rr + 64 < m ? (int)posR[rr + 64] : -1;
                        const uint64_t bm0 = __ballot(x0 >= Plo && x0 < Phi);
                        const uint64_t bm1 = __ballot(x1 >= Plo && x1 < Phi);
                        const int c0 = __popcll(bm0), c1 = __popcll(bm1);
                        if (cU + c0 > Tmin) {
                            rs += select64(bm0, Tmin - cU);
                        } else if (cU + c0 + c1 > Tmin) {
                            rs += 64 + select64(bm1, Tmin - cU - c0);
                        } else {
                            rs += 128;
                            cU += c0 + c1;
                            continue;
                        }
                    } else {
                        const int st = rs > 64 ? rs - 64 : 0, rr = st + lane;
                        const int x = rr < rs ? (int)posR[rr] : -1;
                        const uint64_t bm = __ballot(x >= Plo && x < Phi);
                        const int c = __popcll(bm);
                        if (cU - c > Tmin) {
                            rs = st;
                            cU -= c;
                            continue;
                        }
                        rs = st + select64(bm, Tmin - (cU - c));
                    }
                    cU = Tmin;
                    break;
                }
                /* own members below rs: Tmin minus this lane's excluded ones there */
                int na;
                {
                    const int xL = Plo + lane, xR = PhiMin + lane;
                    const uint64_t mL = __ballot(xL < PloMax && (int)rkx[xL] < rs);
                    const uint64_t mR = __ballot(xR < Phi && (int)rkx[xR] < rs);
                    const int dl = valid ? plo - Plo : 0, dr = valid ? phi - PhiMin : 0;   /* both <= 63 */
                    na = t - Tmin + __popcll(mL & ((1ull << dl) - 1ull)) + __popcll(mR >> dr);
                }
                STAMP(14);
                /* the next members of U from rs, in rank order (at most `need`).
                 * The partial ones (they miss some valid lane) are taken in slot
                 * order as they come, each lane skipping those it misses while
                 * locating its na-th own member (ia) and the next (ib); once every
                 * valid lane's ib lies below the count collected, later members
                 * cannot move either, so the walk stops there (usually within the
                 * first 64 ranks; `need` bounds it in any case). */
                int cnt = 0, ia = na, ib = -1;
                const int lbase = i0 + off;                      /* member at position p: lanes [p - lbase, p - lbase + W) */
                bool more = true;
                for (int r = rs; more && cnt < need && r < m; r += 128) {   /* two chunks of ranks per round trip */
#ifdef RQ_DIAG_Q
                    dq[3] += 1;
#endif
                    const int rr = r + lane;
                    const int xs[2] = {rr < m ? (int)posR[rr] : -1, rr + 64 < m ? (int)posR[rr + 64] : -1};
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        if (!more || cnt >= need) break;         /* uniform */
                        const int x = xs[h];
                        const bool mb = x >= Plo && x < Phi;
                        const uint64_t bm = __ballot(mb);
                        const int slot = cnt + __popcll(bm & ltm);
                        /* only members within 63 indices of U's ends miss a valid lane */
                        const bool edge = mb && slot < need && (x < PloMax || x >= PhiMin);
                        bool part = false;
                        uint32_t lr = 0;
                        if (mb && slot < need) wl[slot] = (uint32_t)(rr + 64 * h);
                        if (edge) {
                            const int pos = t0i + spos(x);
                            const int l0 = pos - lbase, l1 = l0 + Wi - 1;
                            const int ca = l0 > ja ? l0 : ja, cb = l1 < jb ? l1 : jb;
                            part = ca > ja || cb < jb;
                            /* an empty range (cb < ca) misses every lane */
                            lr = (uint32_t)slot | ((uint32_t)(ca & 127) << 16) | ((uint32_t)((cb + 1) & 127) << 24);
                        }
                        cnt += __popcll(bm);
                        for (uint64_t pm = __ballot(part); pm; pm &= pm - 1) {   /* slot order = lane order */
                            const uint32_t pr = (uint32_t)__builtin_amdgcn_readlane((int)lr, __ffsll((long long)pm) - 1);
                            const int li = (int)(pr & 0xFFFFu), ca = (int)((pr >> 16) & 127u), cb1 = (int)(pr >> 24);
                            const bool miss = lane < ca || lane >= cb1;
#ifdef RQ_DIAG_Q
                            dq[2] += 1;
#endif
                            if (ib < 0) {
                                if (li <= ia) {
                                    if (miss) ++ia;
                                    continue;
                                }
                                ib = ia + 1;
                            }
                            if (li == ib && miss) ++ib;
                        }
                        more = __ballot(valid && (ib >= 0 ? ib : ia + 1) >= cnt) != 0;
                    }
                }
#ifdef RQ_DIAG_Q
                dq[5] += (unsigned long long)cnt;
#endif
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                STAMP(15);
                if (ib < 0) ib = ia + 1;
                ia = ia < need ? ia : need - 1;                  /* (never binds; keeps a corrupted walk in bounds) */
                ib = ib < need ? ib : need - 1;
                if (valid) {
                    const int k = kq;
                    const double idxf = idxq;
                    const bool interp = intq;
                    const double va = svl ? svl[wl[ia]] : dval(t0 + spos(posR[wl[ia]]));
                    if (!interp) {
                        res = va;
                    } else {
                        const double vb = svl ? svl[wl[ib]] : dval(t0 + spos(posR[wl[ib]]));
                        res = va + (vb - va) * (idxf - (double)k);
                    }
                    vfirst = vfirst < i ? vfirst : i;
                    vlast = vlast > i ? vlast : i;
                }
                __builtin_amdgcn_wave_barrier();                 /* the scratch is rewritten by the next pass */
                pPlo = Plo;
                pPhi = Phi;
            }
            if (i < (int)o1) out[i] = res;
            STAMP(6);
        }
    }
#ifdef RQ_DIAG_W
    if (lane == 0 && A.stamps) A.stamps[blockIdx.x * 16 + wid] = __builtin_amdgcn_s_memtime() - tw0;
#endif
    for (int o = 32; o > 0; o >>= 1) {
        vfirst = min(vfirst, __shfl_xor(vfirst, o));
        vlast = max(vlast, __shfl_xor(vlast, o));
    }
    if (lane == 0) {
        atomicMin(&s_first, vfirst);
        atomicMax(&s_last, vlast);
    }
    __threadfence_block();
    __syncthreads();
    STAMP(7);                                                /* (the other waves' query tail) */
#ifndef RQ_DIAG_W
    STAMP_FLUSH(A.stamps);
#endif
#ifdef RQ_DIAG_Q
    if (threadIdx.x == 0 && A.stamps)
        for (int k = 0; k < 8; ++k) A.stamps[blockIdx.x * 16 + 8 + k] = dq[k];
#endif
    if (chunked) {                                           /* bfill / ffill over all chunks: k_rollq_fill */
        if (tid == 0 && s_last >= 0) {
            atomicMin(&A.vfirst[f], s_first);
            atomicMax(&A.vlast[f], s_last);
        }
        return false;
    }
    /* ---- .bfill().ffill() ---- */
    const int first = s_first, last = s_last;
    if (last < 0) {
        if (tid == 0) A.allnan[f] = 1;
        return false;
    }
    if (tid == 0) A.allnan[f] = 0;
    const double vf = out[first], vl = out[last];
    for (int64_t i = tid; i < first; i += WM_T) out[i] = vf;
    for (int64_t i = last + 1 + tid; i < n; i += WM_T) out[i] = vl;
    return false;
}

/* The pruned variant runs a recording it cannot take (too many kept samples,
 * a non-finite curve, a compact-key collision) through the unpruned body in
 * the same workgroup, so no second launch is needed for it; its dynamic LDS
 * is the larger of the two layouts. */
template <bool PRUNE>
__global__ __launch_bounds__(WM_T) void k_rollq_wm_t(RollqArgs A, uint16_t *pos_scratch, int32_t *full) {
    __shared__ RqShared sh;
    if (rollq_wm_body<PRUNE>(A, pos_scratch, full, sh) && PRUNE) {
        __syncthreads();
        (void)rollq_wm_body<false>(A, pos_scratch, full, sh);
    }
}

template __global__ void k_rollq_wm_t<true>(RollqArgs, uint16_t *, int32_t *);
template __global__ void k_rollq_wm_t<false>(RollqArgs, uint16_t *, int32_t *);

/* one rolling quantile of recording blockIdx.x: pruned, or unpruned in the
 * same workgroup when the pruned structure cannot take it */
__device__ __forceinline__ void rollq_wm_run(const RollqArgs &a, int32_t *full, RqShared &sh) {
    if (rollq_wm_body<true>(a, nullptr, full, sh)) {
        __syncthreads();
        (void)rollq_wm_body<false>(a, nullptr, full, sh);
    }
}

/* ---------------------------------------------------------------------------
 * k_floor_wm: the noise floor after the draft, one workgroup per recording
 * (bpm_analysis.py:1088-1117, recordings of at most WM_MMAX decimated
 * samples): sanitize (sanitize_wg) from k_draft_bounds' / k_draft_points'
 * decisions or the full draft; then < 5 raw troughs: the static floor,
 * quantile(env, noise_floor_q), selected here when no earlier stage selected
 * it (qn, the lazy level); > 2 kept troughs: the final rolling quantile; else
 * the draft floor (the full draft when it was computed, else its rolling
 * quantile here); an all-NaN floor: quantile(env, 0.1).  One launch for what
 * took k_sanitize, k_rollq_wm_t (draft fallback), k_rollq_wm_t (final),
 * k_floor_final and the lazy k_quantile_reg, with no device round trip of the
 * per-recording decisions.  (The full draft before sanitize stays a launch of
 * its own: a second rolling-quantile call site in this kernel spills.)
 * ------------------------------------------------------------------------- */
static_assert(WM_T == QR_T && WM_MMAX <= QR_MAX,
              "k_floor_wm runs qr_select with its own threads over up to WM_MMAX samples");
__global__ __launch_bounds__(WM_T) void k_floor_wm(FloorWmArgs A) {
    __shared__ RqShared sh;
    __shared__ int s_sc[WM_T / 64 + 1];
    extern __shared__ __align__(16) unsigned char smem[];
    const RollqArgs &R = A.rq;
    const int f = blockIdx.x;
    if (f >= R.n_files || !A.sa.active[f]) return;
    const int64_t d0 = R.doff[f], n = R.doff[f + 1] - d0;
    const int m = A.sa.nraw[f], tid = threadIdx.x;
    const bool have_draft = m >= 5 && A.exact[f];            /* the full draft, computed before */
    const int w = __builtin_amdgcn_readfirstlane(sanitize_wg<WM_T>(A.sa, f, s_sc));   /* uniform */
    __syncthreads();
    const bool final = m >= 5 && w > 2;
    if (m >= 5 && (final || !have_draft)) {                 /* the final floor, or the draft floor here */
        RollqArgs a = R;
        a.troughs = final ? A.sa.out : A.sa.raw;
        a.tv = final ? A.sa.outv : A.sa.rawv;
        a.ntr = final ? A.sa.nout : A.sa.nraw;
        a.allnan = final ? A.an_final : A.an_draft;
        a.out = A.floor;
        a.run = A.sa.active;                                 /* (1 here) */
        rollq_wm_run(a, A.full, sh);
        __syncthreads();
    }
    bool fill = false, from_draft = false, nanfb = false;
    double v = 0.0;
    const double *qv = A.qv + (int64_t)f * Q_SLOTS;
    if (m < 5) {                                             /* static floor */
        if (A.qn.n_levels > 0) {
            const double *x = R.env + d0;
            uint64_t key[QR_IT];
#pragma unroll
            for (int it = 0; it < QR_IT; ++it) {
                const int64_t i = (int64_t)it * QR_T + tid;
                key[it] = i < n ? f64_key(x[i]) : 0ull;
            }
            qr_select(key, n, A.qn, f, *reinterpret_cast<QrShared *>(smem));
            __syncthreads();
        }
        v = qv[Q_NOISE];
        fill = true;
    } else if (final) {
        nanfb = A.an_final[f] != 0;
    } else {
        from_draft = have_draft;
        nanfb = A.an_draft[f] != 0;
    }
    if (nanfb) {
        fill = true;
        from_draft = false;
        v = qv[Q_FALLBACK];
    }
    double *floor = A.floor + d0;
    const double *draft = A.draft + d0;
    if (fill || from_draft)
        for (int64_t i = tid; i < n; i += WM_T) floor[i] = from_draft ? draft[i] : v;
    if (tid == 0 && nanfb) A.sa.flags[f] |= BPMX_F_NAN_FLOOR;
}

}  // namespace bpmx
