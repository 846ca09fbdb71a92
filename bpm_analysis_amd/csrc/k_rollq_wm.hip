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
 *   2. wavelet matrix over the rank sequence (ceil(log2 m) levels): per level
 *      a bit vector with a rank directory, {word, ones-before} per 32 samples.
 *   3. every output independently: its window's k-th smallest by one top-down
 *      descent, the (k+1)-th by walking up the rank order to the next rank
 *      inside the window; pandas' linear interpolation, nobs / min_periods
 *      from the window bounds.  NaN outputs are a prefix and a suffix (nobs is
 *      unimodal), filled from the first and last valid output.
 * Recordings longer than WM_MMAX decimated samples take k_rolling_quantile.
 */
#include "bpmx_common.h"
#include "bpmx_kernels.h"
#include "bpmx_stamps.h"

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

/* rank directory entry: 32 positions' bits and the ones before them */
struct WmRec {
    uint32_t word;
    uint32_t ones;
};

template <bool PRUNE>
__global__ __launch_bounds__(WM_T) void k_rollq_wm_t(RollqArgs A, uint16_t *pos_scratch, int32_t *full) {
    constexpr int NWV = WM_T / 64;
    constexpr int MMAX = PRUNE ? WM_PMAX : WM_MMAX;          /* samples in the structure */
    constexpr int MAXIT = MMAX / WM_T;
    const int f = blockIdx.x;
    if (f >= A.n_files) return;
    const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
    if (!A.run[f]) {
        if (PRUNE && tid == 0) full[f] = 0;
        return;
    }
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    const int ntr_all = A.env ? A.ntr[f] : 0;
    /* chunk mode: a long recording's outputs [o0, o1) in workgroup (f, chunk),
     * over the samples [t0, top) their windows reach */
    const bool chunked = PRUNE && A.wm_chunk > 0 && n > WM_MMAX && A.env;
    if (!chunked && blockIdx.y > 0) return;
    const int64_t W = A.window, minp = A.min_periods;
    int64_t o0 = 0, o1 = n, t0 = 0, top = n;
    int jlo = 0, ntr = ntr_all;                              /* troughs staged: [jlo, jlo + ntr) */
    __shared__ int s_jlo, s_jhi;
    if (chunked) {
        if (tid == 0 && blockIdx.y == 0) full[f] = 0;        /* long: never the unpruned variant */
        o0 = (int64_t)blockIdx.y * A.wm_chunk;
        if (o0 >= n) return;
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
            return;
        }
        if (top - t0 > WM_MMAX || ntr > WM_TRMAX) {
            if (tid == 0) A.wm_fail[f] = 1;
            return;
        }
    }
    const bool fused = A.env && ntr <= WM_TRMAX;
    if (!chunked && (n > WM_MMAX || n <= 0 || (PRUNE && !fused))) {   /* k_rolling_quantile / the unpruned variant */
        if (PRUNE && tid == 0) full[f] = (n <= WM_MMAX && n > 0) ? 1 : 0;
        return;
    }
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int s_first, s_last, s_Z[16], s_wt[NWV], s_mk;
    __shared__ unsigned long long s_or[NWV], s_and[NWV];
    __shared__ double s_vmin, s_vmax;

    const double *dense = A.dense + d0;
    double *out = A.out + d0;
    /* kept index of each rank */
    uint16_t *ps = chunked ? A.wm_pos_ch + ((int64_t)f * gridDim.y + blockIdx.y) * WM_PMAX : pos_scratch + d0;
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
        for (int j = tid; j < ntr; j += WM_T) {
            s_tp[j] = (int32_t)tr[j];
            s_tv[j] = A.env[d0 + tr[j]];
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
            return interp_at(x, trg, [&](int j) { return A.env[d0 + trg[j]]; }, ntr_all);
        }
        if (ntr == 0 || x < s_tp[0]) return __builtin_nan("");
        int j = s_bj[(x - xb) >> 6];
        if (j < 0) j = 0;
        while (j + 1 < ntr && s_tp[j + 1] <= x) ++j;
        if (j == ntr - 1 || s_tp[j] == x) return s_tv[j];
        const double y0 = s_tv[j], y1 = s_tv[j + 1];
        const double slope = PRUNE ? s_sl[j] : (y1 - y0) / ((double)s_tp[j + 1] - (double)s_tp[j]);
        double r = slope * ((double)x - (double)s_tp[j]) + y0;
        if (r != r) {
            r = slope * ((double)x - (double)s_tp[j + 1]) + y1;
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
            return;
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
            return;
        }
        if (tid == 0 && !chunked) full[f] = 0;
        for (int pb = wid; pb < NPB; pb += NWV) {
            const uint64_t mk = kmask[pb];
            if ((mk >> lane) & 1) kpos[kpre[pb] + __popcll(mk & lanemask_lt())] = (uint16_t)((pb << 6) + lane);
        }
        m = kc;
        __syncthreads();
    }
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

    /* LDS, sort phase: posA[m8] | posB[m8] | kh[m8] | cnt[NWV][128] (two 16-bit counters per word).
     * Slots >= m are padding: they sort last, so they are neither stored nor counted. */
    const int IT = (m + WM_T - 1) / WM_T;                    /* rounds per wave */
    const int S = 64 * IT;                                   /* slots per wave */
    const int m8 = (m + 7) & ~7;
    uint16_t *posA = (uint16_t *)(smem + Lay.area);
    uint16_t *posB = posA + m8;
    uint32_t *kh = (uint32_t *)(posB + m8);
    uint32_t *cnt = kh + m8;

    /* ---------------- 1. ranks by LSD radix sort ---------------- */
    uint64_t kor = 0, kand = ~0ull;
    for (int p = tid; p < m; p += WM_T) {
        posA[p] = (uint16_t)p;                               /* slot order == index order */
        const uint64_t k = wm_key(dval(t0 + spos(p)));
        kh[p] = (uint32_t)k;
        kor |= k;
        kand &= k;
    }
    for (int o = 32; o > 0; o >>= 1) {
        kor |= (uint64_t)__shfl_xor((long long)kor, o);
        kand &= (uint64_t)__shfl_xor((long long)kand, o);
    }
    if (lane == 0) { s_or[wid] = kor; s_and[wid] = kand; }
    __syncthreads();
    uint64_t vary = 0;
    {
        uint64_t o = 0, a = ~0ull;
        for (int w = 0; w < NWV; ++w) { o |= s_or[w]; a &= s_and[w]; }
        vary = o ^ a;                                        /* key bits that differ somewhere */
    }
    STAMP(0);
    uint32_t *wc = cnt + wid * 128;
    for (int d = 0; d < 8; ++d) {
        if (d == 4 && (vary >> 32)) {                        /* high halves, indexed by index */
            for (int p = tid; p < m; p += WM_T) kh[p] = (uint32_t)(wm_key(dval(t0 + spos(p))) >> 32);
            __syncthreads();
        }
        if (((vary >> (8 * d)) & 0xFFull) == 0) continue;    /* uniform: constant digit, order unchanged */
        const int sh = 8 * (d & 3);
        for (int j = lane; j < 128; j += 64) wc[j] = 0;
        /* digits of all this lane's items first (independent LDS reads) */
        uint32_t dg8[(MAXIT + 3) / 4], rk16[(MAXIT + 1) / 2];   /* packed: digit 8 b, rank 16 b */
#pragma unroll
        for (int i = 0; i < MAXIT; ++i) {
            const int slot = wid * S + i * 64 + lane;
            const uint32_t dg = (i < IT && slot < m) ? (kh[posA[slot]] >> sh) & 0xFFu : 0u;
            if ((i & 3) == 0) dg8[i >> 2] = dg; else dg8[i >> 2] |= dg << (8 * (i & 3));
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < MAXIT; ++i) {
            if (i < IT) {
                const int slot = wid * S + i * 64 + lane;
                const bool valid = slot < m;
                const uint32_t dg = (dg8[i >> 2] >> (8 * (i & 3))) & 0xFFu;
                const uint64_t peers = match8(dg) & __ballot(valid);
                const uint64_t below = peers & lanemask_lt();
                const int leader = valid ? __ffsll((long long)peers) - 1 : lane;
                uint32_t base = 0;
                if (valid && below == 0)   /* LDS atomics of one wave land in issue (= slot) order */
                    base = atomicAdd(&wc[dg >> 1], (uint32_t)__popcll(peers) << (16 * (dg & 1)));
                base = (uint32_t)__shfl((int)base, leader);
                const uint32_t rnk = ((base >> (16 * (dg & 1))) & 0xFFFFu) + (uint32_t)__popcll(below);
                if ((i & 1) == 0) rk16[i >> 1] = rnk; else rk16[i >> 1] |= rnk << 16;
            }
        }
        __syncthreads();
        STAMP(1);
        /* exclusive scan over (digit, wave) order, 4 consecutive entries per thread */
        {
            uint32_t v[4], s = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = tid * 4 + u, dg = e / NWV, w = e % NWV;
                v[u] = (cnt[w * 128 + (dg >> 1)] >> (16 * (dg & 1))) & 0xFFFFu;
                s += v[u];
            }
            uint32_t x = s;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o);
                if (lane >= o) x += y;
            }
            if (lane == 63) s_wt[wid] = (int)x;
            __syncthreads();
            uint32_t run = x - s;
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
#pragma unroll
        for (int i = 0; i < MAXIT; ++i) {
            const int slot = wid * S + i * 64 + lane;
            if (i < IT && slot < m) {
                const uint32_t dg = (dg8[i >> 2] >> (8 * (i & 3))) & 0xFFu;
                const uint32_t rnk = (rk16[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
                posB[(int)c16[(wid * 128 + (dg >> 1)) * 2 + (dg & 1)] + (int)rnk] = posA[slot];
            }
        }
        __syncthreads();
        uint16_t *t = posA; posA = posB; posB = t;
        STAMP(3);
    }
    /* posA[r] = index of rank r.  Build: seqA = the free pos buffer,
     * seqB = posA once consumed; levels over the dead kh / cnt. */
    const int L = m > 1 ? 32 - __clz(m - 1) : 1;              /* levels: ranks < 2^L */
    const int NW = (m + 63) >> 6;                             /* 64-bit words per level */
    const int NR = 2 * NW + 1;                                /* 32-bit records per level (+ sentinel) */
    uint16_t *seqA = posB, *seqB = posA;
    WmRec *lv = (WmRec *)kh;                                  /* [L][NR] */
    for (int r = tid; r < m; r += WM_T) {
        const int p = posA[r];
        ps[r] = (uint16_t)p;
        seqA[p] = (uint16_t)r;
    }
    __syncthreads();
    STAMP(4);

    /* ---------------- 2. wavelet matrix ---------------- */
    constexpr int CWMAX = (MMAX / 64 + NWV - 1) / NWV;       /* words per wave at the maximum */
    const int cw = (NW + NWV - 1) / NWV;                     /* words per wave (<= CWMAX) */
    const int wb = wid * cw, nwv = max(0, min(NW, wb + cw) - wb);
    for (int l = L - 1; l >= 0; --l) {
        WmRec *row = lv + l * NR;
        /* this wave's words into registers first (independent LDS reads), then
         * ones among them (ballots are wave-uniform: scalar sums) */
        uint32_t sq[CWMAX];
        uint32_t wones = 0;
#pragma unroll
        for (int w = 0; w < CWMAX; ++w) {
            const int p = (wb + w) * 64 + lane;
            sq[w] = (w < nwv && p < m) ? (uint32_t)seqA[p] : 0xFFFFFFFFu;   /* all-ones: invalid */
        }
#pragma unroll
        for (int w = 0; w < CWMAX; ++w)
            wones += (uint32_t)__popcll(__ballot(sq[w] != 0xFFFFFFFFu && ((sq[w] >> l) & 1)));
        if (lane == 0) s_wt[wid] = (int)wones;
        __syncthreads();
        uint32_t run = 0, tot = 0;
        for (int w = 0; w < NWV; ++w) {
            const uint32_t t = (uint32_t)s_wt[w];
            run += w < wid ? t : 0u;
            tot += t;
        }
        const int Z = m - (int)tot;                          /* zeros of this level */
        if (tid == 0) {
            row[2 * NW] = WmRec{0u, tot};
            s_Z[l] = Z;
        }
        /* stable partition (zeros, then ones) and the rank directory */
#pragma unroll
        for (int w = 0; w < CWMAX; ++w) {
            if (w < nwv) {
                const int p = (wb + w) * 64 + lane;
                const bool bit = sq[w] != 0xFFFFFFFFu && ((sq[w] >> l) & 1);
                const uint64_t word = __ballot(bit);
                if (lane == 0) {
                    row[2 * (wb + w)] = WmRec{(uint32_t)word, run};
                    row[2 * (wb + w) + 1] = WmRec{(uint32_t)(word >> 32), run + (uint32_t)__popc((uint32_t)word)};
                }
                const int o1 = (int)run + __popcll(word & lanemask_lt());
                if (sq[w] != 0xFFFFFFFFu) seqB[bit ? Z + o1 : p - o1] = (uint16_t)sq[w];
                run += (uint32_t)__popcll(word);
            }
        }
        __syncthreads();
        uint16_t *t = seqA; seqA = seqB; seqB = t;
    }
    /* rank -> index back into LDS over the dead sequence buffer */
    __threadfence_block();
    uint16_t *posR = seqA;
    for (int r = tid; r < m; r += WM_T) posR[r] = ps[r];
    /* sorted values in LDS past the levels when they fit (pruned variant);
     * otherwise each output evaluates its two values from the troughs */
    double *svl = nullptr;
    if (PRUNE) {
        const size_t off = ((size_t)4 * m8 + (size_t)L * NR * 8 + 15) & ~(size_t)15;
        if (off + (size_t)8 * m <= Lay.total - Lay.area) svl = (double *)(smem + Lay.area + off);
    }
    __syncthreads();
    if (svl) {
        for (int r = tid; r < m; r += WM_T) svl[r] = dval(t0 + spos(posR[r]));
        __syncthreads();
    }
    STAMP(5);

    /* ---------------- 3. outputs ---------------- */
    auto rk = [&](const WmRec *row, int i) {
        const WmRec r = row[i >> 5];
        return (int)r.ones + __popc(r.word & ((1u << (i & 31)) - 1u));
    };
    /* the k-th smallest of structure indices [lo, hi): one top-down descent */
    auto kth = [&](int lo, int hi, int k) {
        int r = 0;
        for (int l = L - 1; l >= 0; --l) {
            const WmRec *row = lv + l * NR;
            const int o0 = rk(row, lo), o1 = rk(row, hi);
            const int z = (hi - o1) - (lo - o0);
            if (k < z) { lo -= o0; hi -= o1; }
            else { k -= z; const int Z = s_Z[l]; lo = Z + o0; hi = Z + o1; r |= 1 << l; }
        }
        return r;
    };
    int vfirst = INT_MAX, vlast = -1;
    for (int64_t i = o0 + tid; i < o1; i += WM_T) {
        int64_t s, e;
        win_bounds(i, n, W, s, e);
        const int64_t lo = s > t0 ? s : t0;
        const int64_t nobs = e > lo ? e - lo : 0;
        double res = __builtin_nan("");
        if (nobs >= minp && nobs > 0) {
            const int plo = kidx((int)(lo - t0)), phi = kidx((int)(e - t0));
            double idxf = 0;
            int64_t k = 0;
            if (nobs > 1) {
                idxf = q * (double)(nobs - 1);
                k = (int64_t)idxf;
            }
            const bool interp = !(nobs == 1 || (double)k == idxf);
            /* the window's samples below the structure rank before every kept one */
            const int ra = kth(plo, phi, (int)k - (PRUNE ? lidx((int)(e - t0)) - lidx((int)(lo - t0)) : 0));
            const double va = svl ? svl[ra] : dval(t0 + spos(posR[ra]));
            if (!interp) {
                res = va;
            } else {
                /* k + 1 < (kept samples in the window) here, so an in-window
                 * rank above ra exists: the successor in the window */
                int rb = ra + 1, pb;
                for (;;) {
                    pb = posR[rb];
                    if (pb >= plo && pb < phi) break;
                    ++rb;
                }
                const double vb = svl ? svl[rb] : dval(t0 + spos(pb));
                res = va + (vb - va) * (idxf - (double)k);
            }
            vfirst = vfirst < (int)i ? vfirst : (int)i;
            vlast = vlast > (int)i ? vlast : (int)i;
        }
        out[i] = res;
    }
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
    STAMP(6);
    STAMP_FLUSH(A.stamps);
    if (chunked) {                                           /* bfill / ffill over all chunks: k_rollq_fill */
        if (tid == 0 && s_last >= 0) {
            atomicMin(&A.vfirst[f], s_first);
            atomicMax(&A.vlast[f], s_last);
        }
        return;
    }
    /* ---- .bfill().ffill() ---- */
    const int first = s_first, last = s_last;
    if (last < 0) {
        if (tid == 0) A.allnan[f] = 1;
        return;
    }
    if (tid == 0) A.allnan[f] = 0;
    const double vf = out[first], vl = out[last];
    for (int64_t i = tid; i < first; i += WM_T) out[i] = vf;
    for (int64_t i = last + 1 + tid; i < n; i += WM_T) out[i] = vl;
}

template __global__ void k_rollq_wm_t<true>(RollqArgs, uint16_t *, int32_t *);
template __global__ void k_rollq_wm_t<false>(RollqArgs, uint16_t *, int32_t *);

}  // namespace bpmx
