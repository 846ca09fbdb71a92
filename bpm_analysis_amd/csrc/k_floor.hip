/*
 * k_floor.hip — the dynamic noise floor (bpm_analysis.py:1079-1115).
 *
 *   k_interp            reindex(arange(Nd)).interpolate() of the trough
 *                       samples == numpy arr_interp (slope*(x-x0)+y0), NaN
 *                       before the first trough (interp_at); only for the
 *                       recordings k_rollq_wm does not interpolate itself.
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

#include "bpmx_stamps.h"

namespace bpmx {

__global__ __launch_bounds__(256) void k_interp(InterpArgs A) {
    const int f = blockIdx.y;
    if (f >= A.n_files || !A.run[f]) return;
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    if (n <= A.skip_n && A.ntr[f] <= WM_TRMAX) return;      /* k_rollq_wm interpolates these itself */
    if (n > A.skip_gt) return;
    const int64_t *t = A.troughs + d0;
    const double *e = A.env + d0;
    /* a few workgroups per recording striding over it: a recording the
     * rolling-quantile kernel interpolates itself costs one early exit */
    for (int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x; x < n; x += (int64_t)gridDim.x * 256)
        A.dense[d0 + x] = interp_at(x, t, [&](int j) { return e[t[j]]; }, A.ntr[f]);
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

template <int T, int RQ_MAXCH>
__global__ __launch_bounds__(T) void k_rolling_quantile(RollqArgs A) {
    const int f = blockIdx.x;
    if (f >= A.n_files || !A.run[f]) return;
    if (A.doff[f + 1] - A.doff[f] <= A.wm_max) return;       /* done by k_rollq_wm */
    /* chunk blockIdx.y of the outputs: the window is local, so a chunk starts
     * from an empty union and fills it from its own first window */
    const int64_t c0 = (int64_t)blockIdx.y * A.chunk;
    if (c0 >= A.doff[f + 1] - A.doff[f]) return;
    extern __shared__ __align__(16) unsigned char smem[];
    const int cap = A.cap;
    /* LDS carve-up (rollq_lds_bytes); single sorted buffer A: a merge reads the
     * thread's slice of A into registers, barriers, then writes the merged order. */
    double *Av = (double *)smem;                     /* [cap] sorted union values */
    double *nsv = Av + cap;                          /* [T] new values, sorted */
    double *runv = nsv + T;                          /* [T] per-wave sorted runs | edge list */
    uint32_t *E = (uint32_t *)runv;                  /*     (aliases runv after the merge) */
    uint16_t *Ap = (uint16_t *)(runv + T);           /* [cap] positions mod 2^16 */
    uint16_t *nsp = Ap + cap;                        /* [T] */
    uint16_t *ubv = nsp + T;                         /* [T] */
    int *rpref = (int *)(ubv + T);                   /* [T+1] removed prefix | edge-word prefix */
    int *wpre = rpref;                               /*     (cap/64+2 <= T+1 entries, edge phase) */
    int *sh = rpref + T + 1;                         /* [T/64+2] */
    __shared__ int s_first, s_last, s_nE;

    const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    const double *dense = A.dense + d0;
    double *out = A.out + d0;
    const int64_t W = A.window, minp = A.min_periods;
    const int64_t t0 = A.troughs[d0];
    const int64_t cend = c0 + A.chunk < n ? c0 + A.chunk : n;
    const double q = A.q;
    const double INF = __builtin_inf();
    if (tid == 0) { s_first = INT_MAX; s_last = -1; }
    STAMP_DECL

    int nA = 0;
    int64_t P0prev = 0, P1prev = 0;
    /* the next tile's first chunk of new samples is loaded during this tile's walk */
    double vpre = INF;
    int64_t apre = -1;
    for (int64_t i0 = c0; i0 < cend; i0 += T) {
        const int64_t i1 = i0 + T < cend ? i0 + T : cend;
        int64_t sA, eA, sB, eB;
        win_bounds(i0, n, W, sA, eA);
        win_bounds(i1 - 1, n, W, sB, eB);
        const int64_t P0 = sA > t0 ? sA : t0;
        const int64_t P1 = eB > P0 ? eB : P0;
        STAMP(7);
        /* ---- positions < P0 leave, [max(P1prev,P0), P1) enter (chunks of <= T) ---- */
        bool pending_rem = false;
        if (nA > 0 && P0 > P0prev) {
            if (P0 >= P1prev) nA = 0;
            else pending_rem = true;
        }
        const uint16_t b16 = (uint16_t)P0prev;
        const int cut = (int)(P0 - P0prev);
        int64_t a = P1prev > P0 ? P1prev : P0;
        do {
            const int64_t b = a + T < P1 ? a + T : P1;
            const int nn = b > a ? (int)(b - a) : 0;
            if (nn == 0 && !pending_rem) break;
            /* (1) this thread's slice of A into registers, removed flags counted */
            const int CH = (nA + T - 1) / T;
            const int j0 = tid * CH < nA ? tid * CH : nA;
            const int j1 = j0 + CH < nA ? j0 + CH : nA;
            double ov[RQ_MAXCH];
            uint16_t op[RQ_MAXCH];
            int rc = 0;
#pragma unroll
            for (int c = 0; c < RQ_MAXCH; ++c) {
                if (j0 + c < j1) {
                    ov[c] = Av[j0 + c];
                    op[c] = Ap[j0 + c];
                    rc += (pending_rem && (uint16_t)(op[c] - b16) < cut) ? 1 : 0;
                }
            }
            /* (2) sort the new values: bitonic per wave in registers, then rank across runs */
            double v = (a == apre) ? vpre : (tid < nn ? dense[a + tid] : INF);
            int p = tid;
            for (int k = 2; k <= 64; k <<= 1) {
                for (int j = k >> 1; j > 0; j >>= 1) {
                    const double vo = __shfl_xor(v, j);
                    const int po = __shfl_xor(p, j);
                    const bool other_less = vo < v || (vo == v && po < p);
                    const bool lower = (lane & j) == 0, up = (lane & k) == 0;
                    if (lower == up ? other_less : !other_less) { v = vo; p = po; }
                }
            }
            runv[tid] = v;
            int rtot;
            const int rpre = block_scan_int<T>(rc, sh, &rtot);   /* barriers: runs visible after */
            STAMP(0);
            rpref[tid] = rpre;
            if (tid == 0) rpref[T] = rtot;
            int ub = 0, r = lane;
            if (p < nn) {
                for (int w2 = 0; w2 < T / 64; ++w2) {
                    if (w2 == wid) continue;
                    const double *rv = runv + w2 * 64;
                    int lo3 = 0, hi3 = 64;
                    if (w2 < wid) {   /* earlier positions: equal values rank before */
                        while (lo3 < hi3) { int mid = (lo3 + hi3) >> 1; if (rv[mid] <= v) lo3 = mid + 1; else hi3 = mid; }
                    } else {
                        while (lo3 < hi3) { int mid = (lo3 + hi3) >> 1; if (rv[mid] < v) lo3 = mid + 1; else hi3 = mid; }
                    }
                    r += lo3;
                }
                /* insertion point among the old values (ties: new after old) */
                ub = upper_bound_lds(Av, nA, v);
                nsv[r] = v;
                nsp[r] = (uint16_t)(a + p);
                ubv[r] = (uint16_t)ub;
            }
            __syncthreads();
            STAMP(1);
            /* (3) destinations: old j -> j - removed_before(j) + #{new with ub <= j};
             *                   new rank r -> r + ub - removed_before(ub) */
            int odst[RQ_MAXCH];
            {
                int lo2 = 0, hi2 = nn;
                while (lo2 < hi2) { int mid = (lo2 + hi2) >> 1; if (ubv[mid] <= j0) lo2 = mid + 1; else hi2 = mid; }
                int ptr = lo2, rm = rpre;
#pragma unroll
                for (int c = 0; c < RQ_MAXCH; ++c) {
                    odst[c] = -1;
                    if (j0 + c < j1) {
                        const int j = j0 + c;
                        while (ptr < nn && ubv[ptr] <= j) ptr++;
                        if (pending_rem && (uint16_t)(op[c] - b16) < cut) { rm++; continue; }
                        odst[c] = j - rm + ptr;
                    }
                }
            }
            int ndst = -1;
            if (p < nn) {
                int rb = 0;
                if (pending_rem) {
                    const int c = CH > 0 ? (ub / CH < T ? ub / CH : T) : 0;
                    rb = rpref[c];
                    for (int j = c * CH; j < ub; ++j) rb += ((uint16_t)(Ap[j] - b16) < cut) ? 1 : 0;
                }
                ndst = r + ub - rb;
            }
            __syncthreads();
            /* (4) write the merged order in place */
#pragma unroll
            for (int c = 0; c < RQ_MAXCH; ++c)
                if (j0 + c < j1 && odst[c] >= 0) { Av[odst[c]] = ov[c]; Ap[odst[c]] = op[c]; }
            if (ndst >= 0) { Av[ndst] = v; Ap[ndst] = (uint16_t)(a + p); }
            __syncthreads();
            STAMP(2);
            nA = nA - rtot + nn;
            pending_rem = false;
            a = b;
        } while (a < P1);
        P0prev = P0;
        P1prev = P1 > P1prev ? P1 : P1prev;
        if (i0 + T < cend) {   /* prefetch the next tile's first chunk of new samples */
            const int64_t i0n = i0 + T, i1n = i0n + T < cend ? i0n + T : cend;
            int64_t sAn, eAn, sBn, eBn;
            win_bounds(i0n, n, W, sAn, eAn);
            win_bounds(i1n - 1, n, W, sBn, eBn);
            const int64_t P0n = sAn > t0 ? sAn : t0;
            const int64_t P1n = eBn > P0n ? eBn : P0n;
            const int64_t an = P1prev > P0n ? P1prev : P0n;
            const int64_t bn = an + T < P1n ? an + T : P1n;
            apre = an;
            vpre = (an + tid < bn) ? dense[an + tid] : INF;
        }

        /* ---- edge list: sorted indices whose position may be outside some window of the tile ---- */
        const int64_t LE = sB > t0 ? sB : t0;   /* positions < LE: left edge */
        const int64_t RE = eA;                   /* positions >= RE: right edge */
        const int relLE = (int)(LE - P0), relRE = (int)(RE - P0);
        const uint16_t p16 = (uint16_t)P0;
        const int nwords = (nA + 63) >> 6;
        for (int w = wid; w < nwords; w += T / 64) {
            const int j = (w << 6) + lane;
            const int rel = j < nA ? (int)(uint16_t)(Ap[j] - p16) : 0;
            const bool bit = j < nA && (rel < relLE || rel >= relRE);
            const unsigned long long word = __ballot(bit);
            if (lane == 0) wpre[w] = __popcll(word);
        }
        __syncthreads();
        if (wid == 0) {
            int c = lane < nwords ? wpre[lane] : 0, x = c;
            for (int o = 1; o < 64; o <<= 1) { int y = __shfl_up(x, o); if (lane >= o) x += y; }
            if (lane < nwords) wpre[lane] = x - c;
            if (lane == 63) s_nE = x;
        }
        __syncthreads();
        for (int w = wid; w < nwords; w += T / 64) {
            const int j = (w << 6) + lane;
            const int rel = j < nA ? (int)(uint16_t)(Ap[j] - p16) : 0;
            const bool bit = j < nA && (rel < relLE || rel >= relRE);
            const unsigned long long word = __ballot(bit);
            if (bit) E[wpre[w] + __popcll(word & ((1ull << lane) - 1ull))] = (uint32_t)j | ((uint32_t)rel << 16);
        }
        __syncthreads();
        const int nE = s_nE;
        STAMP(3);

        /* ---- one output per lane; the wave walks the edge list in lockstep ----
         * qa: k-th valid sorted index  = k + #excluded edges at indices <= qa (fixpoint)
         * qb: next valid index after qa = qa+1 + #excluded edges met at exactly qb      */
        const int64_t i = i0 + tid;
        int64_t s = 0, e = 0;
        win_bounds(i < n ? i : n - 1, n, W, s, e);
        const int64_t lo = s > t0 ? s : t0;
        const int64_t nobs = (i < i1 && e > lo) ? e - lo : 0;
        const bool valid = nobs >= minp && nobs > 0;
        const int xlo = (int)(lo - P0), xhi = (int)(e - P0);
        int64_t k = 0;
        double idxf = 0;
        if (valid && nobs > 1) {
            idxf = q * (double)(nobs - 1);
            k = (int64_t)idxf;
        }
        /* excluded edges e_1 < e_2 < ... (sorted indices): the k-th valid index is
         * qa = k + #{j : e_j - (j-1) <= k}, and e_j - (j-1) never decreases, so one
         * pass with a running excluded-count jx is exact and can stop early.  Pure
         * integer VALU (sign-bit tests); the edge arrives in an SGPR. */
        int jx = 0, m = 0;
        const int kk = valid ? (int)k : -(1 << 30);   /* invalid lanes never count */
        for (int e0 = 0; e0 < nE; e0 += 64) {
            const uint32_t mine = (e0 + lane < nE) ? E[e0 + lane] : 0xFFFFFFFFu;
            const int sfirst = (int)(__builtin_amdgcn_readfirstlane((int)mine) & 0xFFFF);
            if (!__ballot(sfirst - jx <= kk)) break;          /* no lane can count another edge */
            const int cnt = nE - e0 < 64 ? nE - e0 : 64;
            for (int u = 0; u < cnt; ++u) {
                const uint32_t ent = (uint32_t)__builtin_amdgcn_readlane((int)mine, u);
                const int sj = (int)(ent & 0xFFFFu), pj = (int)(ent >> 16);
                const int ex = (int)((uint32_t)((pj - xlo) | (xhi - 1 - pj)) >> 31);
                const int ok = 1 - (int)((uint32_t)(kk - sj + jx) >> 31);
                m += ex & ok;
                jx += ex;
            }
        }
        const int qa = (int)k + m;
        int qb = qa + 1;
        if (valid && nobs > 1) {   /* next valid sorted index after qa: skip excluded positions */
            for (;;) {
                const int rel = (int)(uint16_t)(Ap[qb] - p16);
                if (rel >= xlo && rel < xhi) break;
                ++qb;
            }
        }
        STAMP(4);
        if (i < i1) {
            double res = __builtin_nan("");
            if (valid) {
                const double va = Av[qa];
                if (nobs == 1 || (double)k == idxf) res = va;
                else {
                    const double vb = Av[qb];
                    res = va + (vb - va) * (idxf - (double)k);
                }
            }
            out[i] = res;
        }
        {
            const unsigned long long vm = __ballot(valid);
            if (vm && lane == 0) {
                atomicMin(&s_first, (int)(i0 + wid * 64 + __ffsll((long long)vm) - 1));
                atomicMax(&s_last, (int)(i0 + wid * 64 + 63 - __clzll(vm)));
            }
        }
        __syncthreads();
        STAMP(5);
    }
    STAMP_FLUSH(A.stamps);
    /* first / last valid output of this chunk -> the recording's (k_rollq_fill) */
    if (tid == 0 && s_last >= 0) {
        atomicMin(&A.vfirst[f], s_first);
        atomicMax(&A.vlast[f], s_last);
    }
}

/* The same sorted-union algorithm for windows beyond the LDS kernel (any
 * noise_window_sec on any length): the union lives in global scratch, double
 * buffered (a merge reads the old order and writes the new one, so no slice
 * has to fit in registers), positions are absolute int32 (no 16-bit wrap),
 * and the edge list carries (sorted index, relative position) as two words.
 * Only the per-64-word edge prefix stays in LDS (cap/64 + 2 ints).  Each
 * workgroup owns 2 x cap (f64 + i32) of scratch at A.gv / A.gp + wg * 2 cap. */
template <int T>
__global__ __launch_bounds__(T) void k_rolling_quantile_g(RollqArgs A) {
    const int f = blockIdx.x;
    if (f >= A.n_files || !A.run[f]) return;
    if (A.doff[f + 1] - A.doff[f] <= A.wm_max) return;       /* done by k_rollq_wm */
    const int64_t c0 = (int64_t)blockIdx.y * A.chunk;
    if (c0 >= A.doff[f + 1] - A.doff[f]) return;
    extern __shared__ __align__(16) unsigned char smem[];
    const int64_t cap = A.gcap;
    const int64_t wg = (int64_t)blockIdx.x * gridDim.y + blockIdx.y;
    double *Vb[2] = {A.gv + wg * 2 * cap, A.gv + wg * 2 * cap + cap};
    int32_t *Pb[2] = {A.gp + wg * 2 * cap, A.gp + wg * 2 * cap + cap};
    int cur = 0;
    double *nsv = (double *)smem;                    /* [T] new values, sorted */
    double *runv = nsv + T;                          /* [T] per-wave sorted runs */
    int32_t *nsp = (int32_t *)(runv + T);            /* [T] */
    int32_t *ubv = nsp + T;                          /* [T] */
    int *rpref = ubv + T;                            /* [T+1] */
    int *sh = rpref + T + 1;                         /* [T/64+2] */
    int32_t *Ej = sh + T / 64 + 2;                   /* [2T] edge: sorted index */
    int32_t *Er = Ej + 2 * T;                        /* [2T] edge: position relative to P0 */
    int *wpre = Er + 2 * T;                          /* [cap/64 + 2] */
    __shared__ int s_first, s_last, s_nE;

    const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    const double *dense = A.dense + d0;
    double *out = A.out + d0;
    const int64_t W = A.window, minp = A.min_periods;
    const int64_t t0 = A.troughs[d0];
    const int64_t cend = c0 + A.chunk < n ? c0 + A.chunk : n;
    const double q = A.q;
    const double INF = __builtin_inf();
    if (tid == 0) { s_first = INT_MAX; s_last = -1; }

    int64_t nA = 0;
    int64_t P0prev = 0, P1prev = 0;
    for (int64_t i0 = c0; i0 < cend; i0 += T) {
        const int64_t i1 = i0 + T < cend ? i0 + T : cend;
        int64_t sA, eA, sB, eB;
        win_bounds(i0, n, W, sA, eA);
        win_bounds(i1 - 1, n, W, sB, eB);
        const int64_t P0 = sA > t0 ? sA : t0;
        const int64_t P1 = eB > P0 ? eB : P0;
        bool pending_rem = false;
        if (nA > 0 && P0 > P0prev) {
            if (P0 >= P1prev) nA = 0;
            else pending_rem = true;
        }
        int64_t a = P1prev > P0 ? P1prev : P0;
        do {
            const int64_t b = a + T < P1 ? a + T : P1;
            const int nn = b > a ? (int)(b - a) : 0;
            if (nn == 0 && !pending_rem) break;
            const double *Av = Vb[cur];
            const int32_t *Ap = Pb[cur];
            double *Bv = Vb[cur ^ 1];
            int32_t *Bp = Pb[cur ^ 1];
            /* (1) this thread's slice of the old order: removed positions counted */
            const int64_t CH = (nA + T - 1) / T;
            const int64_t j0 = tid * CH < nA ? tid * CH : nA;
            const int64_t j1 = j0 + CH < nA ? j0 + CH : nA;
            int rc = 0;
            if (pending_rem)
                for (int64_t j = j0; j < j1; ++j) rc += Ap[j] < P0 ? 1 : 0;
            /* (2) the new values: bitonic per wave, ranked across the runs */
            double v = tid < nn ? dense[a + tid] : INF;
            int p = tid;
            for (int k = 2; k <= 64; k <<= 1) {
                for (int j = k >> 1; j > 0; j >>= 1) {
                    const double vo = __shfl_xor(v, j);
                    const int po = __shfl_xor(p, j);
                    const bool other_less = vo < v || (vo == v && po < p);
                    const bool lower = (lane & j) == 0, up = (lane & k) == 0;
                    if (lower == up ? other_less : !other_less) { v = vo; p = po; }
                }
            }
            runv[tid] = v;
            int rtot;
            const int rpre = block_scan_int<T>(rc, sh, &rtot);
            rpref[tid] = rpre;
            if (tid == 0) rpref[T] = rtot;
            int64_t ub = 0;
            int r = lane;
            if (p < nn) {
                for (int w2 = 0; w2 < T / 64; ++w2) {
                    if (w2 == wid) continue;
                    const double *rv = runv + w2 * 64;
                    int lo3 = 0, hi3 = 64;
                    if (w2 < wid) {
                        while (lo3 < hi3) { int mid = (lo3 + hi3) >> 1; if (rv[mid] <= v) lo3 = mid + 1; else hi3 = mid; }
                    } else {
                        while (lo3 < hi3) { int mid = (lo3 + hi3) >> 1; if (rv[mid] < v) lo3 = mid + 1; else hi3 = mid; }
                    }
                    r += lo3;
                }
                int64_t lo = 0, hi = nA;                 /* upper bound among the old values */
                while (lo < hi) { const int64_t mid = (lo + hi) >> 1; if (Av[mid] <= v) lo = mid + 1; else hi = mid; }
                ub = lo;
                nsv[r] = v;
                nsp[r] = (int32_t)(a + p);
                ubv[r] = (int32_t)ub;
            }
            __syncthreads();
            /* (3)+(4) old j -> j - removed_before(j) + #{new with ub <= j};
             *         new rank r -> r + ub - removed_before(ub) */
            {
                int lo2 = 0, hi2 = nn;
                while (lo2 < hi2) { int mid = (lo2 + hi2) >> 1; if (ubv[mid] <= j0) lo2 = mid + 1; else hi2 = mid; }
                int ptr = lo2;
                int64_t rm = rpre;
                for (int64_t j = j0; j < j1; ++j) {
                    while (ptr < nn && ubv[ptr] <= j) ptr++;
                    const int32_t pj = Ap[j];
                    if (pending_rem && pj < P0) { rm++; continue; }
                    const int64_t dst = j - rm + ptr;
                    Bv[dst] = Av[j];
                    Bp[dst] = pj;
                }
            }
            if (p < nn) {
                int64_t rb = 0;
                if (pending_rem) {
                    const int64_t c = CH > 0 ? (ub / CH < T ? ub / CH : T) : 0;
                    rb = rpref[c];
                    for (int64_t j = c * CH; j < ub; ++j) rb += Ap[j] < P0 ? 1 : 0;
                }
                const int64_t dst = r + ub - rb;
                Bv[dst] = v;
                Bp[dst] = (int32_t)(a + p);
            }
            __syncthreads();
            cur ^= 1;
            nA = nA - rtot + nn;
            pending_rem = false;
            a = b;
        } while (a < P1);
        P0prev = P0;
        P1prev = P1 > P1prev ? P1 : P1prev;
        const double *Av = Vb[cur];
        const int32_t *Ap = Pb[cur];

        /* ---- edge list: sorted indices whose position may be outside some window of the tile ---- */
        const int64_t LE = sB > t0 ? sB : t0, RE = eA;
        const int nwords = (int)((nA + 63) >> 6);
        for (int w = wid; w < nwords; w += T / 64) {
            const int64_t j = ((int64_t)w << 6) + lane;
            const int32_t pj = j < nA ? Ap[j] : 0;
            const bool bit = j < nA && (pj < LE || pj >= RE);
            const unsigned long long word = __ballot(bit);
            if (lane == 0) wpre[w] = __popcll(word);
        }
        __syncthreads();
        if (wid == 0) {                                  /* exclusive scan of the word counts */
            int run = 0;
            for (int w0 = 0; w0 < nwords; w0 += 64) {
                const int c = w0 + lane < nwords ? wpre[w0 + lane] : 0;
                int x = c;
                for (int o = 1; o < 64; o <<= 1) { const int y = __shfl_up(x, o); if (lane >= o) x += y; }
                if (w0 + lane < nwords) wpre[w0 + lane] = run + x - c;
                run += __shfl(x, 63);
            }
            if (lane == 0) s_nE = run;
        }
        __syncthreads();
        for (int w = wid; w < nwords; w += T / 64) {
            const int64_t j = ((int64_t)w << 6) + lane;
            const int32_t pj = j < nA ? Ap[j] : 0;
            const bool bit = j < nA && (pj < LE || pj >= RE);
            const unsigned long long word = __ballot(bit);
            if (bit) {
                const int k = wpre[w] + __popcll(word & ((1ull << lane) - 1ull));
                Ej[k] = (int32_t)j;
                Er[k] = (int32_t)(pj - P0);
            }
        }
        __syncthreads();
        const int nE = s_nE;

        /* ---- one output per thread (the LDS kernel's edge walk) ---- */
        const int64_t i = i0 + tid;
        int64_t s = 0, e = 0;
        win_bounds(i < n ? i : n - 1, n, W, s, e);
        const int64_t lo = s > t0 ? s : t0;
        const int64_t nobs = (i < i1 && e > lo) ? e - lo : 0;
        const bool valid = nobs >= minp && nobs > 0;
        const int64_t xlo = lo - P0, xhi = e - P0;
        int64_t k = 0;
        double idxf = 0;
        if (valid && nobs > 1) {
            idxf = q * (double)(nobs - 1);
            k = (int64_t)idxf;
        }
        int64_t jx = 0, m = 0;
        if (valid) {
            for (int u = 0; u < nE; ++u) {
                const int64_t sj = Ej[u], pj = Er[u];
                if (sj - jx > k) break;                  /* e_j - (j-1) never decreases */
                const bool ex = pj < xlo || pj >= xhi;
                m += ex ? 1 : 0;
                jx += ex ? 1 : 0;
            }
        }
        const int64_t qa = k + m;
        int64_t qb = qa + 1;
        if (valid && nobs > 1) {
            for (;;) {
                const int64_t rel = Ap[qb] - P0;
                if (rel >= xlo && rel < xhi) break;
                ++qb;
            }
        }
        if (i < i1) {
            double res = __builtin_nan("");
            if (valid) {
                const double va = Av[qa];
                if (nobs == 1 || (double)k == idxf) res = va;
                else {
                    const double vb = Av[qb];
                    res = va + (vb - va) * (idxf - (double)k);
                }
            }
            out[i] = res;
        }
        {
            const unsigned long long vm = __ballot(valid);
            if (vm && lane == 0) {
                atomicMin(&s_first, (int)(i0 + wid * 64 + __ffsll((long long)vm) - 1));
                atomicMax(&s_last, (int)(i0 + wid * 64 + 63 - __clzll(vm)));
            }
        }
        __syncthreads();
    }
    if (tid == 0 && s_last >= 0) {
        atomicMin(&A.vfirst[f], s_first);
        atomicMax(&A.vlast[f], s_last);
    }
}
template __global__ void k_rolling_quantile_g<256>(RollqArgs A);

/* .bfill().ffill() of the chunked rolling quantile: nobs(i) is unimodal, so
 * the NaN outputs are a prefix and a suffix; fill them from the first and
 * last valid output over all chunks (or flag the recording all-NaN). */
__global__ __launch_bounds__(256) void k_rollq_fill(RollqArgs A) {
    const int f = blockIdx.y;
    if (f >= A.n_files || !A.run[f]) return;
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    if (n <= A.wm_max) return;
    const int first = A.vfirst[f], last = A.vlast[f];
    if (last < 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) A.allnan[f] = 1;
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) A.allnan[f] = 0;
    double *out = A.out + d0;
    const double vf = out[first], vl = out[last];
    const int64_t stride = (int64_t)gridDim.x * 256, i00 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (int64_t i = i00; i < first; i += stride) out[i] = vf;
    for (int64_t i = last + 1 + i00; i < n; i += stride) out[i] = vl;
}

template __global__ void k_rolling_quantile<256, 16>(RollqArgs A);
template __global__ void k_rolling_quantile<256, 32>(RollqArgs A);

/* ------------------------------------------------------------------------ */
__global__ __launch_bounds__(256) void k_sanitize(SanitizeArgs A) {
    __shared__ int sh[256 / 64 + 1];
    const int f = blockIdx.x;
    if (f < A.n_files && A.active[f]) (void)sanitize_wg<256>(A, f, sh);
}

/* ------------------------------------------------------------------------ */
/* k_draft_bounds (see DraftBoundArgs).  Per raw trough t: the draft value is
 * r = rolling(W, min_periods, center).quantile(q) at t after bfill/ffill, i.e.
 * at t clamped to the valid outputs [vfirst, vlast]; with nobs window values,
 * k = int(q (nobs - 1)) and r in [s_k, s_(k+1)] (= s_k when q (nobs-1) is whole).
 * Window values lie on segments [t_j, t_(j+1)) of the trough curve (the last
 * one constant), each monotone between env[t_j] and env[t_(j+1)], so with
 * lo_j / hi_j the segment's end values and len_j its samples in the window:
 *   L = min{ lo_j : sum(len_i : lo_i <= lo_j) > k }          -> s_k >= L
 *   U = min{ hi_j : sum(len_i : hi_i <= hi_j) >= k + 2 (k + 1) } -> s_(k+1) <= U
 * keep iff env[t] <= mult r: certain when env[t] <= mult L, certainly not
 * when env[t] > mult U (1 + 2^-50); anything else makes the recording exact. */

/* One walk over the segments in value order: the first whose cumulative
 * in-window length passes thr (> thr, or >= thr with GE) gives the bound.  A
 * segment lies in the window [lo, hi) iff its overlap is positive; records are
 * read DB_WALK at a time ahead of the (sequential) accumulation, which has no
 * branch per record.  (Both walks in one loop, two chunks of reads in flight:
 * no faster.) */
template <bool GE>
__device__ __forceinline__ double db_walk(const DbSeg *sg, int m, int32_t lo, int32_t hi, int64_t thr) {
    constexpr int DB_WALK = 8;
    int64_t c = 0;
    for (int r = 0; r < m; r += DB_WALK) {
        DbSeg g[DB_WALK];
#pragma unroll
        for (int u = 0; u < DB_WALK; ++u) g[u] = sg[r + u < m ? r + u : m - 1];
        double res = 0.0;
        bool hit = false;
#pragma unroll
        for (int u = 0; u < DB_WALK; ++u) {
            const int32_t a = lo > g[u].s ? lo : g[u].s;
            const int32_t b = hi < g[u].e ? hi : g[u].e;
            const int32_t d = (r + u < m && b > a) ? b - a : 0;
            c += d;
            const bool h = !hit && d > 0 && (GE ? c >= thr : c > thr);   /* the first record past thr */
            res = h ? g[u].v : res;
            hit = hit || h;
        }
        if (hit) return res;
    }
    return __builtin_inf();
}

/* Exact draft value at one raw trough, by one wave (every lane active, wave-
 * uniform arguments): the centred rolling quantile of the trough curve at
 * output qp, i.e. k-th / (k+1)-th smallest of the window [lo, hi) of
 * interp_at's values (bpm_analysis.py:1081-1086).  The window covers segments
 * jl..jh of the staged troughs; lane l owns segments jl + l + 64 r.  Within a
 * segment the values fl(slope (x - t_j)) + y_j are weakly monotone in x
 * (rounding is monotone), so in ascending order they read val(a + i) on a
 * rising segment and val(b - 1 - i) on a falling one, and the number below a
 * value is one binary search.  Selection by random pivots: each round takes an
 * active element uniformly (wave prefix scan), counts the elements < and <= it
 * in every segment, and keeps the side holding rank k: expected O(log nobs)
 * rounds.  The (k+1)-th is the k-th itself when enough equal it, else the least
 * element above it (one more binary search position per segment).  Returns
 * false for what it does not take (more than 64 DP_SPL segments, non-finite
 * trough values): the recording then gets the full draft. */
constexpr int DP_SPL_MAX = 4;
#ifndef BPMX_DP_WAVES
#define BPMX_DP_WAVES 5   /* waves per SIMD the one-segment k_draft_points is compiled for (r06: 6 spilled 33 VGPRs; 5: 0.114 -> 0.106 ms on the reference sample) */
#endif
constexpr int DP_IP_ROUNDS = 8;
constexpr int DP_FIX = 4;         /* exact steps after a segment's inverse estimate before bisection */   /* interpolated value pivots before random element pivots */

template <int DP_SPL>
__device__ __forceinline__ bool draft_point(const int32_t *s_tp, const double *s_tv, int base, int m, int64_t n,
                                            int64_t lo, int64_t hi, int jl, int jh, double q, uint32_t seed,
                                            double *res, double seedv = __builtin_nan(""), double *rho = nullptr,
                                            double theta = __builtin_nan(""), int *decided = nullptr) {
    const int lane = lane_id();
    if (decided) *decided = -1;
    if (jh - jl + 1 > 64 * DP_SPL) return false;
    int32_t sa[DP_SPL], sn[DP_SPL], st[DP_SPL], slo[DP_SPL], shi[DP_SPL], sub[DP_SPL];
    double sy[DP_SPL], ssl[DP_SPL], sinv[DP_SPL];
    bool sinc[DP_SPL], scst[DP_SPL];
    bool ok = true;
#pragma unroll
    for (int r = 0; r < DP_SPL; ++r) {
        const int i = jl + lane + 64 * r;
        sn[r] = 0; sa[r] = 0; st[r] = 0; sy[r] = 0.0; ssl[r] = 0.0; sinv[r] = 0.0; sinc[r] = true; scst[r] = true;
        if (i <= jh) {
            const int64_t tj = s_tp[i - base];
            const int64_t nx = i + 1 < m ? (int64_t)s_tp[i + 1 - base] : n;
            const int64_t a = lo > tj ? lo : tj, b = hi < nx ? hi : nx;
            const double y0 = s_tv[i - base];
            double y1 = y0, sl = 0.0;
            if (i + 1 < m) {
                y1 = s_tv[i + 1 - base];
                sl = (y1 - y0) / ((double)nx - (double)tj);      /* interp_at's slope */
                scst[r] = false;
            }
            ok = ok && __builtin_isfinite(y0) && __builtin_isfinite(y1) && __builtin_isfinite(sl);
            sa[r] = (int32_t)a; sn[r] = (int32_t)(b - a); st[r] = (int32_t)tj;
            sy[r] = y0; ssl[r] = sl; sinc[r] = y1 >= y0;
            sinv[r] = sl != 0.0 ? 1.0 / sl : 0.0;
        }
        slo[r] = 0; shi[r] = sn[r]; sub[r] = 0;
    }
    if (__ballot(!ok) != 0) return false;
    /* value of segment r at ascending rank i (interp_at, -ffp-contract=off) */
    auto sorted = [&](int r, int i) -> double {
        const int64_t x = sinc[r] ? (int64_t)sa[r] + i : (int64_t)sa[r] + sn[r] - 1 - i;
        if (scst[r] || x == st[r]) return sy[r];
        return ssl[r] * ((double)x - (double)st[r]) + sy[r];
    };
    const int64_t nobs = hi - lo;
    double idxf = 0.0;
    int64_t k = 0;
    if (nobs > 1) {
        idxf = q * (double)(nobs - 1);
        k = (int64_t)idxf;
    }
    const bool interp = !(nobs == 1 || (double)k == idxf);
    int64_t below = 0, leq = -1;
    double va = 0.0;
    uint32_t rng = seed;
    bool seed_down = false;
    int64_t seed_nless = 0, seed_nleq = 0;
    /* decision mode (theta = env[t] / mult, finite): the caller needs only
     * whether env[t] <= mult * value.  The first two pivots are theta pushed
     * up and down by 2^-48 (far beyond the rounding of the division and of
     * mult * value): fewer than k + 1 elements below the upper one puts s_k,
     * hence the value, above it (keep); at least k + 2 (k + 1 without
     * interpolation) below the lower one puts s_(k+1) (s_k), hence the value,
     * under it (drop).  Either ends the selection after one or two counts;
     * otherwise the rounds go on from the narrowed active set. */
    const bool dmode = decided && __builtin_isfinite(theta);
    const int ib = dmode ? 2 : 0;
    for (int it = 0; it < 256; ++it) {
        const int it2 = it - ib;
        int cnt = 0;
#pragma unroll
        for (int r = 0; r < DP_SPL; ++r) cnt += shi[r] - slo[r];
        const int incl = wave_iscan_dpp<false>(cnt);
        const int tot = __shfl(incl, 63);
        if (tot <= 0) return false;
        const int excl = incl - cnt;
        if (DP_SPL == 1 && tot <= 64) {
            /* few left: lane o takes the active element at offset o (its
             * segment's parameters fetched from the owning lane), a bitonic
             * sort across the wave, then the (k - below)-th and the next */
            const int o = lane;
            int s = 0;                                       /* owner: last lane with excl <= o */
#pragma unroll
            for (int b = 32; b > 0; b >>= 1) {
                const int ex = __shfl(excl, s + b - 1 + 1 > 63 ? 63 : s + b);
                if (s + b <= 63 && ex <= o) s += b;
            }
            const int exs = __shfl(excl, s), los = __shfl(slo[0], s), sas = __shfl(sa[0], s), sns = __shfl(sn[0], s);
            const int sts = __shfl(st[0], s);
            const double sys = __shfl(sy[0], s), ssls = __shfl(ssl[0], s);
            const bool incs = __shfl((int)sinc[0], s) != 0, csts = __shfl((int)scst[0], s) != 0;
            double x = __builtin_inf();
            if (o < tot) {
                const int i = los + (o - exs);
                const int64_t xp = incs ? (int64_t)sas + i : (int64_t)sas + sns - 1 - i;
                x = (csts || xp == sts) ? sys : ssls * ((double)xp - (double)sts) + sys;
            }
#pragma unroll
            for (int kk = 2; kk <= 64; kk <<= 1) {
#pragma unroll
                for (int jj = kk >> 1; jj > 0; jj >>= 1) {
                    const double y = __shfl_xor(x, jj);
                    const bool up = (lane & kk) == 0, lower = (lane & jj) == 0;
                    x = (lower == up) ? fmin(x, y) : fmax(x, y);
                }
            }
            const int t = (int)(k - below);
            va = __shfl(x, t);
            if (rho) {                                       /* elements per unit value near the answer */
                const double x0 = __shfl(x, 0), x1 = __shfl(x, tot - 1);
                *rho = x1 > x0 ? (double)(tot - 1) / (x1 - x0) : __builtin_nan("");
            }
            if (!interp) {
                *res = va;
                return true;
            }
            double vb;
            if (t + 1 < tot) {
                vb = __shfl(x, t + 1);
            } else {                                         /* the least element above the active ones */
                const double mn = shi[0] < sn[0] ? sorted(0, shi[0]) : __builtin_inf();
                vb = wave_min(mn);
            }
            *res = va + (vb - va) * (idxf - (double)k);
            return true;
        }
        double pv;
        if (it < ib) {
            pv = it == 0 ? theta * (1.0 + 0x1p-48) : theta * (1.0 - 0x1p-48);
        } else if (it2 == 0 && __builtin_isfinite(seedv)) {
            /* the neighbouring trough's draft value: its window overlaps this
             * one but for a few segments, so the count there lands near k */
            pv = seedv;
        } else if (it2 == 1 && __builtin_isfinite(seedv) && rho && *rho > 0.0 && __builtin_isfinite(*rho)) {
            /* then a step from it by the count still missing over the
             * neighbour's density of values near its answer */
            pv = seed_down ? seedv - ((double)(seed_nless - k) - 0.5) / *rho
                           : seedv + ((double)(k - seed_nleq) + 0.5) / *rho;
        } else if (it2 < DP_IP_ROUNDS) {
            /* a value pivot interpolated between the active extremes at the
             * target's rank: the values within a segment are evenly spaced, so
             * the active set shrinks by far more than a random pivot's half */
            double amin = __builtin_inf(), amax = -__builtin_inf();
#pragma unroll
            for (int r = 0; r < DP_SPL; ++r)
                if (shi[r] > slo[r]) { amin = fmin(amin, sorted(r, slo[r])); amax = fmax(amax, sorted(r, shi[r] - 1)); }
            amin = wave_min(amin);
            amax = wave_max(amax);
            if (!(amin < amax)) {                            /* every active element is equal */
                va = amin;
                leq = below + tot;
#pragma unroll
                for (int r = 0; r < DP_SPL; ++r) sub[r] = shi[r];   /* beyond: larger values only */
                break;
            }
            pv = amin + (amax - amin) * (((double)(k - below) + 0.5) / (double)tot);
            pv = fmin(fmax(pv, amin), amax);
        } else {
            rng = rng * 1664525u + 1013904223u;
            const int p = (int)(((uint64_t)rng * (uint64_t)tot) >> 32);
            const bool own = p >= excl && p < incl;
            const int owner = __ffsll((unsigned long long)__ballot(own)) - 1;
            double pvl = 0.0;
            if (own) {
                int off = p - excl;
#pragma unroll
                for (int r = 0; r < DP_SPL; ++r) {
                    const int c = shi[r] - slo[r];
                    if (off >= 0 && off < c) pvl = sorted(r, slo[r] + off);
                    off -= c;
                }
            }
            pv = __shfl(pvl, owner);
        }
        int slb[DP_SPL];
        int cl = 0, ce = 0;
#pragma unroll
        for (int r = 0; r < DP_SPL; ++r) {
            /* first active rank with a value >= pv, then > pv: started from
             * the segment formula's inverse (values evenly spaced) and made
             * exact by stepping over at most DP_FIX neighbours; a search
             * that needs more is finished by bisection */
            const int l0 = slo[r], h0 = shi[r];
            int i = l0;
            if (l0 < h0) {
                if (scst[r] || ssl[r] == 0.0) {
                    i = sy[r] < pv ? h0 : l0;                /* every value is y0 */
                } else {
                    const double xf = (double)st[r] + (pv - sy[r]) * sinv[r];
                    const double ie = sinc[r] ? ceil(xf) - (double)sa[r] : (double)(sa[r] + sn[r] - 1) - floor(xf);
                    i = (int)fmin(fmax(ie, (double)l0), (double)h0);   /* NaN: l0 */
                    int g = 0;
                    while (i > l0 && g < DP_FIX && sorted(r, i - 1) >= pv) { --i; ++g; }
                    while (i < h0 && g < DP_FIX && sorted(r, i) < pv) { ++i; ++g; }
                    if (g >= DP_FIX) {
                        int l = l0, h = h0;
                        while (l < h) { const int mid = (l + h) >> 1; if (sorted(r, mid) < pv) l = mid + 1; else h = mid; }
                        i = l;
                    }
                }
            }
            slb[r] = i;
            int u = i;
            if (u < h0) {
                if (scst[r] || ssl[r] == 0.0) {
                    u = sy[r] <= pv ? h0 : u;
                } else {
                    int g = 0;
                    while (u < h0 && g < DP_FIX && sorted(r, u) <= pv) { ++u; ++g; }
                    if (g >= DP_FIX) {
                        int l = u, h = h0;
                        while (l < h) { const int mid = (l + h) >> 1; if (sorted(r, mid) <= pv) l = mid + 1; else h = mid; }
                        u = l;
                    }
                }
            }
            sub[r] = u;
            cl += slb[r] - slo[r];
            ce += sub[r] - slo[r];
        }
        const int64_t nless = below + wave_sum_i(cl), nleq = below + wave_sum_i(ce);
        if (it == 0 && dmode && nless <= k) { *decided = 1; return true; }
        if (it == 1 && dmode && nless >= k + (interp ? 2 : 1)) { *decided = 0; return true; }
        if (it2 == 0) { seed_down = k < nless; seed_nless = nless; seed_nleq = nleq; }
        if (k < nless) {
#pragma unroll
            for (int r = 0; r < DP_SPL; ++r) shi[r] = slb[r];
        } else if (k < nleq) {
            va = pv;
            leq = nleq;
            break;
        } else {
            below = nleq;
#pragma unroll
            for (int r = 0; r < DP_SPL; ++r) slo[r] = sub[r];
        }
    }
    if (leq < 0) return false;
    if (!interp) {
        *res = va;
        return true;
    }
    double vb = va;
    if (leq < k + 2) {
        /* the least element above va: position sub in each segment (the cut
         * above shi holds only larger values) */
        double mn = __builtin_inf();
#pragma unroll
        for (int r = 0; r < DP_SPL; ++r)
            if (sub[r] < sn[r]) mn = fmin(mn, sorted(r, sub[r]));
        vb = wave_min(mn);
    }
    *res = va + (vb - va) * (idxf - (double)k);
    return true;
}

__global__ __launch_bounds__(DB_T) void k_draft_bounds(DraftBoundArgs A) {
    const int f = blockIdx.x;
    if (f >= A.n_files || !A.run[f]) return;
    __shared__ int32_t s_tp[DB_TRMAX];
    __shared__ double s_tv[DB_TRMAX];
    /* segments by lower / upper end value: up to DB_LOCAL_M - 1 troughs as
     * {start, end, end value} records, so a walk step is one independent LDS
     * read; beyond (BPMX_OPT_DRAFT_GLOBAL_RANK only) as index lists */
    __shared__ union {
        int16_t ord[2][DB_TRMAX];
        DbSeg seg[2][DB_LOCAL_M];          /* sorted in place (bitonic, DB_LOCAL_M a power of 2) */
    } s_o;
    int16_t *s_olo = s_o.ord[0], *s_ohi = s_o.ord[1];
    DbSeg *s_slo = s_o.seg[0], *s_shi = s_o.seg[1];
    __shared__ int s_vf, s_vl;
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    const int m = A.nraw[f];
    const int tid = threadIdx.x;
    /* Long recordings (> local_m troughs) rank each window's segments in
     * place, so their troughs split over blockIdx.y chunks of DB_T, each
     * staging only the troughs its windows reach; shorter ones build the
     * recording-wide order once, in chunk 0. */
    const bool local = m > A.local_m;
    if (!local && blockIdx.y > 0) return;
    const int jc0 = local ? (int)blockIdx.y * DB_T : 0;
    const int jc1 = local ? (jc0 + DB_T < m ? jc0 + DB_T : m) : m;
    if (jc0 >= jc1) return;
    if (!local && m > DB_TRMAX) {
        if (tid == 0) A.exact[f] = 1;
        return;
    }
    const int64_t *raw = A.raw + d0;
    const double *rawv = A.rawv + d0;                        /* env at the raw troughs */
    const int64_t W = A.window, t0 = raw[0], off = (W - 1) / 2;
    if (tid == 0) { s_vf = INT_MAX; s_vl = -1; }
    __syncthreads();
    /* valid outputs (nobs >= min_periods) form one interval: with s >= t0 and
     * e <= n (outputs [t0 + W - 1 - off, n - 1 - off]) nobs = W >= min_periods,
     * so only the two edge stretches need the test */
    {
        const int64_t ma = t0 + W - 1 - off, mb = n - 1 - off;
        int vf = INT_MAX, vl = -1;
        auto test = [&](int64_t i) {
            int64_t s, e;
            win_bounds(i, n, W, s, e);
            const int64_t lo = s > t0 ? s : t0;
            if (e - lo >= A.min_periods && e > lo) { vf = min(vf, (int)i); vl = max(vl, (int)i); }
        };
        const int64_t ea = ma < n ? (ma > 0 ? ma : 0) : n;   /* [0, ea) */
        const int64_t sb = mb + 1 > ea ? mb + 1 : ea;        /* [sb, n) */
        for (int64_t i = tid; i < ea; i += DB_T) test(i);
        for (int64_t i = sb + tid; i < n; i += DB_T) test(i);
        if (tid == 0 && ea <= mb) { vf = min(vf, (int)ea); vl = max(vl, (int)min<int64_t>(mb, n - 1)); }
        for (int o = 32; o > 0; o >>= 1) { vf = min(vf, __shfl_xor(vf, o)); vl = max(vl, __shfl_xor(vl, o)); }
        if (lane_id() == 0) { atomicMin(&s_vf, vf); atomicMax(&s_vl, vl); }
    }
    __syncthreads();
    const int vf = s_vf, vl = s_vl;
    if (vl < vf) {                                     /* all-NaN draft: the exact path handles it */
        if (tid == 0) A.exact[f] = 1;
        return;
    }
    /* staged troughs [base, base + ns): all of them (global order), or the
     * chunk's plus every segment its windows touch (+1 for segment ends) */
    auto seg_of_g = [&](int64_t x) -> int {         /* last trough <= x, over global memory */
        int lo = 0, hi = m;
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (raw[mid] <= x) lo = mid + 1; else hi = mid; }
        return lo - 1;
    };
    int base = 0, ns = m;
    if (local) {
        auto qpos = [&](int j) -> int64_t { const int64_t t = raw[j]; return t < vf ? vf : (t > vl ? vl : t); };
        int64_t s, e;
        win_bounds(qpos(jc0), n, W, s, e);
        const int ja = seg_of_g(s > t0 ? s : t0);
        win_bounds(qpos(jc1 - 1), n, W, s, e);
        const int jb = seg_of_g(e - 1);
        base = min(ja, jc0);
        const int top = min(m - 1, max(jb + 1, jc1 - 1));
        ns = top - base + 1;
        if (ns > DB_TRMAX) {                           /* windows too wide to stage: exact path */
            if (tid == 0) A.exact[f] = 1;
            return;
        }
    }
    for (int j = tid; j < ns; j += DB_T) {
        s_tp[j] = (int32_t)raw[base + j];
        s_tv[j] = rawv[base + j];                            /* env at the trough */
    }
    __syncthreads();
    /* staged accessors by trough index */
    auto tp = [&](int j) -> int64_t { return s_tp[j - base]; };
    auto tv = [&](int j) -> double { return s_tv[j - base]; };
    auto seg_lo = [&](int j) -> double { return j + 1 < m ? fmin(tv(j), tv(j + 1)) : tv(j); };
    auto seg_hi = [&](int j) -> double { return j + 1 < m ? fmax(tv(j), tv(j + 1)) : tv(j); };
    /* stable ranks by end value (ties by index) of the ranked segments: all
     * of them, or (long recordings) the staged ones whose both ends are staged
     * — every segment a chunk window touches.  Under DB_LOCAL_M of them they
     * become records for the walks; more, the order lists (recording-wide,
     * BPMX_OPT_DRAFT_GLOBAL_RANK) or, for long recordings, each window's few
     * segments ranked in place (below).  Ranking a subset keeps the relative
     * order of the segments in it, so the walks stop on the same segment. */
    const int nr = local ? (base + ns == m ? ns : ns - 1) : m;
    const bool recs = nr > 0 && nr < DB_LOCAL_M;
    if (recs) {
        /* the records, then each array sorted by (end value, start) — the
         * start orders segments like their index — with a bitonic network
         * over the next power of two (pads: +inf); one compare-exchange per
         * thread and stage (both arrays at once).  The O(nr^2) rank count
         * below took 0.04 ms of f64 compares per step on the metric batch. */
        int np2 = 1;
        while (np2 < nr) np2 <<= 1;
        for (int jr = tid; jr < np2; jr += DB_T) {
            if (jr < nr) {
                const int j = base + jr;
                const int32_t se = j + 1 < m ? (int32_t)tp(j + 1) : (int32_t)n;
                s_slo[jr] = DbSeg{(int32_t)tp(j), se, seg_lo(j)};
                s_shi[jr] = DbSeg{(int32_t)tp(j), se, seg_hi(j)};
            } else {
                s_slo[jr] = s_shi[jr] = DbSeg{INT_MAX, INT_MAX, __builtin_inf()};
            }
        }
        __syncthreads();
        for (int k2 = 2; k2 <= np2; k2 <<= 1)
            for (int j2 = k2 >> 1; j2 > 0; j2 >>= 1) {
                for (int c = tid; c < np2; c += DB_T) {      /* c < np2 / 2: lower ends; the rest: upper ends */
                    DbSeg *arr = c < (np2 >> 1) ? s_slo : s_shi;
                    const int q = c & ((np2 >> 1) - 1);
                    const int i = ((q & ~(j2 - 1)) << 1) | (q & (j2 - 1));   /* i has bit j2 clear */
                    const int l = i | j2;
                    const DbSeg x = arr[i], y = arr[l];
                    const bool up = (i & k2) == 0;
                    const bool gt = x.v > y.v || (x.v == y.v && x.s > y.s);
                    if (gt == up) { arr[i] = y; arr[l] = x; }
                }
                __syncthreads();
            }
    }
    for (int jr = tid; jr < nr && !recs && !local; jr += DB_T) {
        const int j = base + jr;
        const double a = seg_lo(j), b = seg_hi(j);
        int ra = 0, rb = 0;
        double vc = s_tv[0];                       /* tv(i), carried: one LDS read per segment */
#pragma unroll 4
        for (int i = base; i < base + nr; ++i) {
            const double vn = i + 1 < m ? s_tv[i + 1 - base] : vc;
            const double ai = fmin(vc, vn), bi = fmax(vc, vn);
            ra += (ai < a || (ai == a && i < j)) ? 1 : 0;
            rb += (bi < b || (bi == b && i < j)) ? 1 : 0;
            vc = vn;
        }
        s_olo[ra] = (int16_t)j;
        s_ohi[rb] = (int16_t)j;
    }
    __syncthreads();
    auto seg_of = [&](int64_t x) -> int {           /* last trough <= x (x >= t0), among the staged */
        int lo = base, hi = base + ns;
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (tp(mid) <= x) lo = mid + 1; else hi = mid; }
        return lo - 1;
    };
    for (int j = jc0 + tid; j < jc1; j += DB_T) {
        const int64_t t = tp(j);
        const int64_t qp = t < vf ? vf : (t > vl ? vl : t);
        int64_t s, e;
        win_bounds(qp, n, W, s, e);
        const int64_t lo = s > t0 ? s : t0, hi = e, nobs = hi - lo;
        const double idxf = A.q * (double)(nobs - 1);
        const int64_t k = (int64_t)idxf;
        int64_t thr_u = ((double)k == idxf) ? k + 1 : k + 2;
        if (thr_u > nobs) thr_u = nobs;
        const int jl = seg_of(lo), jh = seg_of(hi - 1);
        auto len_of = [&](int i) -> int64_t {          /* samples of segment i inside [lo, hi) */
            const int64_t a = lo > tp(i) ? lo : tp(i);
            const int64_t se = i + 1 < m ? tp(i + 1) : n;
            return (hi < se ? hi : se) - a;
        };
        /* L: first lower end (ascending) whose in-window cumulative length exceeds k;
         * U: first upper end (ascending) whose cumulative reaches thr_u */
        double L = __builtin_inf(), U = __builtin_inf();
        if (recs) {
            L = db_walk<false>(s_slo, nr, (int32_t)lo, (int32_t)hi, k);
            U = db_walk<true>(s_shi, nr, (int32_t)lo, (int32_t)hi, thr_u);
        } else if (!local) {
            int64_t c = 0;
            for (int r = 0; r < m; ++r) {
                const int b = s_olo[r];
                if (b < jl || b > jh) continue;
                c += len_of(b);
                if (c > k) { L = seg_lo(b); break; }
            }
            c = 0;
            for (int r = 0; r < m; ++r) {
                const int b = s_ohi[r];
                if (b < jl || b > jh) continue;
                c += len_of(b);
                if (c >= thr_u) { U = seg_hi(b); break; }
            }
        } else {
            /* the same walks without the global order: segment b's cumulative
             * length over the window's segments ordered (value, index) <= b's;
             * cumulative lengths never decrease along that order, so the
             * walk's stopping segment has the least value among those whose
             * cumulative length passes the threshold */
            for (int b = jl; b <= jh; ++b) {
                const double lb = seg_lo(b), hb = seg_hi(b);
                int64_t cl = 0, ch = 0;
                for (int i = jl; i <= jh; ++i) {
                    const int64_t li = len_of(i);
                    const double loi = seg_lo(i), hii = seg_hi(i);
                    cl += (loi < lb || (loi == lb && i <= b)) ? li : 0;
                    ch += (hii < hb || (hii == hb && i <= b)) ? li : 0;
                }
                if (cl > k) L = fmin(L, lb);
                if (ch >= thr_u) U = fmin(U, hb);
            }
        }
        const double et = tv(j);
        uint8_t dcs;
        if (et <= A.mult * L) dcs = 1;
        else if (et > A.mult * U * (1.0 + 0x1p-50)) dcs = 0;
        else { dcs = 2; atomicAdd(&A.nund[f], 1); }     /* k_draft_points */
        A.dec[d0 + j] = dcs;
    }
    if (A.stats && tid == 0) atomicAdd((unsigned long long *)&A.stats[0], (unsigned long long)(jc1 - jc0));
    if (tid == 0 && blockIdx.y == 0) { A.vfl[2 * f] = vf; A.vfl[2 * f + 1] = vl; }
}

/* The troughs k_draft_bounds leaves undecided (dec 2): the exact draft value at
 * each (draft_point), one wave per trough, DP_CHUNK consecutive raw troughs per
 * workgroup, so a recording's undecided troughs spread over many waves.  A
 * workgroup stages the troughs its windows reach.  A trough draft_point does
 * not take sends the recording to the full draft (exact). */
template <int SPL>
__device__ __forceinline__ void draft_points_chunk(const DraftBoundArgs &A, int f, int m, int jc0, int32_t *s_tp,
                                                   double *s_tv, int16_t *s_und, int *s_nund_p) {
    int &s_nund = *s_nund_p;
    const int jc1 = min(m, jc0 + DP_CHUNK);
    const int tid = threadIdx.x;
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    if (tid == 0) s_nund = 0;
    __syncthreads();
    if (tid < 64) {                                          /* in trough order (DP_CHUNK <= 64) */
        const int j = jc0 + tid;
        const bool und = j < jc1 && A.dec[d0 + j] == 2;
        const uint64_t bm = __ballot(und);
        if (und) s_und[__popcll(bm & ((1ull << tid) - 1ull))] = (int16_t)tid;
        /* another workgroup of this recording may set exact[f] at any time: one
         * read, shared, so every thread takes the same path (the value rides in
         * the count's sign) */
        if (tid == 0)
            s_nund = __hip_atomic_load(&A.exact[f], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? -1 : __popcll(bm);
    }
    __syncthreads();
    const int nu = s_nund;
    if (nu <= 0) return;                                     /* none undecided, or the full draft anyway */
    const int64_t *raw = A.raw + d0;
    const double *rawv = A.rawv + d0;                        /* env at the raw troughs */
    const int64_t W = A.window, t0 = raw[0];
    const int vf = A.vfl[2 * f], vl = A.vfl[2 * f + 1];
    auto seg_of_g = [&](int64_t x) -> int {                 /* last trough <= x, over global memory */
        int lo = 0, hi = m;
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (raw[mid] <= x) lo = mid + 1; else hi = mid; }
        return lo - 1;
    };
    auto qpos = [&](int j) -> int64_t { const int64_t t = raw[j]; return t < vf ? vf : (t > vl ? vl : t); };
    int64_t s, e;
    win_bounds(qpos(jc0), n, W, s, e);
    const int ja = seg_of_g(s > t0 ? s : t0);
    win_bounds(qpos(jc1 - 1), n, W, s, e);
    const int jb = seg_of_g(e - 1);
    const int base = min(ja, jc0);
    const int top = min(m - 1, max(jb + 1, jc1 - 1));
    const int ns = top - base + 1;
    if (ns > DB_TRMAX) {                                     /* windows too wide to stage */
        if (tid == 0) __hip_atomic_store(&A.exact[f], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    for (int j = tid; j < ns; j += DB_T) {
        s_tp[j] = (int32_t)raw[base + j];
        s_tv[j] = rawv[base + j];                            /* env at the trough */
    }
    __syncthreads();
    auto seg_of = [&](int64_t x) -> int {                   /* last trough <= x (x >= t0), among the staged */
        int lo = base, hi = base + ns;
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (s_tp[mid - base] <= x) lo = mid + 1; else hi = mid; }
        return lo - 1;
    };
    bool fail = false;
    /* each wave a run of consecutive undecided troughs, each seeded with the
     * previous one's draft value */
    const int per = (nu + DB_T / 64 - 1) / (DB_T / 64);
    double prev = __builtin_nan(""), rho = __builtin_nan("");
    for (int u = wave_id() * per; u < min(nu, (wave_id() + 1) * per); ++u) {
        const int j = jc0 + s_und[u];
        const int64_t t = s_tp[j - base];
        const int64_t qp = t < vf ? vf : (t > vl ? vl : t);
        win_bounds(qp, n, W, s, e);
        const int64_t lo = s > t0 ? s : t0, hi = e;
        double r = 0.0;
        /* SPL 1: one segment per lane, windows of <= 64 segments (the common
         * case); wider ones stay undecided for the SPL 4 launch, so the
         * common kernel keeps the registers of one segment per lane */
        const int jl = seg_of(lo), jh = seg_of(hi - 1);
        if (SPL == 1 && jh - jl + 1 > 64) {                 /* for the [wide] launch */
            if (lane_id() == 0) atomicAdd(&A.nund[A.n_files + f], 1);
            continue;
        }
        const uint32_t seed = 0x9E3779B9u * (uint32_t)(f + 1) ^ (uint32_t)j * 0x85EBCA6Bu;
        /* only the keep decision is needed: draft_point's decision mode
         * settles most troughs with one or two counts against env / mult */
        const double et = s_tv[j - base];
        const double theta = A.mult > 0.0 ? et / A.mult : __builtin_nan("");
        int dd = -1;
        if (!draft_point<SPL>(s_tp, s_tv, base, m, n, lo, hi, jl, jh, A.q, seed, &r, prev, &rho, theta, &dd)) {
            fail = true;
            continue;
        }
        if (dd >= 0) {                                       /* decided without the value: no seed for the next */
            prev = __builtin_nan("");
            if (lane_id() == 0) A.dec[d0 + j] = (uint8_t)dd;
            continue;
        }
        prev = r;
        if (lane_id() == 0) A.dec[d0 + j] = (r == r && et <= A.mult * r) ? 1 : 0;
    }
    if (fail && lane_id() == 0) __hip_atomic_store(&A.exact[f], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (A.stats && SPL == 1 && tid == 0) atomicAdd((unsigned long long *)&A.stats[1], (unsigned long long)nu);
    if (A.stats && fail && lane_id() == 0) atomicAdd((unsigned long long *)&A.stats[2], 1ull);
    __syncthreads();                                         /* s_und / s_nund reused by the next chunk */
}

/* a few workgroups per recording, each taking chunks y, y + gridDim.y, ...;
 * recordings without undecided troughs (nund, from k_draft_bounds; the [wide]
 * launch: none left for it) cost one load */
template <int SPL>
__global__ __launch_bounds__(DB_T, SPL == 1 ? BPMX_DP_WAVES : 1) void k_draft_points(DraftBoundArgs A) {
    const int f = blockIdx.x;
    if (f >= A.n_files || !A.run[f]) return;
    if (A.nund[(SPL == 1 ? 0 : A.n_files) + f] == 0) return;
    const int m = A.nraw[f];
    __shared__ int32_t s_tp[DB_TRMAX];
    __shared__ double s_tv[DB_TRMAX];
    __shared__ int16_t s_und[DP_CHUNK];
    __shared__ int s_nund;
    for (int jc0 = (int)blockIdx.y * DP_CHUNK; jc0 < m; jc0 += (int)gridDim.y * DP_CHUNK)
        draft_points_chunk<SPL>(A, f, m, jc0, s_tp, s_tv, s_und, &s_nund);
}
template __global__ void k_draft_points<1>(DraftBoundArgs);
template __global__ void k_draft_points<DP_SPL_MAX>(DraftBoundArgs);

__global__ __launch_bounds__(256) void k_floor_final(FinalArgs A) {
    const int f = blockIdx.y;
    if (f >= A.n_files || !A.active[f]) return;
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    const int fl = A.flags[f];
    const double *qv = A.qv + (int64_t)f * Q_SLOTS;
    bool nanfb = false, from_draft = false;
    double v = 0.0;
    if (fl & BPMX_F_STATIC_FLOOR) {
        v = qv[Q_NOISE];
    } else if (fl & BPMX_F_DRAFT_FLOOR) {
        nanfb = A.allnan_draft[f] != 0;
        from_draft = !nanfb;
        v = qv[Q_FALLBACK];
    } else {
        nanfb = A.allnan_final[f] != 0;
        if (!nanfb) return;   /* floor already written by the second rolling pass */
        v = qv[Q_FALLBACK];
    }
    /* a few workgroups per recording striding over it */
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        A.floor[d0 + i] = from_draft ? A.draft[d0 + i] : v;
    if (blockIdx.x == 0 && threadIdx.x == 0 && nanfb) A.flags[f] = fl | BPMX_F_NAN_FLOOR;
}

}  // namespace bpmx
