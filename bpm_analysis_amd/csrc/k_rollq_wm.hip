/*
 * k_rollq_wm.hip — centred rolling quantile by a per-recording wavelet matrix
 * (bpm_analysis.py:1084-1086 / :1104-1106:
 *  .rolling(W, min_periods=3, center=True).quantile(q).bfill().ffill()).
 *
 * One 1024-thread workgroup per recording, everything in LDS:
 *   1. ranks: the finite suffix dense[t0:n) is ordered by (value, position)
 *      with an LSD radix sort on order-preserving 64-bit keys, 8-bit digits,
 *      digits constant over the recording skipped.  What moves is only the
 *      16-bit position (ping-pong in LDS); the current 32-bit key half sits
 *      in LDS indexed by position (low halves for digits 0-3, then high
 *      halves).  Slots are wave-contiguous, so a stable rank is: per-wave
 *      digit counter (LDS atomic, issued in slot order) + peers below in the
 *      same round (ballot match) + one (digit, wave) block scan.
 *   2. wavelet matrix over the rank sequence (ceil(log2 m) levels): per level
 *      a bit vector with a rank directory, {word, ones-before} in 16 B.
 *   3. every output independently: its window's k-th and (k+1)-th smallest by
 *      two interleaved top-down descents (O(log m) LDS reads each), pandas'
 *      linear interpolation, nobs / min_periods from the window bounds.  NaN
 *      outputs are a prefix and a suffix (nobs is unimodal), filled from the
 *      first and last valid output.
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

__global__ __launch_bounds__(WM_T) void k_rollq_wm(RollqArgs A, double *sorted_scratch) {
    constexpr int NWV = WM_T / 64;
    constexpr int MAXIT = WM_MMAX / WM_T;
    const int f = blockIdx.x;
    if (f >= A.n_files || !A.run[f]) return;
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    if (n > WM_MMAX || n <= 0) return;                       /* k_rolling_quantile handles it */
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int s_first, s_last, s_Z[16], s_wt[NWV];
    __shared__ unsigned long long s_or[NWV], s_and[NWV];

    const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
    const double *dense = A.dense + d0;
    double *out = A.out + d0;
    double *sv = sorted_scratch + d0;                        /* sorted values, rank order */
    const int64_t t0 = A.troughs[d0];
    const int m = (int)(n - t0);                             /* finite samples dense[t0:n) */
    const int IT = (m + WM_T - 1) / WM_T;                    /* rounds per wave */
    const int S = 64 * IT;                                   /* slots per wave */
    if (tid == 0) { s_first = INT_MAX; s_last = -1; }
    STAMP_DECL

    /* dense = np.interp of the troughs (k_interp), evaluated here from env at
     * the troughs staged in LDS when there are <= WM_TRMAX of them */
    const int ntr = A.env ? A.ntr[f] : 0;
    const bool fused = A.env && ntr <= WM_TRMAX;
    int32_t *s_tp, *s_bj;
    double *s_tv;
    {
        const int64_t n8 = (n + 7) & ~7LL;
        const int64_t Ln = n > 1 ? 64 - __builtin_clzll((unsigned long long)(n - 1)) : 1;
        const int64_t sort_b = 8 * n8 + (int64_t)NWV * 128 * 4;
        const int64_t wm_b = 4 * n8 + Ln * (2 * ((n + 63) / 64) + 1) * 8;
        s_tv = (double *)(smem + (sort_b > wm_b ? sort_b : wm_b));
        s_tp = (int32_t *)(s_tv + WM_TRMAX);
        s_bj = s_tp + WM_TRMAX;                              /* [n/64 + 1]: last trough <= block start */
    }
    if (fused) {
        const int64_t *tr = A.troughs + d0;
        for (int j = tid; j < ntr; j += WM_T) {
            s_tp[j] = (int32_t)tr[j];
            s_tv[j] = A.env[d0 + tr[j]];
        }
        __syncthreads();
        for (int64_t b = tid; b <= (n >> 6); b += WM_T) {
            int lo = 0, hi = ntr;
            while (lo < hi) { const int mid = (lo + hi) >> 1; if (s_tp[mid] <= (b << 6)) lo = mid + 1; else hi = mid; }
            s_bj[b] = lo - 1;
        }
        __syncthreads();
    }
    /* interp_at's arithmetic, with the bracketing trough found from the block table */
    auto dval = [&](int64_t x) -> double {
        if (!fused) return dense[x];
        if (ntr == 0 || x < s_tp[0]) return __builtin_nan("");
        int j = s_bj[x >> 6];
        if (j < 0) j = 0;
        while (j + 1 < ntr && s_tp[j + 1] <= x) ++j;
        if (j == ntr - 1 || s_tp[j] == x) return s_tv[j];
        const double y0 = s_tv[j], y1 = s_tv[j + 1];
        const double slope = (y1 - y0) / ((double)s_tp[j + 1] - (double)s_tp[j]);
        double r = slope * ((double)x - (double)s_tp[j]) + y0;
        if (r != r) {
            r = slope * ((double)x - (double)s_tp[j + 1]) + y1;
            if (r != r && y0 == y1) r = y0;
        }
        return r;
    };

    /* LDS, sort phase: posA[m8] | posB[m8] | kh[m8] | cnt[NWV][128] (two 16-bit counters per word).
     * Slots >= m are padding: they sort last, so they are neither stored nor counted. */
    const int m8 = (m + 7) & ~7;
    uint16_t *posA = (uint16_t *)smem;
    uint16_t *posB = posA + m8;
    uint32_t *kh = (uint32_t *)(posB + m8);
    uint32_t *cnt = kh + m8;

    /* ---------------- 1. ranks by LSD radix sort ---------------- */
    uint64_t kor = 0, kand = ~0ull;
    for (int p = tid; p < m; p += WM_T) {
        posA[p] = (uint16_t)p;                               /* slot order == position order */
        const uint64_t k = wm_key(dval(t0 + p));
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
        if (d == 4 && (vary >> 32)) {                        /* high halves, indexed by position */
            for (int p = tid; p < m; p += WM_T) kh[p] = (uint32_t)(wm_key(dval(t0 + p)) >> 32);
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
    /* posA[r] = position of rank r.  Build: seqA = the free pos buffer,
     * seqB = posA once consumed; levels over the dead kh / cnt. */
    const int L = m > 1 ? 32 - __clz(m - 1) : 1;              /* levels: ranks < 2^L */
    const int NW = (m + 63) >> 6;                             /* 64-bit words per level */
    const int NR = 2 * NW + 1;                                /* 32-bit records per level (+ sentinel) */
    uint16_t *seqA = posB, *seqB = posA;
    WmRec *lv = (WmRec *)kh;                                  /* [L][NR] */
    for (int r = tid; r < m; r += WM_T) {
        const int p = posA[r];
        sv[r] = dval(t0 + p);
        seqA[p] = (uint16_t)r;
    }
    __syncthreads();
    STAMP(4);

    /* ---------------- 2. wavelet matrix ---------------- */
    const int cw = (NW + NWV - 1) / NWV;                     /* words per wave (<= 64) */
    const int wb = wid * cw, we = min(NW, wb + cw);
    for (int l = L - 1; l >= 0; --l) {
        WmRec *row = lv + l * NR;
        /* ones among this wave's words (ballots are wave-uniform: scalar sums) */
        uint32_t wones = 0;
        for (int w = wb; w < we; ++w) {
            const int p = w * 64 + lane;
            wones += (uint32_t)__popcll(__ballot(p < m && ((seqA[p] >> l) & 1)));
        }
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
        for (int w = wb; w < we; ++w) {
            const int p = w * 64 + lane;
            const uint32_t v = p < m ? seqA[p] : 0u;
            const bool bit = p < m && ((v >> l) & 1);
            const uint64_t word = __ballot(bit);
            if (lane == 0) {
                row[2 * w] = WmRec{(uint32_t)word, run};
                row[2 * w + 1] = WmRec{(uint32_t)(word >> 32), run + (uint32_t)__popc((uint32_t)word)};
            }
            const int o1 = (int)run + __popcll(word & lanemask_lt());
            if (p < m) seqB[bit ? Z + o1 : p - o1] = (uint16_t)v;
            run += (uint32_t)__popcll(word);
        }
        __syncthreads();
        uint16_t *t = seqA; seqA = seqB; seqB = t;
    }
    __threadfence_block();
    STAMP(5);

    /* ---------------- 3. outputs ---------------- */
    const int64_t W = A.window, minp = A.min_periods;
    const double q = A.q;
    auto rk = [&](const WmRec *row, int i) {
        const WmRec r = row[i >> 5];
        return (int)r.ones + __popc(r.word & ((1u << (i & 31)) - 1u));
    };
    /* k-th and (k+1)-th smallest of positions [lo, hi): two interleaved descents */
    auto kth2 = [&](int lo, int hi, int k, int &ra, int &rb) {
        int la = lo, ha = hi, ka = k, lb = lo, hb = hi, kb = k + 1;
        ra = 0;
        rb = 0;
        for (int l = L - 1; l >= 0; --l) {
            const WmRec *row = lv + l * NR;
            const int oa0 = rk(row, la), oa1 = rk(row, ha), ob0 = rk(row, lb), ob1 = rk(row, hb);
            const int Z = s_Z[l];
            const int za = (ha - oa1) - (la - oa0), zb = (hb - ob1) - (lb - ob0);
            if (ka < za) { la -= oa0; ha -= oa1; }
            else { ka -= za; la = Z + oa0; ha = Z + oa1; ra |= 1 << l; }
            if (kb < zb) { lb -= ob0; hb -= ob1; }
            else { kb -= zb; lb = Z + ob0; hb = Z + ob1; rb |= 1 << l; }
        }
    };
    int vfirst = INT_MAX, vlast = -1;
    for (int64_t i = tid; i < n; i += WM_T) {
        int64_t s, e;
        win_bounds(i, n, W, s, e);
        const int64_t lo = s > t0 ? s : t0;
        const int64_t nobs = e > lo ? e - lo : 0;
        double res = __builtin_nan("");
        if (nobs >= minp && nobs > 0) {
            const int plo = (int)(lo - t0), phi = (int)(e - t0);
            double idxf = 0;
            int64_t k = 0;
            if (nobs > 1) {
                idxf = q * (double)(nobs - 1);
                k = (int64_t)idxf;
            }
            const bool interp = !(nobs == 1 || (double)k == idxf);
            int ra, rb;
            kth2(plo, phi, (int)k, ra, rb);   /* rb is meaningless when !interp (k+1 may equal nobs) */
            const double va = sv[ra];
            if (!interp) {
                res = va;
            } else {
                const double vb = sv[rb];
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

}  // namespace bpmx
