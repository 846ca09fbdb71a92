/*
 * k_detect.hip — quantiles, block statistics and find_peaks.
 *
 *   k_quantile     np.quantile(env, q) 'linear' (bpm_analysis.py:1067, :225,
 *                  :1075, :1114): exact order statistics by 8-bit radix select
 *                  on order-preserving f64 keys, then numpy's _lerp.
 *   k_block_stats  max/min of env per 64-sample block (prominence accelerator).
 *   k_find_peaks   scipy.signal.find_peaks(sign*env, height, distance,
 *                  prominence) (scipy/signal/_peak_finding.py:729-1010):
 *                  one workgroup per recording:
 *                  (1) _local_maxima_1d: every rising edge checks its plateau,
 *                      ordered compaction by block scans;
 *                  (2) height filter hmin <= x[peak];
 *                  (3) _select_by_peak_distance: the greedy keep-highest pass
 *                      is the lexicographically-first independent set in
 *                      priority order, computed by rounds of local decisions
 *                      (a candidate is kept once every higher-priority
 *                      neighbour within `distance` is removed, removed once one
 *                      is kept) — same set as the sequential loop;
 *                  (4) _peak_prominences, wlen=-1: one wave per candidate scans
 *                      64 samples per step, and 64 blocks per step through the
 *                      block max/min tables once its own block is exhausted;
 *                  (5) prominence >= threshold, ordered compaction.
 */
#include "bpmx_common.h"
#include "bpmx_kernels.h"

namespace bpmx {

/* ------------------------------------------------------------------------ */
__global__ __launch_bounds__(256) void k_quantile(QuantArgs A) {
    const int f = blockIdx.x, l = blockIdx.y;
    if (f >= A.n_files || l >= A.n_levels || !A.active[f]) return;
    const int64_t n = A.doff[f + 1] - A.doff[f];
    const double *x = A.env + A.doff[f];
    const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
    __shared__ unsigned int hist[256];
    __shared__ long long s_r;
    __shared__ int s_digit;
    __shared__ unsigned long long s_min[4];
    __shared__ long long s_cnt[4];

    const double q = A.q[l];
    const double vi = (double)(n - 1) * q;
    const bool top = vi >= (double)(n - 1);
    const long long lo = top ? (long long)(n - 1) : (long long)floor(vi);
    uint64_t prefix = 0, mask = 0;
    long long r = lo;
    for (int shift = 56; shift >= 0; shift -= 8) {
        hist[tid] = 0;
        __syncthreads();
        for (int64_t i = tid; i < n; i += 256) {
            uint64_t k = f64_key(x[i]);
            if ((k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 255], 1u);
        }
        __syncthreads();
        if (wid == 0) {
            unsigned int c0 = hist[lane * 4], c1 = hist[lane * 4 + 1], c2 = hist[lane * 4 + 2], c3 = hist[lane * 4 + 3];
            long long s = (long long)c0 + c1 + c2 + c3, incl = s;
            for (int o = 1; o < 64; o <<= 1) {
                long long t = __shfl_up(incl, o);
                if (lane >= o) incl += t;
            }
            long long excl = incl - s;
            if (excl <= r && r < incl) {
                long long rr = r - excl;
                unsigned int cs[4] = {c0, c1, c2, c3};
                int d = 0;
                while (rr >= (long long)cs[d]) { rr -= cs[d]; ++d; }
                s_digit = lane * 4 + d;
                s_r = rr;
            }
        }
        __syncthreads();
        prefix |= (uint64_t)s_digit << shift;
        mask |= 0xFFull << shift;
        r = s_r;
        __syncthreads();
    }
    const double va = key_f64(prefix);
    double res = va;
    if (!top) {
        unsigned long long mn = ~0ull;
        long long cnt = 0;
        for (int64_t i = tid; i < n; i += 256) {
            uint64_t k = f64_key(x[i]);
            if (k <= prefix) cnt++;
            else if (k < mn) mn = k;
        }
        for (int o = 32; o > 0; o >>= 1) {
            unsigned long long om = __shfl_xor(mn, o);
            mn = om < mn ? om : mn;
            cnt += __shfl_xor(cnt, o);
        }
        if (lane == 0) { s_min[wid] = mn; s_cnt[wid] = cnt; }
        __syncthreads();
        unsigned long long m = s_min[0];
        long long c = 0;
        for (int w = 0; w < 4; ++w) { m = s_min[w] < m ? s_min[w] : m; c += s_cnt[w]; }
        const double vb = (c > lo + 1) ? va : key_f64(m);
        res = np_lerp(va, vb, vi - (double)lo);
    }
    if (tid < Q_SLOTS && ((A.slot[l] >> tid) & 1)) A.qv[(int64_t)f * Q_SLOTS + tid] = res;
}

/* ------------------------------------------------------------------------ */
__global__ __launch_bounds__(256) void k_block_stats(BlockStatArgs A) {
    const int f = blockIdx.x;
    if (f >= A.n_files || !A.active[f]) return;
    const int64_t n = A.doff[f + 1] - A.doff[f];
    const int64_t nb = (n + 63) >> 6;
    const double *x = A.env + A.doff[f];
    double *bmx = A.bmax + A.boff[f], *bmn = A.bmin + A.boff[f];
    const int lane = lane_id();
    const double INF = __builtin_inf();
    for (int64_t b = wave_id(); b < nb; b += 4) {
        int64_t i = (b << 6) + lane;
        double v = i < n ? x[i] : __builtin_nan("");
        double mx = wave_max(i < n ? v : -INF);
        double mn = wave_min(i < n ? v : INF);
        if (lane == 0) { bmx[b] = mx; bmn[b] = mn; }
    }
}

/* ------------------------------------------------------------------------ */
/* prominence of peak p (value xp = sg*e[p]) — _peak_prominences, wlen = -1:
 * min of x over (left_higher, p] and [p, right_higher), prom = xp - max(...) */
__device__ double prominence_wave(const double *e, double sg, int64_t n, const double *bmx, const double *bmn,
                                  int64_t p, double xp) {
    const int lane = lane_id();
    const int64_t nb = (n + 63) >> 6;
    const double INF = __builtin_inf();
    const int64_t blk = p >> 6;
    double lmin, rmin;
    {   /* left */
        const int64_t pos = (blk << 6) + lane;
        const bool valid = pos <= p;
        const double v = valid ? sg * e[pos] : -INF;
        const unsigned long long m = __ballot(valid && v > xp);
        if (m) {
            const int L = 63 - __clzll(m);
            lmin = wave_min((valid && lane > L) ? v : INF);
        } else {
            lmin = wave_min(valid ? v : INF);
            for (int64_t bs = blk - 1; bs >= 0; bs -= 64) {
                const int64_t b = bs - lane;
                const bool vb = b >= 0;
                const double bm = vb ? (sg > 0 ? bmx[b] : -bmn[b]) : -INF;
                const double bn = vb ? (sg > 0 ? bmn[b] : -bmx[b]) : INF;
                const unsigned long long mb = __ballot(vb && bm > xp);
                if (mb) {
                    const int Lb = __ffsll((long long)mb) - 1;
                    lmin = fmin(lmin, wave_min(lane < Lb ? bn : INF));
                    const int64_t q = ((bs - Lb) << 6) + lane;      /* a full block left of p */
                    const double v2 = sg * e[q];
                    const unsigned long long m2 = __ballot(v2 > xp);
                    const int L2 = 63 - __clzll(m2);
                    lmin = fmin(lmin, wave_min(lane > L2 ? v2 : INF));
                    break;
                }
                lmin = fmin(lmin, wave_min(bn));
            }
        }
    }
    {   /* right */
        const int64_t pos = (blk << 6) + lane;
        const bool valid = pos >= p && pos < n;
        const double v = valid ? sg * e[pos] : -INF;
        const unsigned long long m = __ballot(valid && v > xp);
        if (m) {
            const int R = __ffsll((long long)m) - 1;
            rmin = wave_min((valid && lane < R) ? v : INF);
        } else {
            rmin = wave_min(valid ? v : INF);
            for (int64_t bs = blk + 1; bs < nb; bs += 64) {
                const int64_t b = bs + lane;
                const bool vb = b < nb;
                const double bm = vb ? (sg > 0 ? bmx[b] : -bmn[b]) : -INF;
                const double bn = vb ? (sg > 0 ? bmn[b] : -bmx[b]) : INF;
                const unsigned long long mb = __ballot(vb && bm > xp);
                if (mb) {
                    const int Rb = __ffsll((long long)mb) - 1;
                    rmin = fmin(rmin, wave_min(lane < Rb ? bn : INF));
                    const int64_t q = ((bs + Rb) << 6) + lane;
                    const bool vq = q < n;
                    const double v2 = vq ? sg * e[q] : -INF;
                    const unsigned long long m2 = __ballot(vq && v2 > xp);
                    const int R2 = __ffsll((long long)m2) - 1;
                    rmin = fmin(rmin, wave_min((vq && lane < R2) ? v2 : INF));
                    break;
                }
                rmin = fmin(rmin, wave_min(bn));
            }
        }
    }
    return xp - fmax(lmin, rmin);
}

enum { ST_UNDECIDED = 0, ST_KEPT = 1, ST_REMOVED = 2, ST_FINAL = 3 };

__device__ __forceinline__ uint8_t ld_state(const uint8_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void st_state(uint8_t *p, uint8_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

constexpr int FP_T = 1024;

__global__ __launch_bounds__(FP_T) void k_find_peaks(PeakArgs A) {
    const int f = blockIdx.x;
    if (f >= A.n_files || !A.active[f]) return;
    const int64_t d0 = A.doff[f];
    const int64_t n = A.doff[f + 1] - d0;
    const double *e = A.env + d0;
    const double *h = A.height ? A.height + d0 : nullptr;
    const double sg = A.sign;
    int32_t *cand = A.cand + d0;
    uint8_t *st = A.state + d0;
    const int tid = threadIdx.x;
    __shared__ int sh[FP_T / 64 + 1];
    __shared__ int s_flag;

    /* (1)+(2) local maxima with plateau midpoints, height filter */
    int m = 0;
    for (int64_t c0 = 1; c0 < n - 1; c0 += FP_T) {
        const int64_t i = c0 + tid;
        bool is = false;
        int64_t p = 0;
        if (i < n - 1) {
            const double xi = sg * e[i];
            if (sg * e[i - 1] < xi) {
                int64_t ia = i + 1;
                while (ia < n - 1 && sg * e[ia] == xi) ia++;
                if (sg * e[ia] < xi) {
                    p = (i + ia - 1) >> 1;
                    is = true;
                    if (h && !(h[p] <= sg * e[p])) is = false;
                }
            }
        }
        int tot;
        const int off = block_scan_flag<FP_T>(is, sh, &tot);
        if (is) cand[m + off] = (int32_t)p;
        m += tot;
    }
    __syncthreads();

    /* (3) distance: rounds of local decisions */
    const int64_t dist = A.distance;
    for (int j = tid; j < m; j += FP_T) st_state(&st[j], dist > 1 ? ST_UNDECIDED : ST_KEPT);
    __syncthreads();
    if (dist > 1) {
        /* every round decides at least the highest-priority undecided candidate,
         * so m + 1 rounds always suffice; the cap only bounds a corrupted input */
        for (int round = 0; round <= m; ++round) {
            if (tid == 0) s_flag = 0;
            __syncthreads();
            bool pending = false;
            for (int j = tid; j < m; j += FP_T) {
                if (ld_state(&st[j]) != ST_UNDECIDED) continue;
                const int64_t pj = cand[j];
                const double vj = sg * e[pj];
                bool killed = false, blocked = false;
                for (int k = j - 1; k >= 0 && pj - cand[k] < dist; --k) {
                    if (sg * e[cand[k]] > vj) {          /* earlier index wins only when strictly higher */
                        const uint8_t s = ld_state(&st[k]);
                        if (s == ST_KEPT) { killed = true; break; }
                        if (s == ST_UNDECIDED) blocked = true;
                    }
                }
                if (!killed) {
                    for (int k = j + 1; k < m && cand[k] - pj < dist; ++k) {
                        if (sg * e[cand[k]] >= vj) {     /* later index wins ties (stable argsort order) */
                            const uint8_t s = ld_state(&st[k]);
                            if (s == ST_KEPT) { killed = true; break; }
                            if (s == ST_UNDECIDED) blocked = true;
                        }
                    }
                }
                if (killed) st_state(&st[j], ST_REMOVED);
                else if (!blocked) st_state(&st[j], ST_KEPT);
                else pending = true;
            }
            if (pending) s_flag = 1;
            __syncthreads();
            const int again = s_flag;
            __syncthreads();
            if (!again) break;
        }
    }

    /* (4) prominences of the kept candidates, one wave each */
    const double thr = A.qv[(int64_t)f * Q_SLOTS + A.qslot];
    const double *bmx = A.bmax + A.boff[f], *bmn = A.bmin + A.boff[f];
    for (int j = wave_id(); j < m; j += FP_T / 64) {
        if (ld_state(&st[j]) != ST_KEPT) continue;
        const int64_t p = cand[j];
        const double prom = prominence_wave(e, sg, n, bmx, bmn, p, sg * e[p]);
        if (lane_id() == 0) st_state(&st[j], thr <= prom ? ST_FINAL : ST_REMOVED);
    }
    __syncthreads();

    /* (5) ordered compaction */
    int64_t *out = A.out + d0;
    int w = 0;
    for (int c0 = 0; c0 < m; c0 += FP_T) {
        const int j = c0 + tid;
        const bool keep = j < m && ld_state(&st[j]) == ST_FINAL;
        int tot;
        const int off = block_scan_flag<FP_T>(keep, sh, &tot);
        if (keep) out[w + off] = cand[j];
        w += tot;
    }
    if (tid == 0) {
        A.nout[f] = w;
        if (A.run_out) A.run_out[f] = w >= A.run_min ? 1 : 0;
    }
}

}  // namespace bpmx
