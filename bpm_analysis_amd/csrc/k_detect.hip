/*
 * k_detect.hip — quantiles, block statistics and find_peaks.
 *
 *   k_quantile_reg / k_ql_*  np.quantile(env, q) 'linear' (bpm_analysis.py:1067,
 *                  :225, :1075, :1114): exact order statistics by radix select
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
#include "bpmx_qsel.h"
#include "bpmx_fpscan.h"
#include "bpmx_stamps.h"

namespace bpmx {

/* ------------------------------------------------------------------------ */
/* ------------------------------------------------------------------------ */
/* the same quantiles for long recordings over many workgroups: k_ql_init sets
 * each (recording, level)'s rank; per 11-bit digit (most significant first)
 * k_ql_hist counts the keys that match the prefix found so far, every chunk
 * of every recording in its own workgroup (LDS bins per level, merged into
 * global bins), and k_ql_select picks the digit holding the rank; after six
 * passes the prefix is the order statistic's key.  The next order statistic
 * is the same key when the final bin holds another one, else the smallest key
 * above it (k_ql_next), then numpy's _lerp (k_ql_final). */
namespace {
__device__ __forceinline__ bool ql_sel(const QuantArgs &Q, int f) {
    if (f >= Q.n_files || !Q.active[f] || (Q.skip && Q.skip[f])) return false;
    return Q.doff[f + 1] - Q.doff[f] > Q.skip_le;
}
__device__ __forceinline__ int ql_shift(int pass) {            /* 53, 42, 31, 20, 9, 0 (last digit 9 bits) */
    return pass < QL_PASSES - 1 ? 64 - QL_BITS * (pass + 1) : 0;
}
}  // namespace

__global__ __launch_bounds__(64) void k_ql_init(QlArgs A) {
    const int f = blockIdx.x, l = threadIdx.x;
    if (!ql_sel(A.Q, f) || l >= A.Q.n_levels) return;
    const int64_t n = A.Q.doff[f + 1] - A.Q.doff[f];
    const double vi = (double)(n - 1) * A.Q.q[l];
    QlState s;
    s.top = vi >= (double)(n - 1);
    s.lo = s.top ? (long long)(n - 1) : (long long)floor(vi);
    s.r = s.lo;
    s.prefix = 0; s.mask = 0; s.next = ~0ull; s.eq = 0;
    A.st[(int64_t)f * Q_SLOTS + l] = s;
}

__global__ __launch_bounds__(256) void k_ql_hist(QlArgs A) {
    const int f = blockIdx.y;
    if (!ql_sel(A.Q, f)) return;
    const int64_t d0 = A.Q.doff[f], n = A.Q.doff[f + 1] - d0;
    const int64_t c0 = (int64_t)blockIdx.x * QL_CHUNK;
    if (c0 >= n) return;
    const int64_t c1 = min<int64_t>(n, c0 + QL_CHUNK);
    const int L = A.Q.n_levels, sh = ql_shift(A.pass);
    const unsigned int dmask = A.pass < QL_PASSES - 1 ? (unsigned)(QL_BINS - 1) : 511u;
    __shared__ unsigned int hist[Q_SLOTS][QL_BINS];
    __shared__ unsigned long long s_pre[Q_SLOTS], s_msk[Q_SLOTS];
    for (int i = threadIdx.x; i < L * QL_BINS; i += 256) hist[i / QL_BINS][i % QL_BINS] = 0u;
    if (threadIdx.x < L) {
        const QlState st = A.st[(int64_t)f * Q_SLOTS + threadIdx.x];
        s_pre[threadIdx.x] = st.prefix;
        s_msk[threadIdx.x] = st.mask;
    }
    __syncthreads();
    const double *x = A.Q.env + d0;
    for (int64_t i = c0 + threadIdx.x; i < c1; i += 256) {
        const uint64_t k = f64_key(x[i]);
        const unsigned int dg = (unsigned int)(k >> sh) & dmask;
        for (int l = 0; l < L; ++l)
            if ((k & s_msk[l]) == s_pre[l]) atomicAdd(&hist[l][dg], 1u);
    }
    __syncthreads();
    unsigned int *g = A.hist + (((int64_t)A.pass * A.Q.n_files + f) * Q_SLOTS) * QL_BINS;
    for (int i = threadIdx.x; i < L * QL_BINS; i += 256) {
        const unsigned int c = hist[i / QL_BINS][i % QL_BINS];
        if (c) atomicAdd(&g[(i / QL_BINS) * QL_BINS + (i % QL_BINS)], c);
    }
}

/* one workgroup per (recording, level): the digit whose cumulative count passes r */
__global__ __launch_bounds__(256) void k_ql_select(QlArgs A) {
    const int f = blockIdx.x, l = blockIdx.y;
    if (!ql_sel(A.Q, f) || l >= A.Q.n_levels) return;
    const unsigned int *g = A.hist + (((int64_t)A.pass * A.Q.n_files + f) * Q_SLOTS + l) * QL_BINS;
    QlState *ps = A.st + (int64_t)f * Q_SLOTS + l;
    const long long r = ps->r;
    __shared__ int sh[256 / 64 + 1];
    constexpr int PER = QL_BINS / 256;                          /* 8 consecutive bins per thread */
    unsigned int c[PER];
    int sum = 0;
#pragma unroll
    for (int u = 0; u < PER; ++u) { c[u] = g[threadIdx.x * PER + u]; sum += (int)c[u]; }
    int tot;
    const long long before = block_scan_int<256>(sum, sh, &tot);
    if (before <= r && r < before + sum) {                       /* exactly one thread */
        long long rr = r - before;
        int d = 0;
        while (rr >= (long long)c[d]) { rr -= c[d]; ++d; }
        const int digit = threadIdx.x * PER + d, s = ql_shift(A.pass);
        const unsigned long long dm = A.pass < QL_PASSES - 1 ? (unsigned long long)(QL_BINS - 1) : 511ull;
        ps->prefix |= (unsigned long long)digit << s;
        ps->mask |= dm << s;
        ps->r = rr;
        if (A.pass == QL_PASSES - 1) ps->eq = (long long)c[d] > rr + 1 ? 1 : 0;   /* another key equals it */
    }
}

__global__ __launch_bounds__(256) void k_ql_next(QlArgs A) {
    const int f = blockIdx.y;
    if (!ql_sel(A.Q, f)) return;
    const int64_t d0 = A.Q.doff[f], n = A.Q.doff[f + 1] - d0;
    const int64_t c0 = (int64_t)blockIdx.x * QL_CHUNK;
    if (c0 >= n) return;
    const int64_t c1 = min<int64_t>(n, c0 + QL_CHUNK);
    const int L = A.Q.n_levels;
    __shared__ unsigned long long s_pre[Q_SLOTS];
    __shared__ int s_need[Q_SLOTS];
    if (threadIdx.x < L) {
        const QlState st = A.st[(int64_t)f * Q_SLOTS + threadIdx.x];
        s_pre[threadIdx.x] = st.prefix;
        s_need[threadIdx.x] = !st.top && !st.eq;
    }
    __syncthreads();
    unsigned long long mn[Q_SLOTS] = {~0ull, ~0ull, ~0ull, ~0ull};
    const double *x = A.Q.env + d0;
    for (int64_t i = c0 + threadIdx.x; i < c1; i += 256) {
        const uint64_t k = f64_key(x[i]);
#pragma unroll
        for (int l = 0; l < Q_SLOTS; ++l)
            if (l < L && k > s_pre[l] && k < mn[l]) mn[l] = k;
    }
#pragma unroll
    for (int l = 0; l < Q_SLOTS; ++l) {
        if (l >= L || !s_need[l]) continue;
        unsigned long long m = mn[l];
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long om = __shfl_xor(m, o);
            m = om < m ? om : m;
        }
        if ((threadIdx.x & 63) == 0 && m != ~0ull) atomicMin(&A.st[(int64_t)f * Q_SLOTS + l].next, m);
    }
}

__global__ __launch_bounds__(64) void k_ql_final(QlArgs A) {
    const int f = blockIdx.x, l = threadIdx.x;
    if (!ql_sel(A.Q, f) || l >= A.Q.n_levels) return;
    const int64_t n = A.Q.doff[f + 1] - A.Q.doff[f];
    const QlState st = A.st[(int64_t)f * Q_SLOTS + l];
    const double va = key_f64(st.prefix);
    double res = va;
    if (!st.top) {
        const double vb = st.eq ? va : key_f64(st.next);
        res = np_lerp(va, vb, (double)(n - 1) * A.Q.q[l] - (double)st.lo);
    }
    for (int s = 0; s < Q_SLOTS; ++s)
        if ((A.Q.slot[l] >> s) & 1) A.Q.qv[(int64_t)f * Q_SLOTS + s] = res;
}

/* ------------------------------------------------------------------------ */
/* Long recordings' quantiles in two passes over env (r06; k_ql_* took six
 * digit passes, a "next" pass and fifteen launches).  Bins are the
 * order-preserving key's offset from the recording's least finite value's key,
 * shifted so the recording's range spans at most QV_BINS bins, clamped at both
 * ends: monotone in the key for every input (NaN and infinite keys clamp to an
 * end), so the r-th smallest key lies in the bin where the cumulative count
 * passes r, at rank r - (count below) inside it.  The bins adapt to the
 * recording, so the target bin holds few keys on real envelopes (a skewed one
 * only makes the last step longer). */
namespace {
__device__ __forceinline__ int qv_bin(uint64_t k, const QvRange &g) {
    if (k <= g.kmin) return 0;
    const uint64_t d = (k - g.kmin) >> g.shift;
    return d >= (uint64_t)QV_BINS ? QV_BINS - 1 : (int)d;
}
}  // namespace

/* per recording: key range from the block tables, and each level's rank */
__global__ __launch_bounds__(64) void k_qv_range(QvArgs A) {
    const int f = blockIdx.x, lane = threadIdx.x;
    if (!ql_sel(A.Q, f)) return;
    const int64_t b0 = A.boff[f], nb = A.boff[f + 1] - b0;
    double mn = __builtin_inf(), mx = -__builtin_inf();
    for (int64_t b = lane; b < nb; b += 64) {
        mn = fmin(mn, A.bmin[b0 + b]);
        mx = fmax(mx, A.bmax[b0 + b]);
    }
    mn = wave_min(mn);
    mx = wave_max(mx);
    if (lane == 0) {
        QvRange g;
        g.pad = 0;
        if (!(mn <= mx)) {                                    /* no finite value: bins by the key's top bits */
            g.kmin = 0;
            g.shift = 64 - QV_BITS;
        } else {
            g.kmin = f64_key(mn);
            const uint64_t span = f64_key(mx) - g.kmin;
            const int bits = span ? 64 - __clzll((long long)span) : 0;
            g.shift = bits > QV_BITS ? bits - QV_BITS : 0;
        }
        A.rg[f] = g;
    }
    const int64_t n = A.Q.doff[f + 1] - A.Q.doff[f];
    if (lane < A.Q.n_levels) {
        const double vi = (double)(n - 1) * A.Q.q[lane];
        QvState s;
        s.top = vi >= (double)(n - 1);
        s.lo = s.top ? (long long)(n - 1) : (long long)floor(vi);
        s.r = 0; s.next = ~0ull; s.bin = 0; s.cnt = 0; s.cbin = 0;
        A.st[(int64_t)f * Q_SLOTS + lane] = s;
    }
}

/* one histogram of the bins per recording (every level shares it) */
__global__ __launch_bounds__(256) void k_qv_hist(QvArgs A) {
    const int f = blockIdx.y;
    if (!ql_sel(A.Q, f)) return;
    const int64_t d0 = A.Q.doff[f], n = A.Q.doff[f + 1] - d0;
    const int64_t c0 = (int64_t)blockIdx.x * QV_CHUNK;
    if (c0 >= n) return;
    const int64_t c1 = min<int64_t>(n, c0 + QV_CHUNK);
    __shared__ unsigned int hist[QV_BINS];
    for (int i = threadIdx.x; i < QV_BINS; i += 256) hist[i] = 0u;
    const QvRange g = A.rg[f];
    __syncthreads();
    const double *x = A.Q.env + d0;
    /* a wave's 64 consecutive samples fall in runs of equal bins (the
     * envelope is smooth): one LDS atomic per run, with the run's length */
    const int lane = lane_id();
    for (int64_t i0 = c0 + (threadIdx.x & ~63); i0 < c1; i0 += 256) {   /* uniform per wave */
        const int64_t i = i0 + lane;
        const int nv = (int)min<int64_t>(64, c1 - i0);
        const int b = i < c1 ? qv_bin(f64_key(x[i]), g) : -1;
        const int bprev = __shfl_up(b, 1);
        const bool start = b >= 0 && (lane == 0 || bprev != b);
        const uint64_t sm = __ballot(start);
        const uint64_t after = sm & ~((2ull << lane) - 1ull);
        const int nxt = after ? __ffsll((long long)after) - 1 : nv;
        if (start) atomicAdd(&hist[b], (unsigned int)(nxt - lane));
    }
    __syncthreads();
    unsigned int *gh = A.hist + (int64_t)f * QV_BINS;
    for (int i = threadIdx.x; i < QV_BINS; i += 256) {
        const unsigned int c = hist[i];
        if (c) atomicAdd(&gh[i], c);
    }
}

/* per (recording, level): the bin where the cumulative count passes the rank */
__global__ __launch_bounds__(256) void k_qv_select(QvArgs A) {
    const int f = blockIdx.x, l = blockIdx.y;
    if (!ql_sel(A.Q, f) || l >= A.Q.n_levels) return;
    const unsigned int *gh = A.hist + (int64_t)f * QV_BINS;
    QvState *ps = A.st + (int64_t)f * Q_SLOTS + l;
    const long long r = ps->lo;
    __shared__ int sh[256 / 64 + 1];
    constexpr int PER = QV_BINS / 256;                          /* consecutive bins per thread */
    unsigned int c[PER];
    int sum = 0;
#pragma unroll
    for (int u = 0; u < PER; ++u) { c[u] = gh[threadIdx.x * PER + u]; sum += (int)c[u]; }
    int tot;
    const long long before = block_scan_int<256>(sum, sh, &tot);
    if (before <= r && r < before + sum) {                       /* exactly one thread */
        long long rr = r - before;
        int d = 0;
        while (rr >= (long long)c[d]) { rr -= c[d]; ++d; }
        ps->bin = threadIdx.x * PER + d;
        ps->r = rr;
        ps->cbin = c[d];
    }
}

/* the target bins' keys, per level, and the least key above each target bin */
__global__ __launch_bounds__(256) void k_qv_collect(QvArgs A) {
    const int f = blockIdx.y;
    if (!ql_sel(A.Q, f)) return;
    const int64_t d0 = A.Q.doff[f], n = A.Q.doff[f + 1] - d0;
    const int64_t c0 = (int64_t)blockIdx.x * QV_CHUNK;
    if (c0 >= n) return;
    const int64_t c1 = min<int64_t>(n, c0 + QV_CHUNK);
    const int L = A.Q.n_levels, lane = lane_id();
    const QvRange g = A.rg[f];
    __shared__ int s_tb[Q_SLOTS];
    if (threadIdx.x < L) s_tb[threadIdx.x] = A.st[(int64_t)f * Q_SLOTS + threadIdx.x].bin;
    __syncthreads();
    int tb[Q_SLOTS];
    unsigned long long mn[Q_SLOTS];
#pragma unroll
    for (int l = 0; l < Q_SLOTS; ++l) { tb[l] = l < L ? s_tb[l] : QV_BINS; mn[l] = ~0ull; }
    const double *x = A.Q.env + d0;
    unsigned long long *cb = A.cand + d0 * Q_SLOTS;
    for (int64_t i0 = c0; i0 < c1; i0 += 256) {                 /* uniform trip count: ballots inside */
        const int64_t i = i0 + threadIdx.x;
        const bool in = i < c1;
        const uint64_t k = in ? f64_key(x[i]) : 0ull;
        const int b = in ? qv_bin(k, g) : -1;
#pragma unroll
        for (int l = 0; l < Q_SLOTS; ++l) {
            if (l >= L) continue;
            const bool hit = b == tb[l];
            if (b > tb[l] && k < mn[l]) mn[l] = k;
            const uint64_t bal = __ballot(hit);
            if (bal) {                                           /* one counter atomic per wave and level */
                unsigned int base = 0;
                if (lane == __ffsll((long long)bal) - 1)
                    base = atomicAdd(&A.st[(int64_t)f * Q_SLOTS + l].cnt, (unsigned int)__popcll(bal));
                base = (unsigned int)__shfl((int)base, __ffsll((long long)bal) - 1);
                if (hit) cb[(int64_t)l * n + base + __popcll(bal & ((1ull << lane) - 1ull))] = k;
            }
        }
    }
#pragma unroll
    for (int l = 0; l < Q_SLOTS; ++l) {
        if (l >= L) continue;
        unsigned long long m = mn[l];
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long om = __shfl_xor(m, o);
            m = om < m ? om : m;
        }
        if (lane == 0 && m != ~0ull) atomicMin(&A.st[(int64_t)f * Q_SLOTS + l].next, m);
    }
}

/* per (recording, level): the r-th and (r+1)-th smallest of the gathered keys
 * by an 8-bit radix select over them (L2-resident: a few hundred keys on the
 * C5 envelopes), the (r+1)-th from the bins above when the bin ends at r;
 * then numpy's _lerp as k_ql_final */
__global__ __launch_bounds__(256) void k_qv_final(QvArgs A) {
    const int f = blockIdx.x, l = blockIdx.y;
    if (!ql_sel(A.Q, f) || l >= A.Q.n_levels) return;
    const int64_t d0 = A.Q.doff[f], n = A.Q.doff[f + 1] - d0;
    const QvState st = A.st[(int64_t)f * Q_SLOTS + l];
    const unsigned long long *cb = A.cand + d0 * Q_SLOTS + (int64_t)l * n;
    const long long c = st.cnt;
    __shared__ unsigned int hist[256];
    __shared__ unsigned long long s_pre;
    __shared__ long long s_rank;
    auto select = [&](long long rank) -> unsigned long long {
        unsigned long long prefix = 0ull, mask = 0ull;
        for (int pass = 0; pass < 8; ++pass) {
            const int shf = 56 - 8 * pass;
            hist[threadIdx.x] = 0u;
            __syncthreads();
            for (long long i = threadIdx.x; i < c; i += 256) {
                const unsigned long long k = cb[i];
                if ((k & mask) == prefix) atomicAdd(&hist[(k >> shf) & 255u], 1u);
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                long long rr = rank;
                int d = 0;
                while (d < 255 && rr >= (long long)hist[d]) { rr -= hist[d]; ++d; }
                s_pre = prefix | ((unsigned long long)d << shf);
                s_rank = rr;
            }
            __syncthreads();
            prefix = s_pre;
            rank = s_rank;
            mask |= 0xFFull << shf;
            __syncthreads();
        }
        return prefix;
    };
    const unsigned long long ka = select(st.r);
    double res = key_f64(ka);
    if (!st.top) {
        const unsigned long long kb = st.r + 1 < c ? select(st.r + 1) : st.next;
        res = np_lerp(res, key_f64(kb), (double)(n - 1) * A.Q.q[l] - (double)st.lo);
    }
    if (threadIdx.x == 0)
        for (int s = 0; s < Q_SLOTS; ++s)
            if ((A.Q.slot[l] >> s) & 1) A.Q.qv[(int64_t)f * Q_SLOTS + s] = res;
}

/* ------------------------------------------------------------------------ */
__global__ __launch_bounds__(256) void k_block_stats(BlockStatArgs A) {
    const int f = blockIdx.x;
    if (f >= A.n_files || !A.active[f]) return;
    const int64_t n = A.doff[f + 1] - A.doff[f];
    if (n <= A.skip_le) return;
    const int64_t nb = (n + 63) >> 6;
    const double *x = A.env + A.doff[f];
    double *bmx = A.bmax + A.boff[f], *bmn = A.bmin + A.boff[f];
    const int lane = lane_id();
    const double INF = __builtin_inf();
    for (int64_t b = (int64_t)blockIdx.y * 4 + wave_id(); b < nb; b += 4 * (int64_t)gridDim.y) {
        int64_t i = (b << 6) + lane;
        double v = i < n ? x[i] : __builtin_nan("");
        double mx = wave_max(i < n ? v : -INF);
        double mn = wave_min(i < n ? v : INF);
        if (lane == 0) { bmx[b] = mx; bmn[b] = mn; }
    }
}

/* ------------------------------------------------------------------------ */
/* k_quantile_reg: all quantile levels and the block tables of one recording
 * from a single read of env held in registers (item it of thread t is
 * position it*QR_T + t, so a wave's items of one round form one 64-sample
 * block); the select itself is qr_select (bpmx_qsel.h), which k_hilbert_env
 * also runs on the envelope it writes. */
__global__ __launch_bounds__(QR_T) void k_quantile_reg(QuantArgs A, BlockStatArgs B) {
    const int f = blockIdx.x;
    if (f >= A.n_files || !A.active[f] || (A.skip && A.skip[f])) return;
    const int64_t n = A.doff[f + 1] - A.doff[f];
    if (n > QR_MAX) return;
    const double *x = A.env + A.doff[f];
    const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
    __shared__ QrShared sh;
    const double INF = __builtin_inf();
    uint64_t key[QR_IT];
    double *bmx = B.bmax + B.boff[f], *bmn = B.bmin + B.boff[f];
#pragma unroll
    for (int it = 0; it < QR_IT; ++it) {
        const int64_t i = (int64_t)it * QR_T + tid;
        const bool ok = i < n;
        const double v = ok ? x[i] : 0.0;
        key[it] = ok ? f64_key(v) : 0ull;
        const int64_t b0 = (int64_t)it * QR_T + wid * 64;
        if (A.stats && b0 < n) {                             /* block max/min (k_block_stats) */
            const double mx = wave_max(ok ? v : -INF), mn = wave_min(ok ? v : INF);
            if (lane == 0) { bmx[b0 >> 6] = mx; bmn[b0 >> 6] = mn; }
        }
    }
    qr_select(key, n, A, f, sh);
}

/* ------------------------------------------------------------------------ */
/* prominence of peak p (value xp = sg*e[p]) — _peak_prominences, wlen = -1:
 * min of x over (left_higher, p] and [p, right_higher), prom = xp - max(...).
 * One wave; at most two dependent rounds of global loads: p's own 64-sample
 * block (shared by both sides), then — for a side whose higher sample lies
 * beyond it — the block found by walking the block max tables (LDS). */
template <int NP>
__device__ void prominence_waves(const double *e, double sg, int64_t n, const double *bmx, const double *bmn,
                                 const int64_t *pp, const double *xpp, double *prom) {
    const int lane = lane_id();
    const int64_t nb = (n + 63) >> 6;
    const double INF = __builtin_inf();
    double v[NP], lm[NP], rm[NP];
    int64_t qL[NP], qR[NP];
#pragma unroll
    for (int c = 0; c < NP; ++c) {             /* first round of loads: each peak's own block */
        const int64_t pos = ((pp[c] >> 6) << 6) + lane;
        v[c] = (pp[c] >= 0 && pos < n) ? sg * e[pos] : -INF;
    }
#pragma unroll
    for (int c = 0; c < NP; ++c) {
        const int64_t p = pp[c];
        const double xp = xpp[c];
        const int64_t blk = p >> 6;
        const int64_t pos = (blk << 6) + lane;
        qL[c] = qR[c] = -1;
        lm[c] = rm[c] = INF;
        if (p < 0) continue;                   /* uniform: empty slot */
        const unsigned long long mL = __ballot(pos <= p && v[c] > xp);
        const unsigned long long mR = __ballot(pos >= p && pos < n && v[c] > xp);
        if (mL) {
            const int L = 63 - __clzll(mL);
            lm[c] = (pos <= p && lane > L) ? v[c] : INF;
        } else {
            lm[c] = pos <= p ? v[c] : INF;
            for (int64_t bs = blk - 1; bs >= 0; bs -= 64) {
                const int64_t b = bs - lane;
                const bool vb = b >= 0;
                const double bm = vb ? (sg > 0 ? bmx[b] : -bmn[b]) : -INF;
                const double bn = vb ? (sg > 0 ? bmn[b] : -bmx[b]) : INF;
                const unsigned long long mb = __ballot(vb && bm > xp);
                if (mb) {
                    const int Lb = __ffsll((long long)mb) - 1;
                    lm[c] = fmin(lm[c], lane < Lb ? bn : INF);
                    qL[c] = bs - Lb;
                    break;
                }
                lm[c] = fmin(lm[c], bn);
            }
        }
        if (mR) {
            const int R = __ffsll((long long)mR) - 1;
            rm[c] = (pos >= p && pos < n && lane < R) ? v[c] : INF;
        } else {
            rm[c] = (pos >= p && pos < n) ? v[c] : INF;
            for (int64_t bs = blk + 1; bs < nb; bs += 64) {
                const int64_t b = bs + lane;
                const bool vb = b < nb;
                const double bm = vb ? (sg > 0 ? bmx[b] : -bmn[b]) : -INF;
                const double bn = vb ? (sg > 0 ? bmn[b] : -bmx[b]) : INF;
                const unsigned long long mb = __ballot(vb && bm > xp);
                if (mb) {
                    const int Rb = __ffsll((long long)mb) - 1;
                    rm[c] = fmin(rm[c], lane < Rb ? bn : INF);
                    qR[c] = bs + Rb;
                    break;
                }
                rm[c] = fmin(rm[c], bn);
            }
        }
    }
    double vl[NP], vr[NP];
#pragma unroll
    for (int c = 0; c < NP; ++c) {             /* second round: the far blocks, all at once */
        const int64_t ql = (qL[c] << 6) + lane, qr = (qR[c] << 6) + lane;
        vl[c] = qL[c] >= 0 ? sg * e[ql] : -INF;
        vr[c] = (qR[c] >= 0 && qr < n) ? sg * e[qr] : -INF;
    }
#pragma unroll
    for (int c = 0; c < NP; ++c) {
        const double xp = xpp[c];
        if (qL[c] >= 0) {
            const int L2 = 63 - __clzll(__ballot(vl[c] > xp));
            lm[c] = fmin(lm[c], lane > L2 ? vl[c] : INF);
        }
        if (qR[c] >= 0) {
            const int64_t qr = (qR[c] << 6) + lane;
            const int R2 = __ffsll((long long)__ballot(qr < n && vr[c] > xp)) - 1;
            rm[c] = fmin(rm[c], (qr < n && lane < R2) ? vr[c] : INF);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
        for (int c = 0; c < NP; ++c) {
            lm[c] = fmin(lm[c], __shfl_xor(lm[c], o));
            rm[c] = fmin(rm[c], __shfl_xor(rm[c], o));
        }
    }
#pragma unroll
    for (int c = 0; c < NP; ++c) prom[c] = xpp[c] - fmax(lm[c], rm[c]);
}

constexpr int FP_T = 1024;
#ifndef BPMX_FP_NP
#define BPMX_FP_NP 2      /* prominences per wave per round (their loads overlap) */
#endif
#ifndef BPMX_FP_G
#define BPMX_FP_G 8       /* local-maxima iterations per load group */
#endif
#ifndef BPMX_FP_LB
#define BPMX_FP_LB 8      /* min waves per EU (register budget) */
#endif
constexpr int FP_NBMAX = 2048;   /* block tables staged in LDS up to 131072 samples */
constexpr int FP_MC = 2048;      /* candidates kept in LDS up to this many */

__global__ __launch_bounds__(FP_T, BPMX_FP_LB) void k_find_peaks(PeakArgs A) {
    const int f = blockIdx.x;
    if (f >= A.n_files || !A.active[f] || (A.only && !A.only[f])) return;
    const int64_t d0 = A.doff[f];
    const int64_t n = A.doff[f + 1] - d0;
    const double *e = A.env + d0;
    const double *h = A.height ? A.height + d0 : nullptr;
    const double sg = A.sign;
    const int tid = threadIdx.x;
    __shared__ int sh[FP_T / 64 + 1];
    __shared__ int s_flag, s_tie;
    __shared__ double s_bmx[FP_NBMAX], s_bmn[FP_NBMAX];
    __shared__ double s_cv[FP_MC];
    __shared__ int32_t s_cp[FP_MC];
    __shared__ uint8_t s_st[FP_MC];
    STAMP_DECL

    /* block tables (the prominence walks read them): computed here into LDS
     * for recordings they fit (this kernel only runs for the few recordings
     * k_find_peaks_lds hands over), from k_block_stats' global tables beyond */
    const int64_t nblk = (n + 63) >> 6;
    const double *bmx = A.bmax + A.boff[f], *bmn = A.bmin + A.boff[f];
    if (nblk <= FP_NBMAX) {
        const double INF = __builtin_inf();
        for (int64_t b = wave_id(); b < nblk; b += FP_T / 64) {
            const int64_t i = (b << 6) + lane_id();
            const double v = i < n ? e[i] : 0.0;
            const double mx = wave_max(i < n ? v : -INF), mn = wave_min(i < n ? v : INF);
            if (lane_id() == 0) { s_bmx[b] = mx; s_bmn[b] = mn; }
        }
        bmx = s_bmx;
        bmn = s_bmn;
    }

    STAMP(0);
    /* (1)+(2) local maxima with plateau midpoints, height filter.  Position
     * i = 1 + (g*FP_G + it)*FP_T + tid; a group of FP_G iterations issues its
     * loads together, then one (iteration, wave)-ordered scan places the hits. */
    constexpr int FP_G = BPMX_FP_G;
    __shared__ int s_gc[FP_G][FP_T / 64];
    int m = 0;
    const int64_t iters = n > 2 ? (n - 2 + FP_T - 1) / FP_T : 0;
    int32_t *cp_g = A.cand + d0;
    for (int64_t g0 = 0; g0 < iters; g0 += FP_G) {
        int32_t pk[FP_G];
        unsigned hits = 0;
#pragma unroll
        for (int it = 0; it < FP_G; ++it) {
            const int64_t i = 1 + (g0 + it) * FP_T + tid;
            pk[it] = 0;
            if (g0 + it < iters && i < n - 1) {
                const double xi = sg * e[i];
                if (sg * e[i - 1] < xi) {
                    int64_t ia = i + 1;
                    while (ia < n - 1 && sg * e[ia] == xi) ia++;
                    if (sg * e[ia] < xi) {
                        const int64_t p = (i + ia - 1) >> 1;
                        if (!h || h[p] <= sg * e[p]) { hits |= 1u << it; pk[it] = (int32_t)p; }
                    }
                }
            }
        }
#pragma unroll
        for (int it = 0; it < FP_G; ++it) {
            const unsigned long long bal = __ballot((hits >> it) & 1u);
            if (lane_id() == 0) s_gc[it][wave_id()] = __popcll(bal);
        }
        __syncthreads();
        if (wave_id() == 0) {                                /* exclusive scan over FP_G x 16 counts */
            constexpr int NE = FP_G * (FP_T / 64);
            int v[NE / 64], sum = 0;
#pragma unroll
            for (int u = 0; u < NE / 64; ++u) {
                v[u] = (&s_gc[0][0])[lane_id() * (NE / 64) + u];
                sum += v[u];
            }
            int x = sum;
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(x, o);
                if (lane_id() >= o) x += y;
            }
            int run = x - sum;
#pragma unroll
            for (int u = 0; u < NE / 64; ++u) {
                (&s_gc[0][0])[lane_id() * (NE / 64) + u] = run;
                run += v[u];
            }
            if (lane_id() == 63) s_flag = x;
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < FP_G; ++it) {
            const unsigned long long bal = __ballot((hits >> it) & 1u);
            if ((hits >> it) & 1u) {
                const int k = m + s_gc[it][wave_id()] + __popcll(bal & ((1ull << lane_id()) - 1ull));
                cp_g[k] = pk[it];
            }
        }
        m += s_flag;
        __syncthreads();
    }
    if (A.cand_out) {                                        /* bpmx_run_ordered: the candidate list */
        for (int j = tid; j < m; j += FP_T) A.cand_out[d0 + j] = cp_g[j];
        if (tid == 0) A.ncand_out[f] = m;
    }
    /* the caller's visiting ranks (np.argsort of the heights): they decide the
     * distance filter alone; without them the stable order below */
    const int32_t *rk = (A.rank && A.use_rank && A.use_rank[f]) ? A.rank + d0 : nullptr;
    const bool lds = m <= FP_MC;
    int32_t *cp = lds ? s_cp : cp_g;
    uint8_t *st = lds ? s_st : A.state + d0;
    if (lds) {
        for (int j = tid; j < m; j += FP_T) {
            const int32_t p = cp_g[j];
            s_cp[j] = p;
            s_cv[j] = sg * e[p];
        }
    }
    __syncthreads();
    STAMP(1);
    auto cval = [&](int k) { return lds ? s_cv[k] : sg * e[cp[k]]; };

    /* (3) distance: rounds of local decisions */
    const int64_t dist = A.distance;
    for (int j = tid; j < m; j += FP_T) st_state(&st[j], dist > 1 ? ST_UNDECIDED : ST_KEPT);
    if (tid == 0) s_tie = 0;
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
                const int64_t pj = cp[j];
                const double vj = cval(j);
                const int32_t rj = rk ? rk[j] : 0;
                bool killed = false, blocked = false;
                for (int k = j - 1; k >= 0 && pj - cp[k] < dist; --k) {
                    if (rk ? rk[k] > rj : cval(k) > vj) { /* earlier index wins only when strictly higher */
                        const uint8_t s = ld_state(&st[k]);
                        if (s == ST_KEPT) { killed = true; break; }
                        if (s == ST_UNDECIDED) blocked = true;
                    }
                }
                if (!killed) {
                    for (int k = j + 1; k < m && cp[k] - pj < dist; ++k) {
                        if (rk ? rk[k] > rj : cval(k) >= vj) {  /* later index wins ties (stable argsort order) */
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

    STAMP(2);
    /* decisive tie (include/bpmx.h BPMX_F_*_TIE): a removed candidate with no
     * strictly higher kept candidate within dist was removed by an equal one
     * (none with the caller's ranks: the order is then the reference's) */
    if (dist > 1 && !rk) {
        for (int j = tid; j < m; j += FP_T) {
            if (ld_state(&st[j]) != ST_REMOVED) continue;
            const int64_t pj = cp[j];
            const double vj = cval(j);
            bool dom = false;
            for (int k = j - 1; !dom && k >= 0 && pj - cp[k] < dist; --k)
                dom = cval(k) > vj && st_kept_by_distance(ld_state(&st[k]));
            for (int k = j + 1; !dom && k < m && cp[k] - pj < dist; ++k)
                dom = cval(k) > vj && st_kept_by_distance(ld_state(&st[k]));
            if (!dom) s_tie = 1;
        }
    }
    /* (4) prominences of the kept candidates, one wave each */
    const double thr = A.qv[(int64_t)f * Q_SLOTS + A.qslot];
    /* the kept candidates are taken NP at a time per wave so that their global
     * loads overlap */
    constexpr int NP = BPMX_FP_NP;
#ifdef BPMX_STAMPS
    __shared__ unsigned long long s_wt_prom[FP_T / 64];
    const unsigned long long tp0 = __builtin_amdgcn_s_memtime();
#endif
    {
        const int nw = FP_T / 64, wv = wave_id();
        int j = wv;
        for (;;) {
            int64_t pp[NP];
            double xp[NP], pr[NP];
            int jj[NP];
#pragma unroll
            for (int c = 0; c < NP; ++c) {
                while (j < m && ld_state(&st[j]) != ST_KEPT) j += nw;
                jj[c] = j < m ? j : -1;
                pp[c] = j < m ? cp[j] : -1;
                xp[c] = j < m ? cval(j) : 0.0;
                j += nw;
            }
            if (jj[0] < 0) break;
            prominence_waves<NP>(e, sg, n, bmx, bmn, pp, xp, pr);
            if (lane_id() == 0) {
#pragma unroll
                for (int c = 0; c < NP; ++c)
                    if (jj[c] >= 0) st_state(&st[jj[c]], thr <= pr[c] ? ST_FINAL : ST_PREMOVED);
            }
        }
    }
#ifdef BPMX_STAMPS
    if (lane_id() == 0) s_wt_prom[wave_id()] = __builtin_amdgcn_s_memtime() - tp0;
#endif
    __syncthreads();
    STAMP(3);
#ifdef BPMX_STAMPS
    if (threadIdx.x == 0) {
        unsigned long long mx = 0, sm = 0;
        for (int w = 0; w < FP_T / 64; ++w) { mx = s_wt_prom[w] > mx ? s_wt_prom[w] : mx; sm += s_wt_prom[w]; }
        _st_acc[5] += mx;
        _st_acc[6] += sm / (FP_T / 64);
    }
#endif

    /* (5) ordered compaction */
    int64_t *out = A.out + d0;
    int w = 0;
    for (int q0 = 0; q0 < m; q0 += FP_T) {
        const int j = q0 + tid;
        const bool keep = j < m && ld_state(&st[j]) == ST_FINAL;
        int tot;
        const int off = block_scan_flag<FP_T>(keep, sh, &tot);
        if (keep) {
            out[w + off] = cp[j];
            if (A.outv) A.outv[d0 + w + off] = sg * cval(j);
        }
        w += tot;
    }
    if (tid == 0) {
        A.nout[f] = w;
        if (A.run_out) A.run_out[f] = w >= A.run_min ? 1 : 0;
        if (A.flags) {
            if (rk) A.flags[f] |= A.ordered_bit;
            else if (s_tie) A.flags[f] |= A.tie_bit;
        }
    }
    STAMP(4);
    STAMP_FLUSH(A.stamps);
}

/* ------------------------------------------------------------------------ */
/* k_find_peaks_lds: the same find_peaks, with prominences from the local
 * extrema held in LDS instead of walks over the samples in global memory.
 *
 * Between two consecutive local maxima c_i, c_(i+1) of the signal (scipy's
 * _local_maxima_1d, plateau midpoints) there is no other local maximum, so
 * the samples there fall to exactly one valley (a strict local minimum or a
 * flat bottom) and rise again; call its value v_i.  v_(-1) = min(x[0], the
 * valley before c_0, if any) and v_(M-1) = min(x[n-1], the valley after the
 * last maximum) cover the edges.  _peak_prominences (wlen = -1) walks left
 * from peak c_j while x <= x[c_j] and stops at the first higher sample; every
 * sample it passes lies in gaps k* .. j-1, where c_k* is the nearest maximum
 * with x[c_k*] > x[c_j] (the higher sample sits on c_k*'s falling slope), and
 * each gap's minimum is its valley, so
 *     left_min = min(v_k*, ..., v_(j-1))   (k* = -1 if none is higher)
 * and symmetrically on the right.  All of it is in LDS: per recording ~1000
 * maxima (native mode) to ~2400 (reference mode); a recording with more than
 * FL_MC maxima is flagged for k_find_peaks.  Everything else — height,
 * distance rounds, prominence threshold, ordered output — is k_find_peaks'. */

__global__ __launch_bounds__(FP_T, 8) void k_find_peaks_lds(PeakArgs A) {
    const int f = blockIdx.x;
    if (f >= A.n_files) return;
    const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
    if (!A.active[f]) {
        if (tid == 0) A.fallback[f] = 0;
        return;
    }
    const int64_t d0 = A.doff[f];
    const int64_t n = A.doff[f + 1] - d0;
    if (n > A.lds_nmax) {                                    /* long recording: the k_fpl_* kernels */
        if (tid == 0) A.fallback[f] = 1;
        return;
    }
    const int sgn = A.sign > 0 ? 1 : -1;
    const int so = A.scan_ok ? A.scan_ok[f] : 0;             /* this run's scan record (read before tid 0 updates it) */
    const double *e = A.env + d0;
    const double *h = A.height ? A.height + d0 : nullptr;
    const double sg = A.sign;
    const double INF = __builtin_inf();
    constexpr int NW = FP_T / 64;
    constexpr int FP_G = 4;                                  /* iterations per load group (register budget) */
    __shared__ int32_t s_mp[FL_MC];
    __shared__ double s_mh[FL_MC];
    __shared__ double s_vv[FL_MC + 1];
    __shared__ uint8_t s_st[FL_MC];
    /* block summaries for the prominence walks at 8, 64 and 512 maxima:
     * max height, min of the gap valleys a left walk crosses (vv[k + 1]) and
     * a right walk crosses (vv[k]) */
    constexpr int FL_B1 = FL_MC / 8, FL_B2 = FL_MC / 64, FL_B3 = FL_MC / 512;
    __shared__ double s_bh[FL_B1 + FL_B2 + FL_B3], s_bvl[FL_B1 + FL_B2 + FL_B3], s_bvr[FL_B1 + FL_B2 + FL_B3];
    __shared__ int s_gc[2][FP_G][NW];
    __shared__ int sh[NW + 1];
    __shared__ int s_tie;
    STAMP_DECL

    /* (1) local maxima (plateau midpoints) and valleys, in order: wave w
     * scans its own contiguous run of positions 64 at a time (coalesced loads,
     * no workgroup barrier), compacting its hits into its own stretch of the
     * global scratch (a run of c positions holds at most c hits); one scan of
     * the 16 per-wave counts then places every run (bpmx_fpscan.h).  When this
     * run's scan record holds the lists (written only by the trough launch,
     * read by the peak launch) they are taken as they are, swapped for the
     * other sign: -env's maxima are env's valleys and its valleys env's maxima. */
    static_assert(NW == FPS_NW, "the scan record's per-wave runs");
    int64_t w0, w1;
    fp_scan_run(n, wid, w0, w1);
    int32_t *mp_g, *vp_g;
    double *mv_g, *vv_g, vsg = 1.0;                          /* the extrema's values, made for the lists' sign */
    int cm, cv;                                              /* wave-uniform counts */
    if (so != 0) {
        const bool direct = so == sgn;
        mp_g = (direct ? A.cand : A.vcand) + d0;
        vp_g = (direct ? A.vcand : A.cand) + d0;
        mv_g = (direct ? A.cval : A.vval) + d0;
        vv_g = (direct ? A.vval : A.cval) + d0;
        vsg = direct ? 1.0 : -1.0;
        const int c0 = A.scan_cnt[((int64_t)f * NW + wid) * 2], c1 = A.scan_cnt[((int64_t)f * NW + wid) * 2 + 1];
        cm = direct ? c0 : c1;
        cv = direct ? c1 : c0;
    } else {
        mp_g = A.cand + d0;
        vp_g = A.vcand + d0;
        mv_g = A.cval + d0;
        vv_g = A.vval + d0;
        fp_scan_wave([&](int64_t i) { return sg * e[i]; }, n, w0, w1, mp_g, vp_g, mv_g, vv_g, cm, cv);
        if (A.scan_ok && lane == 0) {
            A.scan_cnt[((int64_t)f * NW + wid) * 2] = cm;
            A.scan_cnt[((int64_t)f * NW + wid) * 2 + 1] = cv;
        }
    }
    if (lane == 0) { s_gc[0][0][wid] = cm; s_gc[1][0][wid] = cv; }
    __syncthreads();
    int M = 0, om = 0;
    for (int w = 0; w < NW; ++w) {
        if (w == wid) om = M;
        M += s_gc[0][0][w];
    }
    STAMP(1);
    if (M > FL_MC) {                                         /* k_find_peaks takes this recording */
        if (tid == 0) {
            A.fallback[f] = 1;
            if (A.scan_ok) A.scan_ok[f] = 0;                 /* (it rewrites cand) */
        }
        return;
    }
    if (tid == 0) {
        A.fallback[f] = 0;
        if (A.scan_ok && so == 0) A.scan_ok[f] = sgn;
    }
    const int64_t dist = A.distance;
    for (int t = lane; t < cm; t += 64) {                    /* this wave's run of maxima */
        const int32_t p = mp_g[w0 - 1 + t];
        const double xv = vsg * mv_g[w0 - 1 + t];
        const int k = om + t;
        s_mp[k] = p;
        s_mh[k] = xv;
        s_st[k] = (!h || h[p] <= xv) ? (dist > 1 ? ST_UNDECIDED : ST_KEPT) : ST_HEIGHT;   /* height filter */
    }
    if (tid == 0) s_tie = 0;
    for (int k = tid; k <= M; k += FP_T) s_vv[k] = k == 0 ? sg * e[0] : (k == M ? sg * e[n - 1] : INF);
    __syncthreads();
    /* valley -> its gap: gap g (between c_g and c_(g+1)) is s_vv[g + 1].
     * Maxima and valleys alternate along the recording (between two maxima
     * the samples fall to exactly one valley, plateaus included), so the
     * wave's valley t has t of the wave's maxima before it, plus one when the
     * wave's first extremum is a maximum */
    const int vfirst = (cm > 0 && (cv == 0 || mp_g[w0 - 1] < vp_g[w0 - 1])) ? 1 : 0;
    for (int t = lane; t < cv; t += 64) {
        const int lo = om + t + vfirst;
        const double val = vsg * vv_g[w0 - 1 + t];
        if (lo == 0 || lo == M) s_vv[lo] = fmin(s_vv[lo], val);   /* edge gaps: at most one valley each */
        else s_vv[lo] = val;
    }
    __syncthreads();
    STAMP(2);

    /* (3) distance: rounds of local decisions (k_find_peaks' rule: a
     * candidate is removed once a higher-priority candidate within `dist` is
     * kept, kept once none is undecided).  Positions and heights do not
     * change, so each candidate's higher-priority neighbours (left: strictly
     * higher, right: at least as high) are listed once, up to eight (8-bit offsets) in
     * registers; a round then only reads their states. */
#ifdef BPMX_FP_NODIST
    if (false) {
#else
    if (dist > 1) {
#endif
        constexpr int FP_R = FL_MC / FP_T;
        constexpr int FP_NB = 8;                             /* neighbours listed per candidate */
        uint32_t nb[FP_R][2];                                /* eight signed 8-bit offsets k - j */
        int nbc[FP_R];                                       /* count; -1: more than eight or too far (full scan) */
#pragma unroll
        for (int r = 0; r < FP_R; ++r) {
            const int j = tid + r * FP_T;
            nb[r][0] = nb[r][1] = 0u;
            nbc[r] = 0;
            if (j >= M || s_st[j] != ST_UNDECIDED) continue;
            const int64_t pj = s_mp[j];
            const double vj = s_mh[j];
            int c = 0;
            auto add = [&](int k) {
                const int o = k - j;
                if (o < -128 || o > 127) c = FP_NB;          /* forces the full scan */
                if (c < FP_NB) nb[r][c >> 2] |= ((uint32_t)o & 0xFFu) << (8 * (c & 3));
                ++c;
            };
            for (int k = j - 1; k >= 0 && pj - s_mp[k] < dist; --k)
                if (s_mh[k] > vj && s_st[k] == ST_UNDECIDED) add(k);
            for (int k = j + 1; k < M && s_mp[k] - pj < dist; ++k)
                if (s_mh[k] >= vj && s_st[k] == ST_UNDECIDED) add(k);
            nbc[r] = c <= FP_NB ? c : -1;
        }
        STAMP(6);
        /* Rounds run wave-locally (a candidate's neighbours are mostly in its
         * own wave: lanes j +- 1 ...) until the wave makes no progress; one
         * workgroup barrier then lets decisions cross wave boundaries.  A
         * decision needs a KEPT neighbour (final) or no UNDECIDED one (a stale
         * read only delays it), so unsynchronised reads are safe. */
        /* this thread's undecided entries: only it writes their states */
        uint32_t und = 0u;
#pragma unroll
        for (int r = 0; r < FP_R; ++r) {
            const int j = tid + r * FP_T;
            if (j < M && s_st[j] == ST_UNDECIDED) und |= 1u << r;
        }
        for (int gi = 0; gi <= M; ++gi) {
            for (int lr = 0; lr <= M; ++lr) {
                bool progress = false;
                /* the neighbour counts opaque per round: otherwise the 24
                 * (r, q < nbc[r]) lane masks are hoisted out of the rounds into
                 * SGPRs, which spill, and every round pays a readlane per mask */
                int nbv[FP_R];
#pragma unroll
                for (int r = 0; r < FP_R; ++r) {
                    nbv[r] = nbc[r];
                    asm volatile("" : "+v"(nbv[r]));
                }
                /* every listed neighbour's state first (independent LDS reads),
                 * then the decisions */
                uint32_t kill = 0u, block = 0u;
#pragma unroll
                for (int r = 0; r < FP_R; ++r) {
                    if (!((und >> r) & 1u) || nbv[r] < 0) continue;
                    const int j = tid + r * FP_T;
#pragma unroll
                    for (int q = 0; q < FP_NB; ++q) {
                        if (q < nbv[r]) {
                            const int k = j + (int)(int8_t)((nb[r][q >> 2] >> (8 * (q & 3))) & 0xFFu);
                            const uint8_t st = ld_state(&s_st[k]);
                            kill |= (st == ST_KEPT ? 1u : 0u) << r;
                            block |= (st == ST_UNDECIDED ? 1u : 0u) << r;
                        }
                    }
                }
#pragma unroll
                for (int r = 0; r < FP_R; ++r) {
                    if (!((und >> r) & 1u)) continue;
                    const int j = tid + r * FP_T;
                    bool killed = (kill >> r) & 1u, blocked = (block >> r) & 1u;
                    if (nbc[r] < 0) {                         /* more than FP_NB: scan */
                        const int64_t pj = s_mp[j];
                        const double vj = s_mh[j];
                        for (int k = j - 1; k >= 0 && pj - s_mp[k] < dist; --k) {
                            if (s_mh[k] > vj) {
                                const uint8_t st = ld_state(&s_st[k]);
                                if (st == ST_KEPT) { killed = true; break; }
                                if (st == ST_UNDECIDED) blocked = true;
                            }
                        }
                        if (!killed) {
                            for (int k = j + 1; k < M && s_mp[k] - pj < dist; ++k) {
                                if (s_mh[k] >= vj) {
                                    const uint8_t st = ld_state(&s_st[k]);
                                    if (st == ST_KEPT) { killed = true; break; }
                                    if (st == ST_UNDECIDED) blocked = true;
                                }
                            }
                        }
                    }
                    if (killed || !blocked) {
                        st_state(&s_st[j], killed ? ST_REMOVED : ST_KEPT);
                        und &= ~(1u << r);
                        progress = true;
                    }
                }
                if (!__ballot(progress)) break;                  /* wave-uniform */
            }
            if (!__syncthreads_or(und != 0u)) break;
        }
    }
    STAMP(3);

    /* (4) prominences of the kept maxima, one thread each: walk the maxima
     * outwards to the nearest higher one, taking the gap valleys passed on the
     * way; aligned runs of 512, 64 or 8 maxima that are all no higher are
     * skipped whole through their block maximum and block valley minimum */
    {
        /* level 1 (8 maxima) from the maxima, levels 2 and 3 from the level below */
        const int N1 = (M + 7) >> 3, N2 = (M + 63) >> 6, N3 = (M + 511) >> 9;
        for (int b = tid; b < N1; b += FP_T) {
            double hx = -INF, vl = INF, vr = INF;
            for (int k = b * 8; k < min(M, b * 8 + 8); ++k) {
                hx = fmax(hx, s_mh[k]);
                vl = fmin(vl, s_vv[k + 1]);
                vr = fmin(vr, s_vv[k]);
            }
            s_bh[b] = hx; s_bvl[b] = vl; s_bvr[b] = vr;
        }
        __syncthreads();
        for (int lv = 0; lv < 2; ++lv) {
            const int src = lv == 0 ? 0 : FL_B1, dst = lv == 0 ? FL_B1 : FL_B1 + FL_B2;
            const int nd_ = lv == 0 ? N2 : N3, ns_ = lv == 0 ? N1 : N2;
            for (int b = tid; b < nd_; b += FP_T) {
                double hx = -INF, vl = INF, vr = INF;
                for (int c = b * 8; c < min(ns_, b * 8 + 8); ++c) {
                    hx = fmax(hx, s_bh[src + c]);
                    vl = fmin(vl, s_bvl[src + c]);
                    vr = fmin(vr, s_bvr[src + c]);
                }
                s_bh[dst + b] = hx; s_bvl[dst + b] = vl; s_bvr[dst + b] = vr;
            }
            __syncthreads();
        }
        const double thr = A.qv[(int64_t)f * Q_SLOTS + A.qslot];
        const double *bh2 = s_bh + FL_B1, *bh3 = s_bh + FL_B1 + FL_B2;
        /* the kept maxima, compacted (in order) into the recording's stretch
         * of the state scratch (2 bytes each; at most n / 2 of them), so the
         * walks run on ~K / 64 full waves instead of every wave's few kept
         * lanes; the distance filter's removals get the tie check first */
        int16_t *kl = reinterpret_cast<int16_t *>(A.state + ((d0 + 1) & ~(int64_t)1));
        int K = 0;
        for (int q0 = 0; q0 < M; q0 += FP_T) {
            const int j = q0 + tid;
            const uint8_t sj = j < M ? s_st[j] : (uint8_t)ST_HEIGHT;
            if (sj == ST_REMOVED) {
                /* removed by the distance filter: a decisive tie (include/bpmx.h
                 * BPMX_F_*_TIE) unless a strictly higher candidate the filter
                 * kept lies within dist */
                const int64_t pj = s_mp[j];
                const double vj = s_mh[j];
                bool dom = false;
                for (int k = j - 1; !dom && k >= 0 && pj - s_mp[k] < dist; --k)
                    dom = s_mh[k] > vj && st_kept_by_distance(s_st[k]);
                for (int k = j + 1; !dom && k < M && s_mp[k] - pj < dist; ++k)
                    dom = s_mh[k] > vj && st_kept_by_distance(s_st[k]);
                if (!dom) s_tie = 1;
            }
            int tot;
            const int off = block_scan_flag<FP_T>(sj == ST_KEPT, sh, &tot);
            if (sj == ST_KEPT) kl[K + off] = (int16_t)j;
            K += tot;
        }
        __syncthreads();
        STAMP(7);
        for (int i = tid; i < K; i += FP_T) {
            const int j = kl[i];
            const double hj = s_mh[j];
            double lmin = INF, rmin = INF;
            /* the two walks step together, and a step reads every candidate
             * (block maxima and valley minima of the 512-, 64- and 8-maximum
             * blocks, the gap valley, the maximum) before choosing, so one LDS
             * round trip covers a step of both sides.  Left: at k, the largest
             * aligned block ending at k with no higher maximum; right: the
             * largest aligned full block starting at k. */
            int kl = j - 1, kr = j + 1;
            bool dl = false, dr = false;
            while (!(dl && dr)) {
                if (!dl) {
                    if (kl < 0) {
                        lmin = fmin(lmin, s_vv[0]);
                        dl = true;
                    } else {
                        const double b3 = bh3[kl >> 9], b2 = bh2[kl >> 6], b1 = s_bh[kl >> 3];
                        const double v3 = s_bvl[FL_B1 + FL_B2 + (kl >> 9)], v2 = s_bvl[FL_B1 + (kl >> 6)];
                        const double v1 = s_bvl[kl >> 3], vv = s_vv[kl + 1], mh = s_mh[kl];
                        const bool c3 = (kl & 511) == 511 && b3 <= hj;
                        const bool c2 = !c3 && (kl & 63) == 63 && b2 <= hj;
                        const bool c1 = !c3 && !c2 && (kl & 7) == 7 && b1 <= hj;
                        lmin = fmin(lmin, c3 ? v3 : (c2 ? v2 : (c1 ? v1 : vv)));
                        if (!(c3 || c2 || c1) && mh > hj) dl = true;
                        else kl -= c3 ? 512 : (c2 ? 64 : (c1 ? 8 : 1));
                    }
                }
                if (!dr) {
                    if (kr >= M) {
                        rmin = fmin(rmin, s_vv[M]);
                        dr = true;
                    } else {
                        const double b3 = bh3[kr >> 9], b2 = bh2[kr >> 6], b1 = s_bh[kr >> 3];
                        const double v3 = s_bvr[FL_B1 + FL_B2 + (kr >> 9)], v2 = s_bvr[FL_B1 + (kr >> 6)];
                        const double v1 = s_bvr[kr >> 3], vv = s_vv[kr], mh = s_mh[kr];
                        const bool c3 = (kr & 511) == 0 && kr + 511 < M && b3 <= hj;
                        const bool c2 = !c3 && (kr & 63) == 0 && kr + 63 < M && b2 <= hj;
                        const bool c1 = !c3 && !c2 && (kr & 7) == 0 && kr + 7 < M && b1 <= hj;
                        rmin = fmin(rmin, c3 ? v3 : (c2 ? v2 : (c1 ? v1 : vv)));
                        if (!(c3 || c2 || c1) && mh > hj) dr = true;
                        else kr += c3 ? 512 : (c2 ? 64 : (c1 ? 8 : 1));
                    }
                }
            }
            const double prom = hj - fmax(lmin, rmin);
            st_state(&s_st[j], thr <= prom ? ST_FINAL : ST_PREMOVED);
        }
    }
    __syncthreads();
    STAMP(4);

    /* (5) ordered compaction */
    int64_t *out = A.out + d0;
    int w = 0;
    for (int q0 = 0; q0 < M; q0 += FP_T) {
        const int j = q0 + tid;
        const bool keep = j < M && s_st[j] == ST_FINAL;
        int tot;
        const int off = block_scan_flag<FP_T>(keep, sh, &tot);
        if (keep) {
            out[w + off] = s_mp[j];
            if (A.outv) A.outv[d0 + w + off] = sg * s_mh[j];
        }
        w += tot;
    }
    if (tid == 0) {
        A.nout[f] = w;
        if (A.run_out) A.run_out[f] = w >= A.run_min ? 1 : 0;
        if (s_tie && A.flags) A.flags[f] |= A.tie_bit;
    }
    STAMP(5);
    STAMP_FLUSH(A.stamps);
}

}  // namespace bpmx
