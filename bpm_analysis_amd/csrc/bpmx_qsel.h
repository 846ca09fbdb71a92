/*
 * bpmx_qsel.h — the per-recording quantile select of k_quantile_reg
 * (np.quantile(env, q), 'linear': bpm_analysis.py:1067, :225, :1075, :1114)
 * as a device function over keys already held in registers, so that
 * k_hilbert_env can run it on the envelope it has just produced (no reload,
 * no launch) and k_quantile_reg on the envelope it loads.
 *
 * Item it of thread t is position it * QR_T + t.  Per level: MSD radix select
 * of rank floor((n-1)q) on the order-preserving keys (8-bit digits; digits
 * constant over the recording are taken from any key); once <= 64 keys are
 * left under the prefix they are gathered and the r-th is taken directly;
 * then the next order statistic and numpy's _lerp.
 */
#ifndef BPMX_QSEL_H
#define BPMX_QSEL_H

#include "bpmx_common.h"
#include "bpmx_kernels.h"

namespace bpmx {

/* workgroup scratch (LDS) of the select; ~3.7 KB */
struct QrShared {
    unsigned int hist[256];
    unsigned int hist0[256];       /* the first varying digit's histogram: the same for every level */
    long long r;
    int digit, csel, cc;
    unsigned long long ck[64];
    unsigned long long a[QR_T / 64], b[QR_T / 64];
    long long cnt[QR_T / 64];
};

/* every thread of the QR_T-thread workgroup calls this with its QR_IT keys
 * (positions >= n ignored); writes A.qv[f][slot] for every level */
__device__ __forceinline__ void qr_select(const uint64_t (&key)[QR_IT], int64_t n, const QuantArgs &A, int f,
                                          QrShared &S) {
    const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
    constexpr int NW = QR_T / 64;
    uint64_t kor = 0, kand = ~0ull;
#pragma unroll
    for (int it = 0; it < QR_IT; ++it) {
        const int64_t i = (int64_t)it * QR_T + tid;
        if (i < n) { kor |= key[it]; kand &= key[it]; }
    }
    for (int o = 32; o > 0; o >>= 1) {
        kor |= (uint64_t)__shfl_xor((long long)kor, o);
        kand &= (uint64_t)__shfl_xor((long long)kand, o);
    }
    if (lane == 0) { S.a[wid] = kor; S.b[wid] = kand; }
    __syncthreads();
    uint64_t vary, common;
    {
        uint64_t o = 0, a = ~0ull;
        for (int w = 0; w < NW; ++w) { o |= S.a[w]; a &= S.b[w]; }
        vary = o ^ a;
        common = a;                                          /* the bits every key shares */
    }
    __syncthreads();
    /* every level's first pass has no prefix yet: one histogram of the
     * highest varying digit serves them all */
    int shift0 = -1;
    for (int sh = 56; sh >= 0; sh -= 8)
        if ((vary >> sh) & 0xFFull) { shift0 = sh; break; }
    if (shift0 >= 0) {
        if (tid < 256) S.hist0[tid] = 0;
        __syncthreads();
#pragma unroll
        for (int it = 0; it < QR_IT; ++it) {
            const int64_t i = (int64_t)it * QR_T + tid;
            if (i < n) atomicAdd(&S.hist0[(key[it] >> shift0) & 255], 1u);
        }
        __syncthreads();
    }
    for (int l = 0; l < A.n_levels; ++l) {
        const double q = A.q[l];
        const double vi = (double)(n - 1) * q;
        const bool top = vi >= (double)(n - 1);
        const long long lo = top ? (long long)(n - 1) : (long long)floor(vi);
        uint64_t prefix = 0, mask = 0;
        long long r = lo;
        for (int shift = 56; shift >= 0; shift -= 8) {
            if (((vary >> shift) & 0xFFull) == 0) {          /* uniform: constant digit */
                prefix |= common & (0xFFull << shift);
                mask |= 0xFFull << shift;
                continue;
            }
            const unsigned int *hs = shift == shift0 ? S.hist0 : S.hist;   /* uniform */
            if (shift != shift0) {
                if (tid < 256) S.hist[tid] = 0;
                __syncthreads();
#pragma unroll
                for (int it = 0; it < QR_IT; ++it) {
                    const int64_t i = (int64_t)it * QR_T + tid;
                    if (i < n && (key[it] & mask) == prefix) atomicAdd(&S.hist[(key[it] >> shift) & 255], 1u);
                }
                __syncthreads();
            }
            if (wid == 0) {
                const unsigned int c0 = hs[lane * 4], c1 = hs[lane * 4 + 1], c2 = hs[lane * 4 + 2], c3 = hs[lane * 4 + 3];
                const long long sm = (long long)c0 + c1 + c2 + c3;
                long long incl = sm;
                for (int o = 1; o < 64; o <<= 1) {
                    const long long t = __shfl_up(incl, o);
                    if (lane >= o) incl += t;
                }
                const long long excl = incl - sm;
                if (excl <= r && r < incl) {
                    long long rr = r - excl;
                    const unsigned int cs[4] = {c0, c1, c2, c3};
                    int d = 0;
                    while (rr >= (long long)cs[d]) { rr -= cs[d]; ++d; }
                    S.digit = lane * 4 + d;
                    S.r = rr;
                    S.csel = (int)cs[d];
                }
                if (lane == 0) S.cc = 0;
            }
            __syncthreads();
            prefix |= (uint64_t)S.digit << shift;
            mask |= 0xFFull << shift;
            r = S.r;
            if (shift > 0 && S.csel <= 64) {
                /* few keys left under the prefix (after one or two digits on
                 * an envelope): gather them and take the r-th smallest directly
                 * instead of the remaining digit passes */
#pragma unroll
                for (int it = 0; it < QR_IT; ++it) {
                    const int64_t i = (int64_t)it * QR_T + tid;
                    if (i < n && (key[it] & mask) == prefix) S.ck[atomicAdd(&S.cc, 1)] = key[it];
                }
                __syncthreads();
                if (wid == 0) {
                    const int c = S.cc;
                    const unsigned long long mine = lane < c ? S.ck[lane] : ~0ull;
                    int below = 0, same = 0;
                    for (int j = 0; j < c; ++j) {
                        const unsigned long long o = S.ck[j];
                        below += o < mine;
                        same += o == mine;
                    }
                    if (lane < c && below <= r && r < below + same) S.ck[0] = mine;   /* all writers agree */
                }
                __syncthreads();
                prefix = S.ck[0];
                mask = ~0ull;
                __syncthreads();
                break;
            }
        }
        const double va = key_f64(prefix);
        double res = va;
        if (!top) {
            unsigned long long mn = ~0ull;
            long long cnt = 0;
#pragma unroll
            for (int it = 0; it < QR_IT; ++it) {
                const int64_t i = (int64_t)it * QR_T + tid;
                if (i < n) {
                    if (key[it] <= prefix) cnt++;
                    else if (key[it] < mn) mn = key[it];
                }
            }
            for (int o = 32; o > 0; o >>= 1) {
                const unsigned long long om = __shfl_xor(mn, o);
                mn = om < mn ? om : mn;
                cnt += __shfl_xor(cnt, o);
            }
            __syncthreads();
            if (lane == 0) { S.a[wid] = mn; S.cnt[wid] = cnt; }
            __syncthreads();
            unsigned long long m = S.a[0];
            long long c = 0;
            for (int w = 0; w < NW; ++w) { m = S.a[w] < m ? S.a[w] : m; c += S.cnt[w]; }
            const double vb = (c > lo + 1) ? va : key_f64(m);
            res = np_lerp(va, vb, vi - (double)lo);
        }
        if (tid < Q_SLOTS && ((A.slot[l] >> tid) & 1)) A.qv[(int64_t)f * Q_SLOTS + tid] = res;
        __syncthreads();
    }
}

}  // namespace bpmx

#endif
