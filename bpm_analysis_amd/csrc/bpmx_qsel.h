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

#include <type_traits>

#include "bpmx_common.h"
#include "bpmx_kernels.h"

namespace bpmx {

#ifdef BPMX_QS_STAMPS                  /* tools/hbench -DBPMX_QS_STAMPS: per-phase cycles of the select */
__device__ unsigned long long qs_dbg[8 * 4096];
#define QS_DECL unsigned long long qs_acc[8] = {0}, qs_t = __builtin_amdgcn_s_memtime();
#define QS_T(k)                                                                   \
    do {                                                                          \
        if (threadIdx.x == 0) {                                                   \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();           \
            qs_acc[k] += t_ - qs_t;                                               \
            qs_t = t_;                                                            \
        }                                                                         \
    } while (0)
#define QS_FLUSH()                                                                \
    do {                                                                          \
        if (threadIdx.x == 0)                                                     \
            for (int k_ = 0; k_ < 8; ++k_) qs_dbg[(blockIdx.x & 4095) * 8 + k_] = qs_acc[k_]; \
    } while (0)
#else
#define QS_DECL
#define QS_T(k) do {} while (0)
#define QS_FLUSH() do {} while (0)
#endif

/* workgroup scratch (LDS) of the select; ~18 KB */
struct alignas(16) QrShared {
    unsigned int hw[QR_T / 64][256];   /* per-wave digit histograms (no cross-wave atomics on one bin) */
    unsigned int hist0[256];       /* the first varying digit's histogram: the same for every level */
    long long r;
    int digit, csel, cc, nxt;
    unsigned long long ck[64];
    unsigned long long va, vb;
    unsigned long long a[QR_T / 64], b[QR_T / 64];
    long long cnt[QR_T / 64];
};

/* adds the wave's digits (dg < 0: none) to its own histogram row h.  A run
 * [s, e] of equal digits over consecutive lanes adds e + 1 - s as -s at its
 * first lane and e + 1 at its last (one atomic per lane that starts or ends a
 * run, none for the lanes inside; the row's sums are exact mod 2^32).  Item it
 * of the 64 lanes is 64 consecutive positions of a smooth envelope, so a wave
 * has a few runs per item.  No lane-mask arithmetic: two DPP moves, two
 * compares, one subtract.  Every lane must be active. */
__device__ __forceinline__ void qr_hist_add(unsigned int *h, int dg) {
    const int lane = lane_id();
    const int prev = __builtin_amdgcn_update_dpp(-2, dg, 0x138, 0xf, 0xf, false);   /* wave_shr:1, lane 0: -2 */
    const int next = __builtin_amdgcn_update_dpp(-2, dg, 0x130, 0xf, 0xf, false);   /* wave_shl:1, lane 63: -2 */
    const bool st = prev != dg, en = next != dg;
    if (dg >= 0 && (st || en)) atomicAdd(&h[dg], (unsigned int)((en ? lane + 1 : 0) - (st ? lane : 0)));
}

/* wave-wide OR / AND / unsigned min of a 64-bit value by DPP row shifts and
 * broadcasts (no LDS round trips), the result uniform.  Every lane active. */
template <int OP>   /* 0 OR, 1 AND, 2 MIN */
__device__ __forceinline__ uint64_t qr_wave_red64(uint64_t x) {
    const uint64_t id = OP == 0 ? 0ull : ~0ull;
    const int idl = (int)(uint32_t)id, idh = (int)(uint32_t)(id >> 32);
#define QR_DPP_STEP(ctrl, rmask)                                                                  \
    {                                                                                             \
        const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(idl, (int)(uint32_t)x, ctrl, rmask, 0xf, false); \
        const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(idh, (int)(uint32_t)(x >> 32), ctrl, rmask, 0xf, false); \
        const uint64_t t = ((uint64_t)hi << 32) | lo;                                             \
        x = OP == 0 ? (x | t) : OP == 1 ? (x & t) : (t < x ? t : x);                              \
    }
    QR_DPP_STEP(0x111, 0xf)   /* row_shr:1 */
    QR_DPP_STEP(0x112, 0xf)   /* row_shr:2 */
    QR_DPP_STEP(0x114, 0xf)   /* row_shr:4 */
    QR_DPP_STEP(0x118, 0xf)   /* row_shr:8 */
    QR_DPP_STEP(0x142, 0xa)   /* row_bcast:15 -> rows 1, 3 */
    QR_DPP_STEP(0x143, 0xc)   /* row_bcast:31 -> rows 2, 3 */
#undef QR_DPP_STEP
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 63);
    return ((uint64_t)hi << 32) | lo;
}

/* every thread of the QR_T-thread workgroup calls this with its QR_IT keys
 * (positions >= n ignored); writes A.qv[f][slot] for every level.
 * Per digit pass: each wave counts into its own histogram row (run-length
 * atomics), one barrier, wave 0 sums the rows, scans and picks the digit, one
 * barrier.  The (r+1)-th smallest comes from the gathered keys when it lies
 * under the same prefix (a final pass over all keys only when it does not).
 * (r05 form: one shared histogram, atomics per item, ds_bpermute reductions:
 * 45 K cycles per recording, most of it same-bin atomics from all waves and
 * LDS round trips of the reductions, tools/hbench HB_Q=1.) */
__device__ __forceinline__ void qr_select(const uint64_t (&key)[QR_IT], int64_t n, const QuantArgs &A, int f,
                                          QrShared &S) {
    const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
    constexpr int NW = QR_T / 64;
    QS_DECL
    uint64_t kor = 0, kand = ~0ull;
#pragma unroll
    for (int it = 0; it < QR_IT; ++it) {
        const int64_t i = (int64_t)it * QR_T + tid;
        if (i < n) { kor |= key[it]; kand &= key[it]; }
    }
    kor = qr_wave_red64<0>(kor);
    kand = qr_wave_red64<1>(kand);
    if (lane == 0) { S.a[wid] = kor; S.b[wid] = kand; }
    unsigned int *hrow = S.hw[wid];
    __syncthreads();
    uint64_t vary, common;
    {
        uint64_t o = 0, a = ~0ull;
        for (int w = 0; w < NW; ++w) { o |= S.a[w]; a &= S.b[w]; }
        vary = o ^ a;
        common = a;                                          /* the bits every key shares */
    }
    QS_T(0);
#if defined(QS_STOP) && QS_STOP == 1                             /* timing diagnostics (wrong outputs) */
    return;
#endif
    /* every level's first pass has no prefix yet: one histogram of the
     * highest varying digit serves them all */
    int shift0 = -1;
    for (int sh = 56; sh >= 0; sh -= 8)
        if ((vary >> sh) & 0xFFull) { shift0 = sh; break; }
    /* items with a position < n: this thread's count, and the wave-uniform
     * bound; copied opaquely into each item loop below, or the compiler hoists
     * the 24 per-item lane masks out of the level and digit loops into SGPRs
     * that spill */
    const int nvt = n > tid ? (int)((n - tid + QR_T - 1) / QR_T) : 0;
    const int nvu = __builtin_amdgcn_readfirstlane((int)((n + QR_T - 1) / QR_T));
    for (int l = 0; l < A.n_levels; ++l) {
        const double q = A.q[l];
        const double vi = (double)(n - 1) * q;
        const bool top = vi >= (double)(n - 1);
        const long long lo = top ? (long long)(n - 1) : (long long)floor(vi);
        uint64_t prefix = 0, mask = 0;
        long long r = lo, binsz = n;                         /* rank within the keys under the prefix, their count */
        bool gathered = false, have_b = top;
        uint64_t kb = 0;
        for (int shift = 56; shift >= 0; shift -= 8) {
            if (((vary >> shift) & 0xFFull) == 0) {          /* uniform: constant digit */
                prefix |= common & (0xFFull << shift);
                mask |= 0xFFull << shift;
                continue;
            }
            const bool first = shift == shift0;              /* uniform */
            if (!(first && l > 0)) {                         /* level 0's first pass made hist0 */
                reinterpret_cast<uint4 *>(hrow)[lane] = make_uint4(0u, 0u, 0u, 0u);   /* own row: no barrier */
                int nv = nvt, nu = nvu;
                asm volatile("" : "+v"(nv), "+s"(nu));
                /* on 32-bit halves: the prefix test as two masked compares,
                 * the digit as one bit-field extract */
                auto rfl = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); };   /* uniform values */
                uint32_t mh = rfl((uint32_t)(mask >> 32)), ml = rfl((uint32_t)mask);
                uint32_t ph = rfl((uint32_t)(prefix >> 32)), pl = rfl((uint32_t)prefix);
                uint32_t dsh = rfl((uint32_t)(shift & 31)), dhi = rfl(shift >= 32 ? 1u : 0u);
                asm volatile("" : "+s"(mh), "+s"(ml), "+s"(ph), "+s"(pl), "+s"(dsh), "+s"(dhi));
#pragma unroll
                for (int it = 0; it < QR_IT; ++it)
                    if (it < nu) {                           /* uniform */
                        const uint32_t kh = (uint32_t)(key[it] >> 32), kl = (uint32_t)key[it];
                        const bool ok = it < nv && (kh & mh) == ph && (kl & ml) == pl;
                        const int dg = (int)__builtin_amdgcn_ubfe(dhi ? kh : kl, dsh, 8u);
                        qr_hist_add(hrow, ok ? dg : -1);
                    }
                __syncthreads();
            }
            QS_T(2);
            if (wid == 0) {
                uint4 c4 = make_uint4(0u, 0u, 0u, 0u);
                if (first && l > 0) {
                    c4 = reinterpret_cast<const uint4 *>(S.hist0)[lane];
                } else {
#pragma unroll 4
                    for (int w = 0; w < NW; ++w) {                   /* (a full unroll keeps 16 uint4 live beside the keys) */
                        const uint4 h = reinterpret_cast<const uint4 *>(S.hw[w])[lane];
                        c4.x += h.x; c4.y += h.y; c4.z += h.z; c4.w += h.w;
                    }
                    if (first) reinterpret_cast<uint4 *>(S.hist0)[lane] = c4;
                }
                const int sm = (int)(c4.x + c4.y + c4.z + c4.w);   /* <= QR_MAX */
                const int incl = wave_iscan_dpp<false>(sm), excl = incl - sm;
                if (excl <= r && r < incl) {
                    long long rr = r - excl;
                    const unsigned int cs[4] = {c4.x, c4.y, c4.z, c4.w};
                    int d = 0;
                    while (rr >= (long long)cs[d]) { rr -= cs[d]; ++d; }
                    S.digit = lane * 4 + d;
                    S.r = rr;
                    S.csel = (int)cs[d];
                }
                if (lane == 0) S.cc = 0;
            }
            __syncthreads();
            QS_T(3);
#if defined(QS_STOP) && QS_STOP == 2
            return;
#endif
            prefix |= (uint64_t)S.digit << shift;
            mask |= 0xFFull << shift;
            r = S.r;
            binsz = S.csel;
            if (shift > 0 && binsz <= 64) {
                /* few keys left under the prefix (after one or two digits on
                 * an envelope): gather them and take the r-th and (r+1)-th
                 * smallest directly instead of the remaining digit passes */
                int nv = nvt;
                asm volatile("" : "+v"(nv));
#pragma unroll
                for (int it = 0; it < QR_IT; ++it)
                    if (it < nv && (key[it] & mask) == prefix) S.ck[atomicAdd(&S.cc, 1)] = key[it];
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
                    if (lane < c && below <= r && r < below + same) S.va = mine;        /* all writers agree */
                    if (lane < c && below <= r + 1 && r + 1 < below + same) S.vb = mine;
                }
                __syncthreads();
#if defined(QS_STOP) && QS_STOP == 3
                return;
#endif
                prefix = S.va;
                mask = ~0ull;
                gathered = true;
                if (!top && r + 1 < binsz) { kb = S.vb; have_b = true; }
                QS_T(4);
                break;
            }
        }
        if (!gathered && !top && r + 1 < binsz) {           /* every key under the full prefix is this one */
            kb = prefix;
            have_b = true;
        }
        const double va = key_f64(prefix);
        double res = va;
        if (!top) {
            if (!have_b) {                                   /* the (r+1)-th is the smallest key above the prefix */
                unsigned long long mn = ~0ull;
                int nv = nvt;
                asm volatile("" : "+v"(nv));
#pragma unroll
                for (int it = 0; it < QR_IT; ++it)
                    if (it < nv && key[it] > prefix && key[it] < mn) mn = key[it];
                mn = qr_wave_red64<2>(mn);
                if (lane == 0) S.a[wid] = mn;
                __syncthreads();
                unsigned long long m = S.a[0];
                for (int w = 1; w < NW; ++w) m = S.a[w] < m ? S.a[w] : m;
                kb = m;
            }
            res = np_lerp(va, key_f64(kb), vi - (double)lo);
        }
        {
            int ts = tid;                                    /* the store address formed here, not hoisted and spilled */
            asm volatile("" : "+v"(ts));
            if (ts < Q_SLOTS && ((A.slot[l] >> ts) & 1)) A.qv[(int64_t)f * Q_SLOTS + ts] = res;
        }
        __syncthreads();
        QS_T(5);
    }
    QS_FLUSH();
}

}  // namespace bpmx

#endif
