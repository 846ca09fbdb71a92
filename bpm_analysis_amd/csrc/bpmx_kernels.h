/*
 * bpmx_kernels.h — kernel argument blocks and launch declarations.
 */
#ifndef BPMX_KERNELS_H
#define BPMX_KERNELS_H

#include "bpmx_common.h"

namespace bpmx {

/* per-file quantile slots in the qv[F][4] table */
enum { Q_TROUGH = 0, Q_PEAK = 1, Q_NOISE = 2, Q_FALLBACK = 3, Q_SLOTS = 4 };

/* A run's per-recording outputs and counters, reset before its stages: by
 * k_init_out, or (native runs with an envelope stage) by k_native_carry's
 * workgroup for its recording, which saves that launch.  Null pointers are
 * skipped; flags == null: nothing to do. */
struct InitOutArgs {
    const int32_t *active;
    int32_t *flags, *ntr, *npk, *runs, *nraw;
    int32_t *z1;           /* draft exact masks (one int per recording) */
    int32_t *z2;           /* draft undecided counters nund[f], nund[F + f] */
    int32_t *z3;           /* find_peaks' scan record: none yet in this run */
    int32_t n_files;
};
__device__ __forceinline__ void init_out_one(const InitOutArgs &I, int f) {
    const int F = I.n_files;
    I.flags[f] = I.active[f] ? 0 : BPMX_F_TOO_SHORT;
    if (I.ntr) I.ntr[f] = 0;
    if (I.npk) I.npk[f] = 0;
    for (int k = 0; k < 5; ++k) I.runs[(int64_t)k * F + f] = 0;
    if (I.nraw) I.nraw[f] = 0;
    if (I.z1) I.z1[f] = 0;
    if (I.z2) { I.z2[f] = 0; I.z2[F + f] = 0; }
    if (I.z3) I.z3[f] = 0;
}

struct EnvRefArgs {
    const void *pcm;
    const int64_t *foff;   /* [F+1] frame offsets */
    const int64_t *doff;   /* [F+1] decimated offsets */
    const int32_t *active; /* [F] */
    int32_t n_files, dtype, channels, ds, env_window;
    double b[5], a[5], zi[4];
    double *scratch;       /* interleaved [(maxNd+30) * F] */
    double *env;           /* [sumNd] */
    double *y;             /* [sumNd] or null */
    double *sums;          /* interleaved [maxNd * F]: the rolling sum after each step (chain mode), or null */
    int32_t *chain;        /* [F]: 1 = env left to k_ref_env_mean (chain mode), 0 = written in the pass */
    int64_t pick_r0;       /* k_ref_pick: first row of this launch's rows */
    /* split forward pass (k_ref_fwd over row chunks while later chunks are
     * picked on a side stream): rows [fwd_rb, fwd_re) and the DF2T state
     * [F][4] between chunks; fwd_z null: k_envelope_ref_t runs the forward pass */
    int64_t fwd_rb, fwd_re;
    double *fwd_z;
    /* chunked Kahan pass (chain mode): k_envelope_ref_t runs steps [0,
     * kahan_ie), k_ref_kahan [kahan_ib, kahan_ie), the RollMean state [F][6]
     * in kahan_z (null: one pass); k_ref_env_mean forms rows from mean_r0 */
    double *kahan_z;
    int64_t kahan_ib, kahan_ie, mean_r0;
#ifdef BPMX_STAMPS
    unsigned long long *stamps;
#endif
};
template <bool WANT_Y>
__global__ void k_ref_env_mean(EnvRefArgs A);
template <bool ZB>
__global__ void k_ref_fwd(EnvRefArgs A);
__global__ void k_ref_kahan(EnvRefArgs A);
constexpr int64_t REF_FWD_ROWS = 1024;   /* first forward chunk's rows, doubling per chunk (multiples of the prefetch block) */

struct QuantArgs {
    const double *env;
    const int64_t *doff;
    const int32_t *active;
    int32_t n_files, n_levels;
    int32_t slot[Q_SLOTS];  /* bitmask of the qv slots level l fills */
    double q[Q_SLOTS];
    double *qv;             /* [F][Q_SLOTS] */
    int64_t skip_le;        /* k_ql_*: files with n <= skip_le are done by k_quantile_reg */
    const int32_t *skip;    /* [F] optional: skip files with skip[f] != 0 (the lazy static-floor level) */
    int32_t stats;          /* k_quantile_reg: also write the block max/min tables */
};

/* k_quantile for long recordings over many workgroups (k_detect.hip):
 * MSD radix select with 11-bit digits (6 passes over the 64-bit keys), each
 * pass a histogram of every chunk of the recording (all levels at once) into
 * global bins, then a select step per (recording, level) */
constexpr int QL_BITS = 11, QL_BINS = 1 << QL_BITS, QL_PASSES = 6, QL_CHUNK = 32768;
struct QlState {
    unsigned long long prefix, mask;
    long long r;            /* rank still to find inside the selected bin */
    long long lo;           /* the order statistic's rank (floor((n-1) q)) */
    unsigned long long next; /* min key above the answer (atomicMin), for the interpolation */
    int32_t top, eq;        /* top: q (n-1) >= n-1; eq: another key equals the answer */
};
struct QlArgs {
    QuantArgs Q;
    QlState *st;            /* [F][Q_SLOTS] */
    unsigned int *hist;     /* [QL_PASSES][F][Q_SLOTS][QL_BINS] (zeroed before pass 0) */
    int32_t pass;
};
/* The same quantiles in five launches and two passes over env (k_detect.hip,
 * r06): bins of the order-preserving key over the recording's own key range
 * (k_qv_range, from the block max/min tables), one histogram for all levels
 * (k_qv_hist), the target bin and the rank inside it per level (k_qv_select),
 * the target bin's keys gathered per level plus the least key above it
 * (k_qv_collect), the exact order statistics among the gathered keys by a
 * radix select and numpy's _lerp (k_qv_final). */
constexpr int QV_BITS = 13, QV_BINS = 1 << QV_BITS, QV_CHUNK = 32768;
struct QvRange {
    unsigned long long kmin;
    int32_t shift, pad;
};
struct QvState {
    long long lo;                 /* the order statistic's rank floor((n - 1) q) */
    long long r;                  /* its rank inside the target bin */
    unsigned long long next;      /* least key in a bin above the target (atomicMin) */
    int32_t bin, top;             /* target bin; q reaches n - 1 */
    uint32_t cnt, cbin;           /* keys gathered; the target bin's count */
};
struct QvArgs {
    QuantArgs Q;
    const int64_t *boff;          /* block-table offsets (k_block_stats) */
    const double *bmax, *bmin;
    QvRange *rg;                  /* [F] */
    QvState *st;                  /* [F][Q_SLOTS] */
    unsigned int *hist;           /* [F][QV_BINS] (zeroed) */
    unsigned long long *cand;     /* level l of recording f at (doff[f] * Q_SLOTS + l * n_f): room for every key */
};
__global__ void k_qv_range(QvArgs A);
__global__ void k_qv_hist(QvArgs A);
__global__ void k_qv_select(QvArgs A);
__global__ void k_qv_collect(QvArgs A);
__global__ void k_qv_final(QvArgs A);
__global__ void k_ql_init(QlArgs A);
__global__ void k_ql_hist(QlArgs A);
__global__ void k_ql_select(QlArgs A);
__global__ void k_ql_next(QlArgs A);
__global__ void k_ql_final(QlArgs A);

struct BlockStatArgs {
    const double *env;
    const int64_t *doff;
    const int64_t *boff;   /* [F+1] offsets of 64-sample block tables */
    const int32_t *active;
    int32_t n_files;
    double *bmax, *bmin;
    int64_t skip_le;        /* k_block_stats: files with n <= skip_le are done by k_quantile_reg */
};

/* one workgroup per recording with all of env in registers (n <= QR_MAX):
 * every radix-select pass and the block max/min tables from one HBM read */
constexpr int QR_T = 1024;
constexpr int QR_IT = 24;
constexpr int64_t QR_MAX = (int64_t)QR_T * QR_IT;

struct PeakArgs {
    const double *env;
    const double *height;  /* per-sample minimum height or null (same indexing as env) */
    const int64_t *doff, *boff;
    const int32_t *active;
    const double *bmax, *bmin;
    const double *qv;
    int32_t qslot;
    int32_t n_files;
    int32_t distance;
    double sign;           /* +1: find_peaks(env), -1: find_peaks(-env) */
    int32_t *cand;         /* scratch [sumNd] */
    uint8_t *state;        /* scratch [sumNd] */
    int64_t *out;          /* [sumNd] */
    double *outv = nullptr;  /* optional [sumNd]: env at each output index (sign removed), beside out */
    int32_t *nout;         /* [F] */
    int32_t *run_out;      /* optional [F]: 1 if nout >= run_min */
    int32_t run_min;
    int32_t *vcand;        /* k_find_peaks_lds: scratch [sumNd], valley positions */
    double *cval, *vval;   /* k_find_peaks_lds: scratch [sumNd], the values of cand / vcand's extrema */
    int32_t *fallback;     /* k_find_peaks_lds: [F] out, 1 = too many maxima for LDS (k_find_peaks takes it) */
    const int32_t *only;   /* k_find_peaks / k_fpl_*: [F] or null, process only recordings with only[f] != 0 */
    int64_t lds_nmax;      /* k_find_peaks_lds: hand recordings longer than this over (fallback = 1) */
    int32_t *flags;        /* [F] per-file flags: tie_bit is OR'd in when the distance filter met a decisive tie */
    int32_t tie_bit;       /* BPMX_F_TROUGH_TIE or BPMX_F_PEAK_TIE */
    /* the run's extrema scan record (bpmx_fpscan.h): ok[f] = +1 / -1 when
     * the trough launch of k_find_peaks_lds (the only writer) left the lists
     * in cand / vcand (made for x = +env / -env), 0 = scan here (and record);
     * null: no record */
    int32_t *scan_ok = nullptr;    /* [F] */
    int32_t *scan_cnt = nullptr;   /* [F][FPS_NW][2] */
    /* bpmx_run_ordered (k_find_peaks only): candidate export and the caller's
     * visiting ranks (include/bpmx.h bpmx_peak_order) */
    int32_t *cand_out = nullptr;   /* [sumNd] or null */
    int32_t *ncand_out = nullptr;  /* [F] */
    const int32_t *rank = nullptr; /* [sumNd] or null */
    const int32_t *use_rank = nullptr;  /* [F] */
    int32_t ordered_bit = 0;       /* BPMX_F_TROUGH_ORDERED or BPMX_F_PEAK_ORDERED */
#ifdef BPMX_STAMPS
    unsigned long long *stamps;
#endif
};

/* find_peaks candidate states (k_find_peaks, k_find_peaks_lds, k_fpl_*).
 * Every state a candidate reaches after the distance filter kept it is odd
 * (KEPT, then FINAL or PREMOVED by the prominence threshold), so the decisive-
 * tie check (st_kept_by_distance) reads the distance outcome while other
 * threads are already overwriting it with the prominence outcome.  REMOVED is
 * reserved for the distance filter's removals; the height filter has its own. */
enum { ST_UNDECIDED = 0, ST_KEPT = 1, ST_REMOVED = 2, ST_FINAL = 3, ST_HEIGHT = 4, ST_PREMOVED = 5 };
__device__ __forceinline__ bool st_kept_by_distance(uint8_t s) { return (s & 1u) != 0; }

__device__ __forceinline__ uint8_t ld_state(const uint8_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void st_state(uint8_t *p, uint8_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

constexpr int FL_MC = 3072;          /* k_find_peaks_lds: local maxima held in LDS */

/* find_peaks for long recordings (k_peaks_long.hip): the local-extrema
 * formulation of k_find_peaks_lds with the extrema in global scratch and the
 * per-sample and per-maximum phases spread over many workgroups */
constexpr int FPL_U = 1024;          /* positions per scan unit (one wave) */
constexpr int64_t FPL_NMIN = 65536;  /* recordings longer than this take the k_fpl_* path */
struct FplArgs {
    int32_t nu;            /* scan units per recording (max over the batch) */
    int32_t *cnt;          /* [F][nu][2] maxima / valley counts per unit, then (k_fpl_place) maxima offsets */
    int32_t *mtot;         /* [F] local maxima per recording */
    int32_t *mp;           /* [sumNd] maxima positions (dense per recording at doff) */
    double *mh;            /* [sumNd] maxima values (sign applied) */
    double *vv;            /* [sumNd + F] gap valleys: vv[g] = valley between maxima g-1 and g */
    double *b32h, *b32l, *b32r;    /* per 32 maxima: max height, min vv[k+1], min vv[k] */
    double *b1kh, *b1kl, *b1kr;    /* per 1024 maxima: the same */
    int32_t *dfail;        /* [F] k_fpl_dist_ch could not cut the recording's maxima into chunks (k_fpl_distance decides it) */
    int32_t dchunk;        /* k_fpl_dist_ch ran (1): k_fpl_distance only decides recordings with dfail set */
};
/* k_fpl_dist_ch: the distance rounds of a long recording in chunks of about
 * FPC_S maxima, cut where consecutive maxima lie >= distance apart (no
 * candidate has a neighbour across the cut), a chunk reaching at most FPC_H
 * maxima past its nominal end */
constexpr int FPC_T = 256, FPC_S = 1024, FPC_H = 1024, FPC_R = (FPC_S + FPC_H) / FPC_T;
__host__ __device__ inline int64_t fpl_b32_off(int64_t d0, int f) { return (d0 >> 5) + 4 * (int64_t)f; }
__host__ __device__ inline int64_t fpl_b1k_off(int64_t d0, int f) { return (d0 >> 10) + 4 * (int64_t)f; }
__global__ void k_fpl_scan(PeakArgs A, FplArgs L);
__global__ void k_fpl_place(PeakArgs A, FplArgs L);
__global__ void k_fpl_fill(PeakArgs A, FplArgs L);
__global__ void k_fpl_distance(PeakArgs A, FplArgs L);
__global__ void k_fpl_dist_ch(PeakArgs A, FplArgs L);
__global__ void k_fpl_prom(PeakArgs A, FplArgs L);
__global__ void k_fpl_compact(PeakArgs A, FplArgs L);

struct InterpArgs {
    const double *env;
    const int64_t *doff;
    const int64_t *troughs;  /* per-file slices at doff */
    const int32_t *ntr;
    const int32_t *run;      /* [F] files to process */
    int32_t n_files;
    double *dense;
    int64_t skip_n;          /* skip files with n <= skip_n and <= WM_TRMAX troughs (k_rollq_wm interpolates) */
    int64_t skip_gt;         /* skip files with n > skip_gt (the chunked k_rollq_wm interpolates those) */
};

struct RollqArgs {
    const double *dense;
    const int64_t *doff;
    const int64_t *troughs;  /* first trough = first non-NaN dense sample */
    const int32_t *run;
    int32_t n_files, window, min_periods, cap;
    double q;
    double *out;
    int32_t *allnan;         /* [F] */
    int32_t wm_max;          /* k_rolling_quantile skips files with n <= wm_max (k_rollq_wm took them) */
    const double *env;       /* k_rollq_wm: interpolate dense from env at the troughs itself ... */
    const double *tv;        /* ... taken from tv (env at each trough, beside troughs; required with env) */
    const int32_t *ntr;      /* ... when the file has <= WM_TRMAX of them (else read dense) */
    int64_t chunk;           /* k_rolling_quantile: outputs per workgroup (blockIdx.y = chunk of the file) */
    int32_t *vfirst, *vlast; /* [F] first / last valid output over all chunks (k_rollq_fill reads them) */
    double *gv;              /* k_rolling_quantile_g: per-workgroup union scratch, 2 x gcap values ... */
    int32_t *gp;             /* ... and 2 x gcap positions */
    int64_t gcap;
    /* k_rollq_wm_t<true> over chunks of long recordings (n > WM_MMAX): wm_chunk
     * outputs per workgroup (blockIdx.y = chunk, 0 = off), each chunk's kept
     * positions in wm_pos_ch (WM_PMAX per chunk); a chunk it cannot take sets
     * wm_fail[f] and the recording goes to k_rolling_quantile */
    int32_t wm_chunk;
    int32_t *wm_fail;
    uint16_t *wm_pos_ch;
#ifdef BPMX_STAMPS
    unsigned long long *stamps;
#endif
};

struct SanitizeArgs {
    const double *env, *draft;
    const int64_t *doff;
    const int32_t *active;
    const int64_t *raw;      /* raw troughs (slices at doff) */
    const double *rawv;      /* env at the raw troughs (find_peaks' outv), beside raw */
    const int32_t *nraw;
    int32_t n_files;
    double mult;
    double *outv;            /* env at the kept troughs, beside out */
    int64_t *out;
    int32_t *nout;
    int32_t *flags;
    int32_t *run2;           /* [F] files that need the second floor pass */
    const uint8_t *dec;      /* [raw trough j at doff + j] keep decision of k_draft_bounds (nullptr: use draft) */
    const int32_t *exact;    /* [F] 1: draft computed in full, decide from it instead */
    int32_t *run_fb;         /* [F] out: draft floor kept (<= 2 troughs) but only bounded: compute it in full */
};

/* sanitize (bpm_analysis.py:1088-1099) of recording f by its NT-thread
 * workgroup: keep raw trough t iff env[t] <= mult * draft[t] (from the draft,
 * or from k_draft_bounds' decisions), ordered, with their env values; < 5 raw
 * troughs: all of them, BPMX_F_STATIC_FLOOR.  Returns the kept count to every
 * thread.  k_sanitize, and k_floor_wm's workgroups (k_rollq_wm.hip). */
template <int NT>
__device__ __forceinline__ int sanitize_wg(const SanitizeArgs &A, int f, int *sh) {
    const int64_t d0 = A.doff[f];
    const int64_t *raw = A.raw + d0;
    int64_t *out = A.out + d0;
    const int m = A.nraw[f];
    const int tid = threadIdx.x;
    const double *rawv = A.rawv + d0;
    double *outv = A.outv + d0;
    if (m < 5) {
        for (int j = tid; j < m; j += NT) { out[j] = raw[j]; outv[j] = rawv[j]; }
        if (tid == 0) {
            A.nout[f] = m;
            A.flags[f] |= BPMX_F_STATIC_FLOOR;
            if (A.run2) A.run2[f] = 0;
        }
        return m;
    }
    const double *draft = A.draft + d0;
    const bool exact = !A.dec || A.exact[f];
    int w = 0;
    for (int c0 = 0; c0 < m; c0 += NT) {
        const int j = c0 + tid;
        bool keep = false;
        int64_t t = 0;
        double tv = 0.0;
        if (j < m) {
            t = raw[j];
            tv = rawv[j];                                    /* env[t] */
            if (exact) {
                const double fl = draft[t];
                keep = (fl == fl) && tv <= A.mult * fl;
            } else {
                keep = A.dec[d0 + j] == 1;
            }
        }
        int tot;
        const int off = block_scan_flag<NT>(keep, sh, &tot);
        if (keep) { out[w + off] = t; outv[w + off] = tv; }
        w += tot;
    }
    if (tid == 0) {
        A.nout[f] = w;
        if (w <= 2) A.flags[f] |= BPMX_F_DRAFT_FLOOR;
        if (A.run2) A.run2[f] = w > 2 ? 1 : 0;
        if (A.run_fb) A.run_fb[f] = (w <= 2 && !exact) ? 1 : 0;
    }
    return w;
}

/* k_floor_wm (k_rollq_wm.hip): the floor stage after the draft bracket in one
 * workgroup per recording (recordings of <= WM_MMAX decimated samples) */
struct FloorWmArgs {
    RollqArgs rq;              /* the rolling-quantile settings; troughs / tv / ntr / out / allnan / run set per call */
    SanitizeArgs sa;           /* raw troughs and values, draft, decisions -> kept troughs, values, counts, flags */
    const int32_t *exact;      /* [F] the draft floor in full here (the bracket left it open) */
    const double *qv;          /* [F][Q_SLOTS] */
    QuantArgs qn;              /* n_levels 1: the static floor's level, selected here (lazy); 0: in qv already */
    double *floor, *draft;     /* draft: the same buffer as sa.draft */
    int32_t *an_draft, *an_final;   /* [F] all-NaN results of the draft / final rolling quantiles */
    int32_t *full;             /* [F] scratch of the pruned / unpruned decision */
};

/* k_draft_bounds: the draft floor (first rolling quantile) is read only at the
 * raw troughs (sanitize) unless <= 2 troughs survive.  Its dense input is
 * piecewise linear between the troughs, so every window's k-th smallest value
 * is bracketed by weighted order statistics of the segments' end values;
 * most troughs' keep decision follows from the bracket alone. */
struct DraftBoundArgs {
    const double *env;
    const int64_t *doff;
    const int64_t *raw;      /* raw troughs */
    const double *rawv;      /* env at the raw troughs (find_peaks' outv), beside raw: no gathers from env */
    const int32_t *nraw;
    const int32_t *run;      /* [F] files with >= 5 raw troughs */
    int32_t n_files, window, min_periods;
    double q, mult;
    uint8_t *dec;            /* [doff + j]: 1 keep, 0 reject (2 while undecided, then resolved by draft_point) */
    int32_t *exact;          /* [F] out: 1 = needs the full draft (all-NaN draft, too many troughs, a window
                                draft_point does not take) */
    int32_t local_m;         /* more troughs than this: rank segments per window (DB_LOCAL_M) */
    int64_t *stats;          /* optional (BPMX_OPT_STATS): += raw troughs, undecided troughs, chunks sent to the
                                full draft by draft_point */
    int32_t *vfl;            /* [F][2] k_draft_bounds out: first / last valid draft output (k_draft_points) */
    int32_t *nund;           /* [2F] zeroed before k_draft_bounds: undecided troughs per recording, then the
                                ones k_draft_points<1> leaves to the [wide] launch */
};
/* k_draft_points: the undecided troughs of DP_CHUNK consecutive raw troughs per
 * workgroup, one wave per trough */
constexpr int DP_CHUNK = 32;
constexpr int DB_T = 256;
constexpr int DB_TRMAX = 2040;   /* troughs per recording staged in LDS (k_draft_bounds: four workgroups per CU) */
constexpr int DB_LOCAL_M = 512;  /* more troughs than this: per-window ranking instead of the global order */
struct DbSeg {                   /* a trough-curve segment [s, e) and one of its end values */
    int32_t s, e;
    double v;
};

struct FinalArgs {
    const double *draft;
    const int64_t *doff;
    const int32_t *active;
    const double *qv;
    const int32_t *allnan_draft, *allnan_final;
    int32_t n_files;
    double *floor;
    int32_t *flags;
};

/* dynamic LDS bytes of k_rolling_quantile<T,...> for a union capacity `cap`
 * (multiple of 64, >= W+T-1): Av f64[cap]; nsv f64[T]; runv f64[T] (later the
 * edge list); Ap u16[cap]; nsp,ubv u16[T]; rpref int[T+1] (later the edge-word
 * prefix, needs cap/64+2 <= T+1); scan scratch int[T/64+2].
 * 39.4 KB at W=3020, T=256: four workgroups per CU. */
__host__ __device__ inline size_t rollq_lds_bytes(int T, int cap) {
    return (size_t)cap * 10 + (size_t)T * 20 + ((size_t)T + 1) * 4 + ((size_t)T / 64 + 2) * 4;
}
constexpr int RQ_T = 256;   /* outputs per tile = threads per workgroup */

template <int DT, bool MULTI, bool ZB>
__global__ void k_envelope_ref_t(EnvRefArgs A);
template <int DT, bool MULTI>
__global__ void k_ref_pick(EnvRefArgs A);
__global__ void k_quantile_reg(QuantArgs A, BlockStatArgs B);
__global__ void k_block_stats(BlockStatArgs A);
__global__ void k_find_peaks(PeakArgs A);
__global__ void k_find_peaks_lds(PeakArgs A);
__global__ void k_interp(InterpArgs A);
__global__ void k_sanitize(SanitizeArgs A);
__global__ void k_draft_bounds(DraftBoundArgs A);
template <int SPL>
__global__ void k_draft_points(DraftBoundArgs A);
__global__ void k_floor_final(FinalArgs A);
template <int T, int RQ_MAXCH>
__global__ void k_rolling_quantile(RollqArgs A);
template <int T>
__global__ void k_rolling_quantile_g(RollqArgs A);
/* dynamic LDS of k_rolling_quantile_g<T> for a union capacity gcap */
__host__ __device__ inline size_t rollq_g_lds_bytes(int T, int64_t gcap) {
    return (size_t)T * 16 + (size_t)T * 8 + ((size_t)T + 1) * 4 + ((size_t)T / 64 + 2) * 4 + (size_t)T * 16 +
           ((size_t)(gcap / 64) + 2) * 4;
}
__global__ void k_rollq_fill(RollqArgs A);

/* wavelet-matrix rolling quantile (k_rollq_wm.hip): one 1024-thread workgroup
 * per recording of <= WM_MMAX decimated samples */
constexpr int WM_T = 1024;
constexpr int WM_ITEMS = 18;                 /* 16-bit positions; LDS ~156 KB at the maximum */
constexpr int WM_MMAX = WM_T * WM_ITEMS;     /* 18432 decimated samples (61 s at 302 Hz) */
constexpr int WM_TRMAX = 512;                /* troughs staged in LDS for the in-kernel interpolation */
constexpr int WM_PMAX = 12288;               /* kept samples of the pruned variant */
/* per-wave output-block scratch of k_rollq_wm_t (32-bit words): collected
 * members (16 lanes need at most 15 + 30 + 30 + 2: k spread + low-count
 * spread + excluded members + two; a block of 64 that needs more than fits
 * runs as four passes of 16), then as many partial-member records.  Small,
 * so that the sorted values fit beside it up to ~8000 kept samples. */
constexpr int WM_DCAP = 96;
constexpr int WM_WSCR = WM_DCAP;              /* per-wave scratch of the output phase: the collected ranks */
/* dynamic LDS of k_rollq_wm_t: trough tables | (pruned) kept masks, prefix,
 * bins | (pruned) kept positions | phase area (histogram / sort / matrix) */
struct WmLayout {
    size_t tab, meta, kpos, area, total;
};
/* pruned variant's per-64 tables (NBK entries each): upper side mask 8, prefix
 * 4, thr 1, b* levels 9; lower side (8-aligned) the same with a* levels */
constexpr int WM_NBK = WM_MMAX / 64 + 2;
constexpr int WM_META_LOW = (WM_NBK * 22 + 7) & ~7;
constexpr int WM_META_B = WM_META_LOW + WM_NBK * 22;
__host__ __device__ inline size_t wm_align16(size_t x) { return (x + 15) & ~(size_t)15; }
__host__ __device__ inline WmLayout wm_layout(int64_t nmax, bool prune) {
    const int64_t n = nmax < 1 ? 1 : (nmax > WM_MMAX ? WM_MMAX : nmax);
    const int64_t m = prune && n > WM_PMAX ? WM_PMAX : n;
    const int64_t L = m > 1 ? 64 - __builtin_clzll((unsigned long long)(m - 1)) : 1;
    const int64_t NW = (m + 63) / 64;
    const int64_t m8 = (m + 7) & ~7LL;
    const int64_t NBK = WM_MMAX / 64 + 2;                              /* per-64 tables */
    const int64_t sort_b = 8 * m8 + (int64_t)(WM_T / 64) * 128 * 4;   /* pos x2, key halves, counters */
    const int64_t wm_b = ((4 * m8 + 15) & ~15LL) + (int64_t)(WM_T / 64) * WM_WSCR * 4;   /* index arrays, block scratch */
    (void)L; (void)NW;
    const int64_t hist_b = prune ? NBK * 64 * 2 + (int64_t)(WM_T / 64) * 64 * 4 + n : 0;   /* + bin per sample */
    int64_t area = sort_b > wm_b ? sort_b : wm_b;
    area = area > hist_b ? area : hist_b;
    WmLayout l;
    l.tab = 0;
    l.meta = wm_align16((size_t)WM_TRMAX * (prune ? 20 : 12) + (size_t)NBK * 4);
    l.kpos = wm_align16(l.meta + (prune ? (size_t)WM_META_B : 0));
    l.area = wm_align16(l.kpos + (prune ? (size_t)m * 2 : 0));
    l.total = l.area + (size_t)area;
    return l;
}
template <bool PRUNE>
__global__ void k_rollq_wm_t(RollqArgs A, uint16_t *pos_scratch, int32_t *full);
__global__ void k_floor_wm(FloorWmArgs A);

}  // namespace bpmx

#endif
