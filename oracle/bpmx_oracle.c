/*
 * bpmx_oracle.c — CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in bpm_analysis_amd/ links, loads or
 * calls this file; it is used by tests/, by __graft_entry__.smoke() as the
 * checker, and by bench.py's cpu_baseline leg (kind "port").
 *
 * It restates, sequentially and in the same floating-point operation order,
 * what the reference computes in pixeru/bpm_analysis (snapshot 2025-07-25):
 *   bpm_analysis.py:1007-1062  preprocess_audio
 *   bpm_analysis.py:1064-1117  _calculate_dynamic_noise_floor
 *   bpm_analysis.py:223-229    PeakClassifier._find_raw_peaks
 * and the third-party routines those lines execute (scipy 1.15.3, numpy 2.2.6,
 * pandas 2.3.3; the reference pins no versions — SURVEY.md §8(c)).  Each
 * function below cites the line it follows.  Pinned against the reference in
 * tests/test_oracle.py through the golden vectors in tests/golden/ (generated
 * by importing the reference in the build container: tests/golden/make_goldens.py)
 * and the vulpine known-answer test.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off; no FMA contraction).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../bpm_analysis_amd/csrc/bpmx_synth.h"

enum { DT_U8 = 0, DT_I16 = 1, DT_I32 = 2, DT_F32 = 3, DT_F64 = 4 };

/* ------------------------------------------------------------------------ */
/* Synthetic input (same header the device generator uses).                  */
/* ------------------------------------------------------------------------ */
int bpmo_synth(uint64_t seed, int64_t n_frames, int32_t fs, int channels, int16_t *out) {
    int cap = (int)(n_frames / (fs / 4 > 0 ? fs / 4 : 1)) + 16;
    int64_t *s1 = (int64_t *)malloc(sizeof(int64_t) * cap);
    int64_t *s2 = (int64_t *)malloc(sizeof(int64_t) * cap);
    int nb = bpmx_synth_beats(seed, n_frames, fs, s1, s2, cap);
    for (int64_t n = 0; n < n_frames; ++n)
        for (int c = 0; c < channels; ++c)
            out[n * channels + c] = bpmx_synth_sample(seed, c, n, fs, s1, s2, nb);
    free(s1);
    free(s2);
    return nb;
}

/* ------------------------------------------------------------------------ */
/* A1/A2: ingest, channel mean, stride pick                                  */
/* bpm_analysis.py:1014-1016 (wavfile.read, np.mean(axis=1)), :1031-1036     */
/* Mono keeps its dtype; C>1 integer -> f64 mean, C>1 float32 -> f32 mean.   */
/* The picked samples are returned as doubles together with the dtype the    */
/* reference would hold them in, which decides the pad arithmetic (A4).      */
/* ------------------------------------------------------------------------ */
static double load_sample(const void *pcm, int dtype, int64_t idx) {
    switch (dtype) {
    case DT_U8: return (double)((const uint8_t *)pcm)[idx];
    case DT_I16: return (double)((const int16_t *)pcm)[idx];
    case DT_I32: return (double)((const int32_t *)pcm)[idx];
    case DT_F32: return (double)((const float *)pcm)[idx];
    default: return ((const double *)pcm)[idx];
    }
}

/* working dtype of x after the channel mean (numpy promotion rules) */
static int work_dtype(int dtype, int channels) {
    if (channels <= 1) return dtype;
    return dtype == DT_F32 ? DT_F32 : DT_F64;
}

static double frame_value(const void *pcm, int dtype, int channels, int64_t frame) {
    if (channels <= 1) return load_sample(pcm, dtype, frame);
    if (dtype == DT_F32) {
        /* np.mean on float32 keeps float32: sum in f32, divide in f32 */
        float s = ((const float *)pcm)[frame * channels];
        for (int c = 1; c < channels; ++c) s = s + ((const float *)pcm)[frame * channels + c];
        return (double)(s / (float)channels);
    }
    double s = load_sample(pcm, dtype, frame * channels);
    for (int c = 1; c < channels; ++c) s = s + load_sample(pcm, dtype, frame * channels + c);
    return s / (double)channels;
}

/* odd extension value 2*end - v computed in the working dtype
 * (scipy/signal/_arraytools.py:57-107 odd_ext: numpy integer arithmetic wraps) */
static double odd_ext_value(int wdt, double end, double v) {
    switch (wdt) {
    case DT_U8: return (double)(uint8_t)(uint32_t)((int64_t)(2 * (int64_t)end) - (int64_t)v);
    case DT_I16: return (double)(int16_t)(uint16_t)(uint32_t)((int64_t)(2 * (int64_t)end) - (int64_t)v);
    case DT_I32: return (double)(int32_t)(uint32_t)((int64_t)(2 * (int64_t)end) - (int64_t)v);
    case DT_F32: {
        volatile float t = (float)end * 2.0f;
        volatile float r = t - (float)v;
        return (double)r;
    }
    default: return 2.0 * end - v;
    }
}

/* ------------------------------------------------------------------------ */
/* A4: transfer-function DF-II-transposed filter, scipy _sigtools._linear_filter */
/* (scipy/signal/_signaltools.py:2175-2177 -> C DOUBLE filt loop):           */
/*   y = Z0 + b0*x ; Z_k = Z_{k+1} + x*b_{k+1} - y*a_{k+1} ; Z_last = x*b_n - y*a_n */
/* a[0] == 1 for butter() output, so the /a0 normalisation is exact.          */
/* ------------------------------------------------------------------------ */
static void df2t5(const double *b, const double *a, const double *x, int64_t n, double *z, double *y) {
    double z0 = z[0], z1 = z[1], z2 = z[2], z3 = z[3];
    for (int64_t k = 0; k < n; ++k) {
        double xn = x[k];
        double yn = z0 + b[0] * xn;
        z0 = z1 + xn * b[1] - yn * a[1];
        z1 = z2 + xn * b[2] - yn * a[2];
        z2 = z3 + xn * b[3] - yn * a[3];
        z3 = xn * b[4] - yn * a[4];
        y[k] = yn;
    }
    z[0] = z0; z[1] = z1; z[2] = z2; z[3] = z3;
}

/* scipy filtfilt(b, a, x) with padtype='odd', padlen=3*max(len(a),len(b))=15
 * (_signaltools.py:4523-4557, _validate_pad :4560-4591).  xd holds the picked
 * samples as doubles; wdt is their numpy dtype (pad arithmetic).  Returns 0,
 * or -1 when nd <= 15 (scipy raises ValueError). */
static int filtfilt_ba(const double *xd, int64_t nd, int wdt, const double *b, const double *a,
                       const double *zi, double *y) {
    const int64_t edge = 15;
    if (nd <= edge) return -1;
    int64_t ne = nd + 2 * edge;
    double *ext = (double *)malloc(sizeof(double) * ne);
    double *yf = (double *)malloc(sizeof(double) * ne);
    for (int64_t j = 0; j < edge; ++j) ext[j] = odd_ext_value(wdt, xd[0], xd[edge - j]);
    for (int64_t j = 0; j < nd; ++j) ext[edge + j] = xd[j];
    for (int64_t j = 0; j < edge; ++j) ext[edge + nd + j] = odd_ext_value(wdt, xd[nd - 1], xd[nd - 2 - j]);
    double z[4];
    for (int k = 0; k < 4; ++k) z[k] = zi[k] * ext[0];
    df2t5(b, a, ext, ne, z, yf);
    /* backward: filter the reversed forward output with zi * y[-1] */
    double y0 = yf[ne - 1];
    for (int64_t j = 0; j < ne / 2; ++j) { double t = yf[j]; yf[j] = yf[ne - 1 - j]; yf[ne - 1 - j] = t; }
    for (int k = 0; k < 4; ++k) z[k] = zi[k] * y0;
    df2t5(b, a, yf, ne, z, ext);
    for (int64_t j = 0; j < nd; ++j) y[j] = ext[ne - 1 - edge - j];
    free(ext);
    free(yf);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* A6: pandas rolling(window=w, min_periods, center=True).mean()             */
/* bounds: pandas/core/indexers/objects.py:93-120 (end = i+1+(w-1)//2,        */
/* start = end - w, both clipped); arithmetic: pandas _libs/window/           */
/* aggregations roll_mean (Kahan add/remove with separate compensations,     */
/* consecutive-same-value rule, sign clamps).                                */
/* ------------------------------------------------------------------------ */
static inline void win_bounds(int64_t i, int64_t n, int64_t w, int64_t *s, int64_t *e) {
    int64_t off = (w - 1) / 2;
    int64_t ee = i + 1 + off, ss = ee - w;
    *e = ee < 0 ? 0 : (ee > n ? n : ee);
    *s = ss < 0 ? 0 : (ss > n ? n : ss);
}

void bpmo_rolling_mean(const double *v, int64_t n, int64_t w, int64_t minp, double *out) {
    double sum = 0, comp_add = 0, comp_rem = 0, prev = NAN;
    int64_t nobs = 0, neg = 0, same = 0, ps = 0, pe = 0;
    for (int64_t i = 0; i < n; ++i) {
        int64_t s, e;
        win_bounds(i, n, w, &s, &e);
        if (i == 0 || s >= pe) {
            sum = comp_add = comp_rem = 0;
            nobs = neg = 0;
            prev = v[s];
            same = 0;
            for (int64_t j = s; j < e; ++j) {
                double val = v[j];
                if (val == val) {
                    nobs++;
                    double y = val - comp_add, t = sum + y;
                    comp_add = t - sum - y;
                    sum = t;
                    if (signbit(val)) neg++;
                    if (val == prev) same++; else same = 1;
                    prev = val;
                }
            }
        } else {
            for (int64_t j = ps; j < s; ++j) {
                double val = v[j];
                if (val == val) {
                    nobs--;
                    double y = -val - comp_rem, t = sum + y;
                    comp_rem = t - sum - y;
                    sum = t;
                    if (signbit(val)) neg--;
                }
            }
            for (int64_t j = pe; j < e; ++j) {
                double val = v[j];
                if (val == val) {
                    nobs++;
                    double y = val - comp_add, t = sum + y;
                    comp_add = t - sum - y;
                    sum = t;
                    if (signbit(val)) neg++;
                    if (val == prev) same++; else same = 1;
                    prev = val;
                }
            }
        }
        double r;
        if (nobs >= minp && nobs > 0) {
            r = sum / (double)nobs;
            if (same >= nobs) r = prev;
            else if (neg == 0 && r < 0) r = 0;
            else if (neg == nobs && r > 0) r = 0;
        } else {
            r = NAN;
        }
        out[i] = r;
        ps = s;
        pe = e;
    }
}

/* ------------------------------------------------------------------------ */
/* A1-A6 together: preprocess_audio minus file I/O (bpm_analysis.py:1007-1062) */
/* Returns nd, or -1 if nd <= 15.                                             */
/* ------------------------------------------------------------------------ */
int64_t bpmo_preprocess_ref(const void *pcm, int dtype, int64_t n_frames, int channels, int64_t ds,
                            const double *b, const double *a, const double *zi, int64_t env_w,
                            double *y_out, double *env_out) {
    if (ds < 1) ds = 1;
    int64_t nd = (n_frames + ds - 1) / ds;
    int wdt = work_dtype(dtype, channels);
    double *xd = (double *)malloc(sizeof(double) * (nd > 0 ? nd : 1));
    for (int64_t j = 0; j < nd; ++j) xd[j] = frame_value(pcm, dtype, channels, j * ds);
    double *y = y_out ? y_out : (double *)malloc(sizeof(double) * (nd > 0 ? nd : 1));
    int rc = filtfilt_ba(xd, nd, wdt, b, a, zi, y);
    free(xd);
    if (rc != 0) {
        if (!y_out) free(y);
        return -1;
    }
    double *ay = (double *)malloc(sizeof(double) * nd);
    for (int64_t j = 0; j < nd; ++j) ay[j] = fabs(y[j]);
    bpmo_rolling_mean(ay, nd, env_w, 1, env_out);
    free(ay);
    if (!y_out) free(y);
    return nd;
}

/* ------------------------------------------------------------------------ */
/* A13: sosfiltfilt at the native rate (native mode; north_star ordering).   */
/* scipy/signal/_signaltools.py:4718-4829 + _sosfilt per-section recursion:  */
/*   xn = s0*x + z0 ; z0 = s1*x - s4*xn + z1 ; z1 = s2*x - s5*xn              */
/* pad: odd, 15 samples (ntaps = 2*2+1), in the input dtype.                 */
/* Writes y (length n_frames, f64).  Returns 0 or -1 when n <= 15.           */
/* ------------------------------------------------------------------------ */
static void sosfilt2(const double *sos, const double *x, int64_t n, double *z, double *y) {
    double z00 = z[0], z01 = z[1], z10 = z[2], z11 = z[3];
    const double *s = sos, *t = sos + 6;
    for (int64_t k = 0; k < n; ++k) {
        double xc = x[k];
        double xn = s[0] * xc + z00;
        z00 = s[1] * xc - s[4] * xn + z01;
        z01 = s[2] * xc - s[5] * xn;
        xc = xn;
        xn = t[0] * xc + z10;
        z10 = t[1] * xc - t[4] * xn + z11;
        z11 = t[2] * xc - t[5] * xn;
        y[k] = xn;
    }
    z[0] = z00; z[1] = z01; z[2] = z10; z[3] = z11;
}

int bpmo_sosfiltfilt(const void *pcm, int dtype, int64_t n, int channels, const double *sos,
                     const double *zi /* [2][2] */, double *y) {
    const int64_t edge = 15;
    if (n <= edge) return -1;
    int wdt = work_dtype(dtype, channels);
    int64_t ne = n + 2 * edge;
    double *ext = (double *)malloc(sizeof(double) * ne);
    double *yf = (double *)malloc(sizeof(double) * ne);
    for (int64_t j = 0; j < n; ++j) ext[edge + j] = frame_value(pcm, dtype, channels, j);
    double x0 = ext[edge], xl = ext[edge + n - 1];
    for (int64_t j = 0; j < edge; ++j) ext[j] = odd_ext_value(wdt, x0, ext[edge + edge - j]);
    for (int64_t j = 0; j < edge; ++j) ext[edge + n + j] = odd_ext_value(wdt, xl, ext[edge + n - 2 - j]);
    double z[4];
    for (int k = 0; k < 4; ++k) z[k] = zi[k] * ext[0];
    sosfilt2(sos, ext, ne, z, yf);
    double y0 = yf[ne - 1];
    for (int64_t j = 0; j < ne / 2; ++j) { double t = yf[j]; yf[j] = yf[ne - 1 - j]; yf[ne - 1 - j] = t; }
    for (int k = 0; k < 4; ++k) z[k] = zi[k] * y0;
    sosfilt2(sos, yf, ne, z, ext);
    for (int64_t j = 0; j < n; ++j) y[j] = ext[ne - 1 - edge - j];
    free(ext);
    free(yf);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* A7: np.quantile(x, q), method 'linear'                                    */
/* numpy/lib/_function_base_impl.py:106-109 (virtual index (n-1)*q),          */
/* :4736-4769 _get_indexes, :4615-4636 _get_gamma, :4639-4660 _lerp.          */
/* ------------------------------------------------------------------------ */
static int cmp_double(const void *pa, const void *pb) {
    double a = *(const double *)pa, b = *(const double *)pb;
    return (a > b) - (a < b);
}

double bpmo_lerp_np(double a, double b, double t) {
    double d = b - a;
    if (t >= 0.5) return b - d * (1.0 - t);
    return a + d * t;
}

double bpmo_quantile(const double *x, int64_t n, double q) {
    if (n <= 0) return NAN;
    double *s = (double *)malloc(sizeof(double) * n);
    memcpy(s, x, sizeof(double) * n);
    qsort(s, (size_t)n, sizeof(double), cmp_double);
    double vi = (double)(n - 1) * q;
    double r;
    if (vi >= (double)(n - 1)) {
        r = s[n - 1];
    } else if (vi < 0) {
        r = s[0];
    } else {
        double lo = floor(vi);
        int64_t i = (int64_t)lo;
        r = bpmo_lerp_np(s[i], s[i + 1], vi - lo);
    }
    free(s);
    return r;
}

/* ------------------------------------------------------------------------ */
/* A8/A12: scipy.signal.find_peaks(x, height, distance, prominence)          */
/* scipy/signal/_peak_finding.py:729-1010; Cython helpers restated:          */
/*   _local_maxima_1d (plateau midpoint), _select_by_peak_distance (greedy   */
/*   keep-highest in argsort order), _peak_prominences (wlen=-1).            */
/* x is read as sgn*v so troughs (find_peaks(-env)) need no copy.            */
/* Ties of priority in the distance filter: numpy's default argsort is not   */
/* stable (its order is implementation-defined: x86-simd-sort on AVX-512,     */
/* introsort elsewhere); this restatement uses the stable order, i.e. among  */
/* equal heights the later peak is visited first, and reports whether that   */
/* choice decided anything (*tie, below).                                     */
/*                                                                            */
/* When is the tie order decisive?  _select_by_peak_distance visits the      */
/* candidates in priority blocks of equal height, highest first; a candidate */
/* is still alive when its block starts iff no KEPT candidate of strictly    */
/* greater height lies within `distance`.  If two alive candidates of one    */
/* block lie within `distance`, whichever is visited first removes the      */
/* other, so the order decides the outcome; otherwise no order can change    */
/* it.  In terms of the finished stable pass (by induction from the highest  */
/* block, whose alive set no order can change): the order was decisive iff   */
/* some REMOVED candidate has no kept candidate of strictly greater height   */
/* within `distance` — it was removed by an equal-height one.                */
/* ------------------------------------------------------------------------ */
typedef struct { double p; int64_t i; } prio_t;
static int cmp_prio(const void *pa, const void *pb) {
    const prio_t *a = (const prio_t *)pa, *b = (const prio_t *)pb;
    if (a->p < b->p) return -1;
    if (a->p > b->p) return 1;
    return (a->i > b->i) - (a->i < b->i);
}

/* _peak_prominences with wlen = -1 (scipy/signal/_peak_finding.py:982-995 ->
 * _peak_finding_utils): walk left while x <= x[p] tracking the minimum, the
 * same to the right; prominence = x[p] - max(left min, right min) */
double bpmo_prominence(const double *v, int64_t n, double sgn, int64_t p) {
    double xp = sgn * v[p];
    double lmin = xp, rmin = xp;
    for (int64_t k = p; k >= 0 && sgn * v[k] <= xp; --k)
        if (sgn * v[k] < lmin) lmin = sgn * v[k];
    for (int64_t k = p; k <= n - 1 && sgn * v[k] <= xp; ++k)
        if (sgn * v[k] < rmin) rmin = sgn * v[k];
    return xp - (lmin > rmin ? lmin : rmin);
}

int64_t bpmo_find_peaks_ex(const double *v, int64_t n, double sgn, const double *height, int64_t distance,
                           double prominence, int64_t *out, int *tie) {
    if (tie) *tie = 0;
#define X(k) (sgn * v[(k)])
    int64_t *pk = (int64_t *)malloc(sizeof(int64_t) * (n / 2 + 2));
    int64_t m = 0;
    /* _local_maxima_1d */
    int64_t i = 1, imax = n - 1;
    while (i < imax) {
        if (X(i - 1) < X(i)) {
            int64_t ia = i + 1;
            while (ia < imax && X(ia) == X(i)) ia++;
            if (X(ia) < X(i)) {
                pk[m++] = (i + ia - 1) / 2;
                i = ia;
            }
        }
        i++;
    }
    /* height: hmin <= x[peak]  (_select_by_property; array hmin indexed by peak) */
    if (height) {
        int64_t w = 0;
        for (int64_t j = 0; j < m; ++j)
            if (height[pk[j]] <= X(pk[j])) pk[w++] = pk[j];
        m = w;
    }
    /* distance */
    if (distance > 0 && m > 0) {
        prio_t *pr = (prio_t *)malloc(sizeof(prio_t) * m);
        uint8_t *keep = (uint8_t *)malloc(m);
        for (int64_t j = 0; j < m; ++j) { pr[j].p = X(pk[j]); pr[j].i = j; keep[j] = 1; }
        qsort(pr, (size_t)m, sizeof(prio_t), cmp_prio);
        for (int64_t r = m - 1; r >= 0; --r) {
            int64_t j = pr[r].i;
            if (!keep[j]) continue;
            for (int64_t k = j - 1; k >= 0 && pk[j] - pk[k] < distance; --k) keep[k] = 0;
            for (int64_t k = j + 1; k < m && pk[k] - pk[j] < distance; ++k) keep[k] = 0;
        }
        /* decisive tie: a removed candidate with no strictly higher kept one in reach */
        for (int64_t j = 0; j < m && tie && !*tie; ++j) {
            if (keep[j]) continue;
            int dominated = 0;
            for (int64_t k = j - 1; k >= 0 && pk[j] - pk[k] < distance && !dominated; --k)
                dominated = keep[k] && X(pk[k]) > X(pk[j]);
            for (int64_t k = j + 1; k < m && pk[k] - pk[j] < distance && !dominated; ++k)
                dominated = keep[k] && X(pk[k]) > X(pk[j]);
            if (!dominated) *tie = 1;
        }
        int64_t w = 0;
        for (int64_t j = 0; j < m; ++j)
            if (keep[j]) pk[w++] = pk[j];
        m = w;
        free(pr);
        free(keep);
    }
    /* prominence (wlen = -1: whole signal) */
    if (!isnan(prominence)) {
        int64_t w = 0;
        for (int64_t j = 0; j < m; ++j)
            if (prominence <= bpmo_prominence(v, n, sgn, pk[j])) pk[w++] = pk[j];
        m = w;
    }
#undef X
    if (out) memcpy(out, pk, sizeof(int64_t) * m);
    free(pk);
    return m;
}

int64_t bpmo_find_peaks(const double *v, int64_t n, double sgn, const double *height, int64_t distance,
                        double prominence, int64_t *out) {
    return bpmo_find_peaks_ex(v, n, sgn, height, distance, prominence, out, NULL);
}

/* ------------------------------------------------------------------------ */
/* A10 (N8): pd.Series(index=t, data=env[t]).reindex(arange(n)).interpolate() */
/* == np.interp on the trough grid, NaN before the first trough (pandas       */
/* limit_direction='forward' keeps leading NaN).  numpy arr_interp formula:   */
/*   slope = (y1 - y0) / (x1 - x0) ; r = slope*(x - x0) + y0 ; r = y0 at x==x0 */
/* ------------------------------------------------------------------------ */
void bpmo_interp_dense(const int64_t *t, int64_t m, const double *env, int64_t n, double *out) {
    int64_t j = 0;
    for (int64_t x = 0; x < n; ++x) {
        if (m == 0 || x < t[0]) { out[x] = NAN; continue; }
        while (j + 1 < m && t[j + 1] <= x) j++;
        if (j == m - 1 || t[j] == x) { out[x] = env[t[j]]; continue; }
        double y0 = env[t[j]], y1 = env[t[j + 1]];
        double slope = (y1 - y0) / ((double)t[j + 1] - (double)t[j]);
        double r = slope * ((double)x - (double)t[j]) + y0;
        if (isnan(r)) {
            r = slope * ((double)x - (double)t[j + 1]) + y1;
            if (isnan(r) && y0 == y1) r = y0;
        }
        out[x] = r;
    }
}

/* ------------------------------------------------------------------------ */
/* A10 (N7): rolling(W, min_periods, center=True).quantile(q)  (pandas        */
/* roll_quantile, interpolation 'linear': idx = int(q*(nobs-1)); exact order  */
/* statistics of the non-NaN window; vlow + (vhigh-vlow)*(idxf-idx)), then    */
/* .bfill().ffill().  Sorted buffer with binary insert/delete.               */
/* ------------------------------------------------------------------------ */
static int64_t lower_bound_d(const double *a, int64_t n, double v) {
    int64_t lo = 0, hi = n;
    while (lo < hi) { int64_t mid = (lo + hi) >> 1; if (a[mid] < v) lo = mid + 1; else hi = mid; }
    return lo;
}

void bpmo_rolling_quantile(const double *v, int64_t n, int64_t w, int64_t minp, double q, double *out) {
    double *buf = (double *)malloc(sizeof(double) * (w + 2));
    int64_t nobs = 0, ps = 0, pe = 0;
    for (int64_t i = 0; i < n; ++i) {
        int64_t s, e;
        win_bounds(i, n, w, &s, &e);
        if (i == 0 || s >= pe) {
            nobs = 0;
            for (int64_t j = s; j < e; ++j) {
                double val = v[j];
                if (val == val) {
                    int64_t at = lower_bound_d(buf, nobs, val);
                    memmove(buf + at + 1, buf + at, sizeof(double) * (nobs - at));
                    buf[at] = val;
                    nobs++;
                }
            }
        } else {
            for (int64_t j = pe; j < e; ++j) {
                double val = v[j];
                if (val == val) {
                    int64_t at = lower_bound_d(buf, nobs, val);
                    memmove(buf + at + 1, buf + at, sizeof(double) * (nobs - at));
                    buf[at] = val;
                    nobs++;
                }
            }
            for (int64_t j = ps; j < s; ++j) {
                double val = v[j];
                if (val == val) {
                    int64_t at = lower_bound_d(buf, nobs, val);
                    memmove(buf + at, buf + at + 1, sizeof(double) * (nobs - at - 1));
                    nobs--;
                }
            }
        }
        if (nobs >= minp && nobs > 0) {
            if (nobs == 1) {
                out[i] = buf[0];
            } else {
                double idxf = q * (double)(nobs - 1);
                int64_t idx = (int64_t)idxf;
                if ((double)idx == idxf) out[i] = buf[idx];
                else out[i] = buf[idx] + (buf[idx + 1] - buf[idx]) * (idxf - (double)idx);
            }
        } else {
            out[i] = NAN;
        }
        ps = s;
        pe = e;
    }
    free(buf);
    /* .bfill().ffill() */
    double next = NAN;
    for (int64_t i = n - 1; i >= 0; --i) {
        if (isnan(out[i])) out[i] = next; else next = out[i];
    }
    double last = NAN;
    for (int64_t i = 0; i < n; ++i) {
        if (isnan(out[i])) out[i] = last; else last = out[i];
    }
}

/* ------------------------------------------------------------------------ */
/* A7-A11: _calculate_dynamic_noise_floor (bpm_analysis.py:1064-1117)         */
/* flags bit0: static fallback (<5 troughs, :1073-1077)                       */
/*       bit1: sanitized <= 2, draft floor kept (:1107-1110)                  */
/*       bit2: all-NaN floor -> quantile(env, 0.1) (:1113-1115)               */
/*       bit5: the trough search's distance filter met a decisive height tie  */
/*             (bpmo_find_peaks_ex; BPMX_F_TROUGH_TIE in include/bpmx.h)      */
/* Returns the number of troughs written (sanitized, or raw in bit0 case).   */
/* ------------------------------------------------------------------------ */
typedef struct {
    int64_t distance;       /* int(min_peak_distance_sec * sr) */
    int64_t noise_window;   /* int(noise_window_sec * sr) */
    int64_t min_periods;    /* 3, hard-coded :1085,:1105 */
    double trough_prom_q;   /* trough_prominence_quantile */
    double noise_floor_q;   /* noise_floor_quantile */
    double reject_mult;     /* trough_rejection_multiplier */
    double fallback_q;      /* 0.1, hard-coded :1114 */
} bpmo_nf_params;

int64_t bpmo_noise_floor(const double *env, int64_t n, const bpmo_nf_params *p, double *floor_out,
                         int64_t *troughs_out, int *flags) {
    *flags = 0;
    double qt = bpmo_quantile(env, n, p->trough_prom_q);
    int64_t *tr = (int64_t *)malloc(sizeof(int64_t) * (n / 2 + 2));
    int tie = 0;
    int64_t nt = bpmo_find_peaks_ex(env, n, -1.0, NULL, p->distance, qt, tr, &tie);
    if (tie) *flags |= 32;
    if (nt < 5) {
        double fb = bpmo_quantile(env, n, p->noise_floor_q);
        for (int64_t i = 0; i < n; ++i) floor_out[i] = fb;
        memcpy(troughs_out, tr, sizeof(int64_t) * nt);
        *flags |= 1;
        free(tr);
        return nt;
    }
    double *dense = (double *)malloc(sizeof(double) * n);
    double *draft = (double *)malloc(sizeof(double) * n);
    bpmo_interp_dense(tr, nt, env, n, dense);
    bpmo_rolling_quantile(dense, n, p->noise_window, p->min_periods, p->noise_floor_q, draft);
    int64_t ns = 0;
    for (int64_t j = 0; j < nt; ++j) {
        double f = draft[tr[j]];
        if (!isnan(f) && env[tr[j]] <= p->reject_mult * f) troughs_out[ns++] = tr[j];
    }
    if (ns > 2) {
        bpmo_interp_dense(troughs_out, ns, env, n, dense);
        bpmo_rolling_quantile(dense, n, p->noise_window, p->min_periods, p->noise_floor_q, floor_out);
    } else {
        memcpy(floor_out, draft, sizeof(double) * n);
        *flags |= 2;
    }
    int all_nan = 1;
    for (int64_t i = 0; i < n; ++i)
        if (!isnan(floor_out[i])) { all_nan = 0; break; }
    if (all_nan) {
        double fb = bpmo_quantile(env, n, p->fallback_q);
        for (int64_t i = 0; i < n; ++i) floor_out[i] = fb;
        *flags |= 4;
    }
    free(dense);
    free(draft);
    free(tr);
    return ns;
}

/* A12: PeakClassifier._find_raw_peaks (bpm_analysis.py:223-229); *tie (may be
 * NULL) = the distance filter met a decisive height tie (BPMX_F_PEAK_TIE) */
int64_t bpmo_raw_peaks_ex(const double *env, int64_t n, const double *floor_v, int64_t distance,
                          double peak_prom_q, int64_t *out, int *tie) {
    double qp = bpmo_quantile(env, n, peak_prom_q);
    return bpmo_find_peaks_ex(env, n, 1.0, floor_v, distance, qp, out, tie);
}

int64_t bpmo_raw_peaks(const double *env, int64_t n, const double *floor_v, int64_t distance, double peak_prom_q,
                       int64_t *out) {
    return bpmo_raw_peaks_ex(env, n, floor_v, distance, peak_prom_q, out, NULL);
}
