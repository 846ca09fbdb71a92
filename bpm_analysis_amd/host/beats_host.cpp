/*
 * beats_host.cpp — the per-file beat stages after the hot path, as native code
 * for host threads ("why next": sequential per file,
 * so C++ on host threads beside the GPU batch).  Host-only; no GPU.
 *
 * Restates bpm_analysis_amd/beats.py (which is pinned against the reference's
 * own outputs, tests/golden/beats) in the same IEEE operation order:
 *   classifier        PeakClassifier.classify_peaks      bpm_analysis.py:64-330
 *                     confidence models                   :1120-1255
 *   preliminary pass  _run_preliminary_pass               :1623-1652, :1612-1620
 *   refinement        _refine_and_correct_peaks           :1257-1412, :1655-1698
 *   BPM curve         calculate_bpm_series                :1463-1484
 * Output: the final beats and the smoothed BPM curve (the series
 * <base>_bpm_plot.csv holds), plus the preliminary pass' start BPM, peak-BPM
 * time and recovery end, and one label per raw peak.  The debug strings,
 * HRV / slope metrics, reports and the plot stay in Python (beats.py): the
 * batch path (shard.run_sharded) needs only beats and curves.
 *
 * Python semantics kept where they decide: min()/max() return the first
 * argument unless the second compares strictly better (so NaN never wins a
 * min/max it is second in), numpy.interp's bracket and NaN retry, numpy's
 * median and 'linear' percentile, datetime.timedelta's round-half-even
 * microseconds and pandas' centred time window (t - w/2, t + w/2] with its
 * Kahan add/remove running mean.
 */
#include <cmath>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/bpmx_host.h"

namespace {

inline double py_min(double a, double b) { return b < a ? b : a; }
inline double py_max(double a, double b) { return b > a ? b : a; }
inline double clipv(double x, double lo, double hi) {      /* numpy.clip on a scalar */
    if (x != x) return x;
    if (x < lo) return lo;
    if (x > hi) return hi;
    return x;
}

/* numpy.interp for one x (compiled_base.c arr_interp) */
double interp1(double x, const double *xp, const double *fp, int n) {
    if (x != x) return x;
    if (x < xp[0]) return fp[0];
    if (x > xp[n - 1]) return fp[n - 1];
    int j = (int)(std::upper_bound(xp, xp + n, x) - xp) - 1;
    if (j == n - 1 || xp[j] == x) return fp[j];
    const double slope = (fp[j + 1] - fp[j]) / (xp[j + 1] - xp[j]);
    double r = slope * (x - xp[j]) + fp[j];
    if (r != r) {
        r = slope * (x - xp[j + 1]) + fp[j + 1];
        if (r != r && fp[j] == fp[j + 1]) r = fp[j];
    }
    return r;
}

const double DEV_X[5] = {0.0, 0.25, 0.40, 0.80, 1.0};
const double CURVE_LO[5] = {0.9, 0.9, 0.7, 0.1, 0.1};
const double CURVE_HI[5] = {0.1, 0.5, 0.75, 0.65, 0.0};
const double RHYTHM_X[4] = {0.0, 0.15, 0.30, 0.50}, RHYTHM_Y[4] = {1.0, 0.8, 0.4, 0.0};
const double AMP_X[4] = {0.0, 0.4, 0.7, 1.0}, AMP_Y[4] = {0.0, 0.4, 0.8, 1.0};

double blend(double bpm, const bpmx_beat_params &p) {
    return clipv((bpm - p.contractility_bpm_low) / (p.contractility_bpm_high - p.contractility_bpm_low), 0, 1);
}
double blended_confidence(double dev, double bpm, const bpmx_beat_params &p) {
    const double b = blend(bpm, p);
    double fp[5];
    for (int i = 0; i < 5; ++i) fp[i] = CURVE_LO[i] + (CURVE_HI[i] - CURVE_LO[i]) * b;
    return interp1(dev, DEV_X, fp, 5);
}
double update_long_term_bpm(double rr, double ltb, const bpmx_beat_params &p) {
    const double target = (1 - 0.05) * ltb + 0.05 * (60.0 / rr);
    const double lim = 3.0 * rr;
    const double step = clipv(target - ltb, -lim, lim);
    return py_max(p.min_bpm, py_min(ltb + step, p.max_bpm));
}

/* numpy.median of a copy */
double median(std::vector<double> v) {
    const size_t n = v.size();
    std::sort(v.begin(), v.end());
    if (n & 1) return v[n / 2];
    return (v[n / 2 - 1] + v[n / 2]) / 2.0;
}
/* numpy.percentile(v, q) 'linear' (numpy _lerp) of a sorted vector */
double percentile_sorted(const std::vector<double> &s, double q) {
    const size_t n = s.size();
    const double vi = (double)(n - 1) * (q / 100.0);
    double lo = std::floor(vi);
    if (lo > (double)(n - 1)) lo = (double)(n - 1);
    const size_t l = (size_t)lo, h = l + 1 < n ? l + 1 : n - 1;
    const double g = vi - lo, a = s[l], b = s[h], d = b - a;
    return g >= 0.5 ? b - d * (1 - g) : a + d * g;
}

/* pandas roll_mean over [start[i], end[i]) with monotone bounds (Kahan add /
 * remove, 'same value' and sign rules: pandas/_libs/window/aggregations.pyx) */
void roll_mean(const double *v, const int64_t *st, const int64_t *en, int64_t n, int64_t minp, double *out) {
    double sum = 0, ca = 0, cr = 0, prev = NAN;
    int64_t nobs = 0, neg = 0, same = 0;
    auto add = [&](double x) {
        if (x != x) return;
        nobs++;
        const double y = x - ca, t = sum + y;
        ca = t - sum - y;
        sum = t;
        if (std::signbit(x)) neg++;
        if (x == prev) same++; else same = 1;
        prev = x;
    };
    auto rem = [&](double x) {
        if (x != x) return;
        nobs--;
        const double y = -x - cr, t = sum + y;
        cr = t - sum - y;
        sum = t;
        if (std::signbit(x)) neg--;
    };
    for (int64_t i = 0; i < n; ++i) {
        const int64_t s = st[i], e = en[i];
        if (i == 0 || s >= en[i - 1]) {
            sum = ca = cr = 0;
            nobs = neg = 0;
            prev = v[s];
            same = 0;
            for (int64_t j = s; j < e; ++j) add(v[j]);
        } else {
            for (int64_t j = st[i - 1]; j < s; ++j) rem(v[j]);
            for (int64_t j = en[i - 1]; j < e; ++j) add(v[j]);
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
    }
}

/* datetime.timedelta(seconds=x) in microseconds (CPython: modf, then the
 * fractional part times 1e6 rounded half to even) */
int64_t timedelta_us(double x) {
    double ip;
    const double fr = std::modf(x, &ip);
    return (int64_t)ip * 1000000 + (int64_t)std::nearbyint(fr * 1e6);
}

/* beats.bpm_series: instantaneous BPM between beats, then the centred '<w>s'
 * time-window mean (min_periods 1) on the beat-time index.  Fills t (beat
 * times of the kept intervals) and curve; returns the count (0: empty). */
int64_t bpm_series(const std::vector<int64_t> &pk, int32_t sr, double window_sec, std::vector<double> &t_ok,
                   std::vector<double> &curve) {
    t_ok.clear();
    curve.clear();
    if (pk.size() < 2) return 0;
    std::vector<double> bpm;
    for (size_t i = 1; i < pk.size(); ++i) {
        const double t0 = (double)pk[i - 1] / (double)sr, t1 = (double)pk[i] / (double)sr;
        const double dt = t1 - t0;
        if (dt > 1e-6) {
            bpm.push_back(60.0 / dt);
            t_ok.push_back(t1);
        }
    }
    const int64_t m = (int64_t)bpm.size();
    if (m == 0) { t_ok.clear(); return 0; }
    if (!(median(bpm) > 0)) return 0;                 /* the reference leaves the curve empty */
    std::vector<int64_t> ns(m), st(m), en(m);
    for (int64_t i = 0; i < m; ++i) ns[i] = timedelta_us(t_ok[i]) * 1000;
    const int64_t half = (int64_t)std::llround(window_sec * 1e9) / 2;
    /* pandas calculate_variable_window_bounds, center=True, closed='right':
     * (t_i - w/2, t_i + w/2] */
    int64_t s = 0, e = 0;
    for (int64_t i = 0; i < m; ++i) {
        const int64_t lo = ns[i] - half, hi = ns[i] + half;
        while (s < i && ns[s] <= lo) ++s;
        if (e < i + 1) e = i + 1;
        while (e < m && ns[e] <= hi) ++e;
        st[i] = s;
        en[i] = e;
    }
    curve.resize(m);
    roll_mean(bpm.data(), st.data(), en.data(), m, 1, curve.data());
    return m;
}

enum { T_NONE = 0, T_S1 = 1, T_S2 = 2, T_LONE = 3, T_NOISE = 4 };

struct Classifier {
    const double *env;
    int32_t sr;
    const bpmx_beat_params &p;
    double thr;                                       /* pairing confidence threshold */
    bool have_rec;
    double t_pk, t_end;
    std::vector<int64_t> pk;
    std::vector<double> envpk, str, dev, dev_t;
    double start_bpm;

    Classifier(const double *env_, const double *floor, const int64_t *peaks, int64_t np, int32_t sr_,
               const bpmx_beat_params &p_, double thr_, double hint, bool have_hint, double tpk, double tend,
               bool have_rec_)
        : env(env_), sr(sr_), p(p_), thr(thr_), have_rec(have_rec_), t_pk(tpk), t_end(tend) {
        pk.assign(peaks, peaks + np);
        envpk.resize(np);
        str.resize(np);
        std::vector<double> strength(np);
        for (int64_t i = 0; i < np; ++i) {
            envpk[i] = env[pk[i]];
            const double s = env[pk[i]] - floor[pk[i]];
            strength[i] = s < 0 ? 0 : s;                   /* strength[strength < 0] = 0 */
            str[i] = s > 0 ? s : 0.0;                      /* max(0, e - f) */
        }
        const int64_t nd = np > 1 ? np - 1 : 0;
        std::vector<double> raw(nd);
        dev_t.resize(nd);
        for (int64_t i = 0; i < nd; ++i) {
            const double a = strength[i], b = strength[i + 1];
            const double mx = (a != a || b != b) ? NAN : (a > b ? a : b);     /* np.maximum */
            raw[i] = std::fabs(b - a) / (mx + 1e-9);
            dev_t[i] = (double)(pk[i] + pk[i + 1]) / 2 / sr;
        }
        int64_t win = (int64_t)((double)nd * p.deviation_smoothing_factor);
        if (win < 5) win = 5;
        dev.resize(nd);
        if (nd > 0) {
            std::vector<int64_t> st(nd), en(nd);
            const int64_t off = (win - 1) / 2;
            for (int64_t i = 0; i < nd; ++i) {
                int64_t e = i + 1 + off, s = e - win;
                en[i] = e < 0 ? 0 : (e > nd ? nd : e);
                st[i] = s < 0 ? 0 : (s > nd ? nd : s);
            }
            roll_mean(raw.data(), st.data(), en.data(), nd, 1, dev.data());
        }
        start_bpm = (have_hint && hint != 0) ? hint : 80.0;
    }

    double dev_asof(double t) const {
        int64_t k = (int64_t)(std::upper_bound(dev_t.begin(), dev_t.end(), t) - dev_t.begin()) - 1;
        while (k >= 0 && dev[k] != dev[k]) --k;
        return k >= 0 ? dev[k] : NAN;
    }

    bool pair(int64_t j, double ratio, double ltb, int64_t n_beats) const {
        const int64_t s1 = pk[j], s2 = pk[j + 1];
        const double gap = (double)(s2 - s1) / (double)sr;
        double conf = blended_confidence(dev_asof((double)s1 / (double)sr), ltb, p);
        if (n_beats >= 5) {
            const double xs[2] = {0.0, 1.0}, ys[2] = {p.stability_confidence_floor, p.stability_confidence_ceiling};
            conf *= interp1(ratio, xs, ys, 2);
        }
        const double a1 = str[j], a2 = str[j + 1];
        const double r21 = a2 / (a1 + 1e-9);
        const double lo = p.contractility_bpm_low;
        const double t1s = (double)s1 / (double)sr;
        const bool recovering = have_rec && t_pk < t1s && t1s < t_end;
        const double xs[2] = {lo, p.contractility_bpm_high}, ys[2] = {p.s2_s1_ratio_low_bpm, p.s2_s1_ratio_high_bpm};
        const double r_max = interp1(recovering ? py_max(ltb, lo) : ltb, xs, ys, 2);
        const double boost_at = p.s1_s2_boost_ratio;
        if (r21 > r_max) {
            const double amt = p.penalty_amount_min + clipv((r21 / r_max - 1.0) / 2.0, 0, 1) *
                                                          (p.penalty_amount_max - p.penalty_amount_min);
            conf -= amt;
        } else if (a1 > a2 * boost_at) {
            const double r12 = a1 / (a2 + 1e-9);
            const double amt = p.boost_amount_min + clipv((r12 - boost_at) / (4.0 - boost_at), 0, 1) *
                                                        (p.boost_amount_max - p.boost_amount_min);
            conf += amt;
        }
        conf = py_max(0.0, py_min(1.0, conf));
        const double cap = py_min(p.s1_s2_interval_cap_sec, (60.0 / ltb) * p.s1_s2_interval_rr_fraction);
        if (p.enable_interval_penalty && gap > cap) {
            const double z0 = cap * p.interval_penalty_start_factor, z1 = cap * p.interval_penalty_full_factor;
            if (gap > z0) {
                const double amt = clipv((gap - z0) / (z1 - z0 + 1e-9), 0, 1) * p.interval_max_penalty;
                conf = py_max(0, conf - amt);
            }
        }
        return conf >= thr;
    }

    /* (valid, rejected on rhythm) */
    void lone(int64_t j, int64_t jl, double ltb, bool &valid, bool &on_rhythm) const {
        const int64_t cur = pk[j], last = pk[jl];
        const double exp_rr = 60.0 / ltb;
        const double rr = (double)(cur - last) / (double)sr;
        const double rs = interp1(std::fabs(rr - exp_rr) / exp_rr, RHYTHM_X, RHYTHM_Y, 4);
        const double ar = str[j] / (str[jl] + 1e-9);
        const double am = interp1(ar, AMP_X, AMP_Y, 4);
        const double conf = (rs * p.lone_s1_rhythm_weight) + (am * p.lone_s1_amplitude_weight);
        if (conf < p.lone_s1_confidence_threshold) { valid = false; on_rhythm = true; return; }
        on_rhythm = false;
        if (j < (int64_t)pk.size() - 1) {
            const double fwd = (double)(pk[j + 1] - cur) / (double)sr;
            if (fwd < exp_rr * p.lone_s1_forward_check_pct && !(envpk[j] > (envpk[j + 1] * 1.7))) {
                valid = false;
                return;
            }
        }
        valid = true;
    }

    /* classify_peaks: s1 (sorted positions) and one tag per raw peak */
    void classify(std::vector<int64_t> &s1, std::vector<int8_t> &tag) const {
        const int64_t n = (int64_t)pk.size();
        tag.assign(n, T_NONE);
        s1.clear();
        if (n < 2) { s1 = pk; return; }
        const int64_t hist_w = p.stability_history_window;
        std::vector<int64_t> beats;
        std::vector<char> paired;
        int64_t n_paired_win = 0;
        double ltb = start_bpm;
        int64_t rr_fails = 0;
        auto add_beat = [&](int64_t j, bool is_pair) {
            beats.push_back(j);
            paired.push_back(is_pair);
            n_paired_win += is_pair;
            if ((int64_t)beats.size() > hist_w) n_paired_win -= paired[paired.size() - hist_w - 1];
        };
        int64_t j = 0;
        while (j < n) {
            const double ratio = (int64_t)beats.size() < hist_w ? 0.5 : (double)n_paired_win / (double)hist_w;
            if (j >= n - 1) {
                add_beat(j, false);
                tag[j] = T_LONE;
                j += 1;
            } else if (pair(j, ratio, ltb, (int64_t)beats.size())) {
                add_beat(j, true);
                tag[j] = T_S1;
                tag[j + 1] = T_S2;
                rr_fails = 0;
                j += 2;
            } else {
                bool valid = true, on_rhythm = false;
                if (!beats.empty()) lone(j, beats.back(), ltb, valid, on_rhythm);
                if (valid) {
                    add_beat(j, false);
                    tag[j] = T_LONE;
                    rr_fails = 0;
                } else {
                    rr_fails = on_rhythm ? rr_fails + 1 : 0;
                    if (rr_fails >= p.cascade_reset_trigger_count) {
                        add_beat(j, false);
                        tag[j] = T_LONE;
                        rr_fails = 0;
                    } else {
                        tag[j] = T_NOISE;
                    }
                }
                j += 1;
            }
            if (beats.size() > 1) {
                const double rr = (double)(pk[beats[beats.size() - 1]] - pk[beats[beats.size() - 2]]) / (double)sr;
                if (rr > 0) ltb = update_long_term_bpm(rr, ltb, p);
            }
        }
        for (int64_t b : beats) s1.push_back(pk[b]);
        std::sort(s1.begin(), s1.end());
    }
};

/* refine: correct_peaks_by_rhythm, then up to 5 discontinuity passes */
std::vector<int64_t> correct_by_rhythm(const std::vector<int64_t> &peaks, const double *env, int32_t sr,
                                       const bpmx_beat_params &p) {
    if (peaks.size() < 5) return peaks;
    std::vector<double> d(peaks.size() - 1);
    for (size_t i = 1; i < peaks.size(); ++i) d[i - 1] = (double)(peaks[i] - peaks[i - 1]) / (double)sr;
    const double thr = median(d) * p.rr_correction_threshold_pct;
    std::vector<int64_t> kept{peaks[0]};
    for (size_t i = 1; i < peaks.size(); ++i) {
        const int64_t q = peaks[i];
        if ((double)(q - kept.back()) / (double)sr < thr) {
            if (env[q] > env[kept.back()]) kept.back() = q;
        } else {
            kept.push_back(q);
        }
    }
    return kept;
}

/* one gap-fill + short-interval pass; noisy[k]: raw peak k's debug string
 * contains "Noise" (classified Noise; a gap correction keeps it in its
 * ORIGINAL_REASON) */
int fix_discontinuities(std::vector<int64_t> &s1, const std::vector<int64_t> &raw, const std::vector<char> &noisy,
                        const double *env, const double *floor, const bpmx_beat_params &p, int32_t sr) {
    const int m = 3;
    if ((int64_t)s1.size() < 2 * m) return 0;
    std::vector<double> rr(s1.size() - 1);
    for (size_t i = 1; i < s1.size(); ++i) rr[i - 1] = (double)(s1[i] - s1[i - 1]) / (double)sr;
    std::vector<double> srt = rr;
    std::sort(srt.begin(), srt.end());
    const double q1 = percentile_sorted(srt, 25), q3 = percentile_sorted(srt, 75);
    const double iqr = q3 - q1;
    std::vector<double> stable;
    for (double v : rr)
        if (v > (q1 - 1.5 * iqr) && v < (q3 + 1.5 * iqr)) stable.push_back(v);
    if (stable.empty()) return 0;
    const double med = median(stable);
    const double short_thr = med * p.rr_correction_threshold_pct;
    const double long_thr = med * p.rr_correction_long_interval_pct;
    std::vector<int64_t> added;
    int n_fix = 0;
    const double waiver = p.penalty_waiver_strength_ratio, max_ratio = p.penalty_waiver_max_s2_s1_ratio;
    for (int64_t i = m; i < (int64_t)s1.size() - 1 - m; ++i) {
        const int64_t a = s1[i], b = s1[i + 1];
        if (!((double)(b - a) / (double)sr > long_thr)) continue;
        const int64_t lo = std::upper_bound(raw.begin(), raw.end(), a) - raw.begin();
        const int64_t hi = std::lower_bound(raw.begin(), raw.end(), b) - raw.begin();
        for (int64_t k = lo; k < hi; ++k) {
            const int64_t c1 = raw[k];
            if (!noisy[k] || std::find(added.begin(), added.end(), c1) != added.end() || k + 1 >= (int64_t)raw.size())
                continue;
            const int64_t c2 = raw[k + 1];
            if (c2 >= b || !noisy[k + 1]) continue;
            const double ex = env[c1] - floor[c1];
            if (py_max(0, ex) > waiver * floor[c1] && (env[c2] / (env[c1] + 1e-9)) < max_ratio) {
                n_fix += 1;
                added.push_back(c1);
                break;
            }
        }
    }
    std::vector<int64_t> merged = s1;
    merged.insert(merged.end(), added.begin(), added.end());
    std::sort(merged.begin(), merged.end());
    merged.erase(std::unique(merged.begin(), merged.end()), merged.end());
    std::vector<int64_t> drop;
    auto dropped = [&](int64_t v) { return std::find(drop.begin(), drop.end(), v) != drop.end(); };
    for (int64_t i = m; i < (int64_t)merged.size() - 1 - m; ++i) {
        const int64_t a = merged[i], b = merged[i + 1];
        if (dropped(a) || dropped(b)) continue;
        if ((double)(b - a) / (double)sr < short_thr) {
            drop.push_back(env[b] > env[a] ? a : b);
            n_fix += 1;
        }
    }
    std::vector<int64_t> out;
    for (int64_t v : merged)
        if (!dropped(v)) out.push_back(v);
    s1.swap(out);
    return n_fix;
}

}  // namespace

extern "C" {

int bpmx_host_abi_version(void) { return BPMX_HOST_ABI_VERSION; }

int bpmx_beats(const double *env, int64_t n_env, const double *floor, const int64_t *peaks, int64_t n_peaks,
               int32_t sr, const bpmx_beat_params *prm, double start_bpm_hint, int64_t *final_out,
               int64_t *n_final, double *bpm_t_out, double *bpm_out, int64_t *n_bpm, double *pass_out,
               int8_t *tags_out) {
    if (!env || !floor || (!peaks && n_peaks > 0) || !prm || !final_out || !n_final || !bpm_t_out || !bpm_out ||
        !n_bpm || sr < 1 || n_env < 0 || n_peaks < 0)
        return BPMX_HOST_E_ARG;
    for (int64_t i = 0; i < n_peaks; ++i)
        if (peaks[i] < 0 || peaks[i] >= n_env) return BPMX_HOST_E_ARG;
    const bpmx_beat_params &p = *prm;
    const bool have_hint = start_bpm_hint == start_bpm_hint;
    *n_final = 0;
    *n_bpm = 0;
    /* preliminary anchor pass at pairing threshold 0.75 (:1623-1652) */
    std::vector<int64_t> anchors, s1, tv;
    std::vector<int8_t> tag;
    std::vector<double> t_ok, curve;
    {
        Classifier c(env, floor, peaks, n_peaks, sr, p, 0.75, start_bpm_hint, have_hint, 0, 0, false);
        c.classify(anchors, tag);
    }
    double est = NAN;
    if (anchors.size() >= 10) {
        std::vector<double> d(anchors.size() - 1);
        for (size_t i = 1; i < anchors.size(); ++i) d[i - 1] = (double)(anchors[i] - anchors[i - 1]) / (double)sr;
        const double med = median(d);
        if (med > 0) est = 60.0 / med;
    }
    /* start_bpm_hint or est or 80.0 (Python truthiness: 0 and None fall through) */
    const double start = (have_hint && start_bpm_hint != 0) ? start_bpm_hint : ((est == est && est != 0) ? est : 80.0);
    bpm_series(anchors, sr, p.output_smoothing_window_sec, t_ok, curve);
    bool have_rec = false;
    double t_pk = NAN, t_end = NAN;
    if (t_ok.size() >= 2) {                           /* find_recovery_phase (:1612-1620) */
        size_t am = 0;                                /* numpy.argmax: the first maximum (a NaN wins) */
        for (size_t i = 1; i < curve.size(); ++i) {
            if (curve[am] != curve[am]) break;
            if (curve[i] != curve[i] || curve[i] > curve[am]) am = i;
        }
        t_pk = t_ok[am];
        t_end = t_pk + p.recovery_phase_duration_sec;
        have_rec = true;
    }
    if (pass_out) { pass_out[0] = start; pass_out[1] = t_pk; pass_out[2] = t_end; }
    /* main classifier */
    Classifier c(env, floor, peaks, n_peaks, sr, p, p.pairing_confidence_threshold, start, true, t_pk, t_end, have_rec);
    c.classify(s1, tag);
    if (tags_out)
        for (int64_t i = 0; i < n_peaks; ++i) tags_out[i] = tag[i];
    if (n_peaks < 2) return BPMX_HOST_E_FEW_PEAKS;    /* the reference's refinement raises KeyError here */
    /* refinement (:1655-1698) */
    std::vector<char> noisy(n_peaks);
    for (int64_t i = 0; i < n_peaks; ++i) noisy[i] = tag[i] == T_NOISE;
    std::vector<int64_t> fin = correct_by_rhythm(s1, env, sr, p);
    for (int it = 0; it < 5; ++it)
        if (fix_discontinuities(fin, c.pk, noisy, env, floor, p, sr) == 0) break;
    for (size_t i = 0; i < fin.size(); ++i) final_out[i] = fin[i];
    *n_final = (int64_t)fin.size();
    /* final BPM curve (:1463-1484), only when >= 2 beats survive (:1749-1757) */
    if (fin.size() >= 2) {
        bpm_series(fin, sr, p.output_smoothing_window_sec, t_ok, curve);
        for (size_t i = 0; i < curve.size(); ++i) { bpm_t_out[i] = t_ok[i]; bpm_out[i] = curve[i]; }
        *n_bpm = (int64_t)curve.size();
    }
    return BPMX_HOST_OK;
}

int bpmx_beats_batch(int32_t n_files, const double *const *env, const int64_t *n_env, const double *const *floor,
                     const int64_t *const *peaks, const int64_t *n_peaks, const int32_t *sr,
                     const bpmx_beat_params *params, double start_bpm_hint, int32_t threads,
                     int64_t *const *final_out, int64_t *n_final, double *const *bpm_t_out, double *const *bpm_out,
                     int64_t *n_bpm, double *pass_out, int8_t *const *tags_out, int32_t *status) {
    if (n_files < 0 || !env || !n_env || !floor || !peaks || !n_peaks || !sr || !params || !final_out || !n_final ||
        !bpm_t_out || !bpm_out || !n_bpm || !status)
        return BPMX_HOST_E_ARG;
    std::atomic<int32_t> next{0};
    auto work = [&]() {
        for (int32_t f; (f = next.fetch_add(1)) < n_files;)
            status[f] = bpmx_beats(env[f], n_env[f], floor[f], peaks[f], n_peaks[f], sr[f], params, start_bpm_hint,
                                   final_out[f], &n_final[f], bpm_t_out[f], bpm_out[f], &n_bpm[f],
                                   pass_out ? pass_out + 3 * (int64_t)f : nullptr, tags_out ? tags_out[f] : nullptr);
    };
    const int32_t nt = threads < 1 ? 1 : (threads > n_files ? (n_files > 0 ? n_files : 1) : threads);
    std::vector<std::thread> pool;
    for (int32_t t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto &th : pool) th.join();
    return BPMX_HOST_OK;
}

}  // extern "C"
