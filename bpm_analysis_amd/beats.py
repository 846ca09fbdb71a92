"""Host-side beat logic on top of the GPU detection path.

What the reference does per file after the raw peaks are known, restated over
flat per-peak arrays instead of a state dict:

* ``PeakClassifier``        S1/S2 pairing state machine       bpm_analysis.py:64-330
  (confidence models :1120-1255: blended pairing confidence, stability/ratio
  adjustment, lone-S1 confidence, long-term BPM update)
* ``run_preliminary_pass``  high-confidence anchor pass         :1623-1652, :1612-1620
* ``refine_peaks``          rhythm correction + gap/conflict fix :1257-1412, :1655-1698
* ``bpm_series``            smoothed BPM curve                   :1463-1484
* ``final_metrics``         inclines/declines, HRR, slopes, HRV  :1414-1461, :1486-1610, :1701-1722
* ``analyze_recording``     the per-file orchestration of analyze_wav_file :1725-1757

The raw peaks, envelope and noise floor come from libbpmx.so (one batched
``bpmx_run``); nothing here re-runs the hot path unless the caller omits the
raw peaks.  Decisions are threshold compares on doubles, so every expression
keeps the reference's operation order (and its Python ``min``/``max`` NaN
behaviour) to decide the same way bit for bit; the debug strings are the
reference's own, so reports and the labeler read them unchanged.
Parity: tests/test_beats.py against goldens made by the reference itself
(tests/golden/make_beat_goldens.py).
"""
from __future__ import annotations

import bisect
import csv
import datetime
import logging
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd

# Peak labels (bpm_analysis.py:26-36)
S1_PAIRED = "S1 (Paired)"
S2_PAIRED = "S2 (Paired)"
LONE_S1 = "Lone S1"
LONE_S1_CASCADE = "Lone S1 (Corrected by Cascade Reset)"
LONE_S1_LAST = "Lone S1 (Last Peak)"
NOISE = "Noise/Rejected"
S1_GAP = "S1 (Paired - Corrected from Gap)"
S2_GAP = "S2 (Paired - Corrected from Gap)"

# per-raw-peak tags used inside the classifier loop (equivalent to the
# reference's substring tests on the debug strings, which are unique per tag)
_T_NONE, _T_S1, _T_S2, _T_LONE, _T_NOISE = 0, 1, 2, 3, 4

_DEV_X = (0.0, 0.25, 0.40, 0.80, 1.0)
_CURVE_LO = (0.9, 0.9, 0.7, 0.1, 0.1)
_CURVE_HI = (0.1, 0.5, 0.75, 0.65, 0.0)
_RHYTHM_X, _RHYTHM_Y = (0.0, 0.15, 0.30, 0.50), (1.0, 0.8, 0.4, 0.0)
_AMP_X, _AMP_Y = (0.0, 0.4, 0.7, 1.0), (0.0, 0.4, 0.8, 1.0)


# Scalar numpy.interp / numpy.clip on Python floats: the same IEEE operations in
# the same order as numpy's compiled loops (numpy/_core/src/multiarray/
# compiled_base.c arr_interp: bracket by binary search, exact hits and the right
# end return fp[j], else slope*(x - xp[j]) + fp[j], NaN retried from the right
# end), without numpy's per-call overhead on the classifier's hot loop.
def _interp(x, xp, fp):
    if x != x:
        return x
    if x < xp[0]:
        return fp[0]
    n = len(xp)
    if x > xp[n - 1]:
        return fp[n - 1]
    j = bisect.bisect_right(xp, x) - 1
    if j == n - 1 or xp[j] == x:
        return fp[j]
    slope = (fp[j + 1] - fp[j]) / (xp[j + 1] - xp[j])
    r = slope * (x - xp[j]) + fp[j]
    if r != r:
        r = slope * (x - xp[j + 1]) + fp[j + 1]
        if r != r and fp[j] == fp[j + 1]:
            r = fp[j]
    return r


def _clip(x, lo, hi):
    """numpy.clip for scalars: NaN propagates, ties keep x (so -0.0 stays -0.0)."""
    if x != x:
        return x
    if x < lo:
        return float(lo)
    if x > hi:
        return float(hi)
    return x


# ---------------------------------------------------------------- confidence models
def _blend(bpm: float, p: Dict):
    return _clip((bpm - p['contractility_bpm_low']) / (p['contractility_bpm_high'] - p['contractility_bpm_low']), 0, 1)


def calculate_blended_confidence(deviation: float, bpm: float, params: Dict) -> float:
    """Pairing confidence from the amplitude deviation on a BPM-blended curve (:1120-1143)."""
    b = _blend(bpm, params)
    return _interp(deviation, _DEV_X, tuple(lo + (hi - lo) * b for lo, hi in zip(_CURVE_LO, _CURVE_HI)))


def update_long_term_bpm(new_rr_sec: float, current_long_term_bpm: float, params: Dict) -> float:
    """EMA (lr 0.05) with a 3 BPM-per-second-of-RR slew limit, clamped to [min_bpm, max_bpm] (:1239-1255)."""
    target = (1 - 0.05) * current_long_term_bpm + 0.05 * (60.0 / new_rr_sec)
    lim = 3.0 * new_rr_sec
    step = _clip(target - current_long_term_bpm, -lim, lim)
    return max(params['min_bpm'], min(current_long_term_bpm + step, params['max_bpm']))


# ---------------------------------------------------------------- classifier
class PeakClassifier:
    """S1/S2/noise classification of the raw peaks (bpm_analysis.py:64-330).

    Same constructor and ``classify_peaks() -> (s1_peaks, all_raw_peaks,
    analysis_data)`` as the reference.  ``raw_peaks`` (extra keyword) takes
    the GPU's raw peaks from a batched run; without it they are found on the
    GPU here (dropin.find_raw_peaks, the reference's ``_find_raw_peaks``)."""

    def __init__(self, audio_envelope: np.ndarray, sample_rate: int, params: Dict,
                 start_bpm_hint: Optional[float], precomputed_noise_floor: pd.Series,
                 precomputed_troughs: np.ndarray, peak_bpm_time_sec: Optional[float],
                 recovery_end_time_sec: Optional[float], raw_peaks: Optional[np.ndarray] = None):
        self.audio_envelope = env = np.asarray(audio_envelope)
        self.sample_rate = sr = sample_rate
        self.params = p = params
        self.peak_bpm_time_sec = peak_bpm_time_sec
        self.recovery_end_time_sec = recovery_end_time_sec
        self.noise_floor = precomputed_noise_floor
        self.troughs = precomputed_troughs
        floor = np.asarray(getattr(precomputed_noise_floor, "values", precomputed_noise_floor), dtype=np.float64)
        self._floor = floor
        if raw_peaks is None:
            from .dropin import find_raw_peaks
            raw_peaks = find_raw_peaks(env, sr, p, floor)
        self.peaks = pk = np.asarray(raw_peaks, dtype=np.int64)

        # amplitude-deviation curve between consecutive raw peaks (:93-101)
        strength = env[pk] - floor[pk]
        strength[strength < 0] = 0
        dev = np.abs(np.diff(strength)) / (np.maximum(strength[:-1], strength[1:]) + 1e-9)
        self._dev_t = (pk[:-1] + pk[1:]) / 2 / sr
        win = max(5, int(len(dev) * p['deviation_smoothing_factor']))
        self._dev = pd.Series(dev).rolling(window=win, min_periods=1, center=True).mean().to_numpy()
        self.deviation_series = pd.Series(self._dev, index=self._dev_t)
        # per raw peak, as Python floats for the sequential loop (same IEEE values)
        self._pkl = pk.tolist()
        self._envpk = env[pk].tolist()
        self._str = [max(0, e - f) for e, f in zip(self._envpk, floor[pk].tolist())]
        self._devl, self._dev_tl = self._dev.tolist(), self._dev_t.tolist()
        self.start_bpm = float(start_bpm_hint) if start_bpm_hint else 80.0

    # -- helpers --------------------------------------------------------
    def _dev_asof(self, t: float) -> float:
        """Series.asof on the smoothed deviations: last non-NaN value at index <= t."""
        d = self._devl
        k = bisect.bisect_right(self._dev_tl, t) - 1
        while k >= 0 and d[k] != d[k]:
            k -= 1
        return d[k] if k >= 0 else float("nan")

    def _pair(self, j: int, ratio: float, ltb: float, n_beats: int) -> Tuple[bool, str]:
        """Pairing decision for raw peaks #j and #j+1 (:231-272, :1146-1197)."""
        p, sr = self.params, self.sample_rate
        s1, s2 = self._pkl[j], self._pkl[j + 1]
        gap = (s2 - s1) / sr
        conf = calculate_blended_confidence(self._dev_asof(s1 / sr), ltb, p)
        why = f"Base Conf (Blended Model {_blend(ltb, p):.0%} High): {conf:.2f}"
        if n_beats >= 5:
            f = _interp(ratio, (0.0, 1.0), (p.get("stability_confidence_floor", 0.85),
                                            p.get("stability_confidence_ceiling", 1.10)))
            conf *= f
            why += f"\n- Stability Pre-Adjust: x{f:.2f} (Pairing Ratio: {ratio:.0%})"
        a1, a2 = self._str[j], self._str[j + 1]
        r21 = a2 / (a1 + 1e-9)
        lo = p['contractility_bpm_low']
        t1, t2 = self.peak_bpm_time_sec, self.recovery_end_time_sec
        recovering = t1 is not None and t2 is not None and t1 < (s1 / sr) < t2
        r_max = np.float64(_interp(max(ltb, lo) if recovering else ltb, (lo, p['contractility_bpm_high']),
                                   (p['s2_s1_ratio_low_bpm'], p['s2_s1_ratio_high_bpm'])))
        boost_at = p.get('s1_s2_boost_ratio', 1.2)
        if r21 > r_max:
            pmin, pmax = p.get("penalty_amount_min", 0.15), p.get("penalty_amount_max", 0.40)
            amt = pmin + _clip((r21 / r_max - 1.0) / 2.0, 0, 1) * (pmax - pmin)
            conf -= amt
            why += f"\n- PENALIZED by {amt:.2f} (S2 Str. Ratio {r21:.1f}x > Expected {r_max:.1f}x)"
        elif a1 > a2 * boost_at:
            bmin, bmax = p.get("boost_amount_min", 0.10), p.get("boost_amount_max", 0.35)
            r12 = a1 / (a2 + 1e-9)
            amt = bmin + _clip((r12 - boost_at) / (4.0 - boost_at), 0, 1) * (bmax - bmin)
            conf += amt
            why += f"\n- BOOSTED by {amt:.2f} (S1 Str. Ratio {r12:.1f}x > S2)"
        conf = max(0.0, min(1.0, conf))

        cap = min(p['s1_s2_interval_cap_sec'], (60.0 / ltb) * p['s1_s2_interval_rr_fraction'])
        if p.get("enable_interval_penalty", True) and gap > cap:
            z0 = cap * p.get("interval_penalty_start_factor", 1.0)
            z1 = cap * p.get("interval_penalty_full_factor", 1.4)
            if gap > z0:
                amt = _clip((gap - z0) / (z1 - z0 + 1e-9), 0, 1) * p.get("interval_max_penalty", 0.75)
                conf = max(0, conf - amt)
                why += f"\n- Interval PENALTY by {amt:.2f} (Interval {gap:.3f}s > Max {cap:.3f}s)"
        thr = p['pairing_confidence_threshold']
        ok = conf >= thr
        why += f"\n- Final Score: {conf:.2f} vs Threshold {thr:.2f} -> {'Paired' if ok else 'Not Paired'}"
        return ok, why

    def _lone(self, j: int, jl: int, ltb: float) -> Tuple[bool, str, bool]:
        """Lone-S1 validation of raw peak #j after the beat at raw peak #jl (:304-329, :1201-1237).
        Returns (valid, detail, rejected_on_rhythm)."""
        p, sr, env = self.params, self.sample_rate, self._envpk
        cur, last = self._pkl[j], self._pkl[jl]
        exp_rr = 60.0 / ltb
        rr = (cur - last) / sr
        rs = _interp(abs(rr - exp_rr) / exp_rr, _RHYTHM_X, _RHYTHM_Y)
        ar = self._str[j] / (self._str[jl] + 1e-9)
        am = _interp(ar, _AMP_X, _AMP_Y)
        wr, wa = p.get('lone_s1_rhythm_weight', 0.65), p.get('lone_s1_amplitude_weight', 0.35)
        conf = (rs * wr) + (am * wa)
        why = (f"Rhythm Fit={rs:.2f} (Interval {rr:.3f}s vs Expected {exp_rr:.3f}s), "
               f"Amplitude Fit={am:.2f} (Strength Ratio {ar:.2f}x)")
        thr = p.get("lone_s1_confidence_threshold", 0.6)
        if conf < thr:
            return False, f"Rejected Lone S1: Confidence {conf:.2f} < Threshold {thr:.2f}. ({why})", True
        if j < len(self._pkl) - 1:
            fwd = (self._pkl[j + 1] - cur) / sr
            if fwd < exp_rr * p.get('lone_s1_forward_check_pct', 0.6) and not (env[j] > (env[j + 1] * 1.7)):
                implied = 60.0 / fwd if fwd > 0 else float('inf')
                return False, f"Rejected Lone S1: Forward check failed (Implies {implied:.0f} BPM)", False
        return True, (f"Validated Lone S1: Confidence {conf:.3f} >= Threshold {thr:.2f}. ({why}, Weights: "
                      f"Rhythm={wr:.2f}, Amplitude={wa:.2f}, Final={conf:.3f})"), False

    # -- main loop ------------------------------------------------------
    def classify_peaks(self) -> Tuple[np.ndarray, np.ndarray, Dict]:
        """One left-to-right pass over the raw peaks (:113-221)."""
        pk, p, sr = self.peaks, self.params, self.sample_rate
        pkl = self._pkl
        n = len(pk)
        if n < 2:
            return pk, pk, {"beat_debug_info": {}}
        hist_w = p.get("stability_history_window", 20)
        kick_thr = p.get("kickstart_check_threshold", 0.3)
        cascade_at = p.get("cascade_reset_trigger_count", 3)
        tag = np.zeros(n, dtype=np.int8)          # per raw peak
        info: Dict = {}
        beats: List[int] = []                     # raw-peak numbers of the candidate beats
        paired: List[bool] = []                   # beat carries the "S1 (Paired)" label
        n_paired_win = 0                          # paired among the last hist_w beats
        ltb = self.start_bpm
        lt_hist: List[Tuple[float, float]] = []
        rr_fails = 0

        def add_beat(j: int, is_pair: bool):
            nonlocal n_paired_win
            beats.append(j)
            paired.append(is_pair)
            n_paired_win += is_pair
            if len(beats) > hist_w:
                n_paired_win -= paired[-hist_w - 1]

        j = 0
        while j < n:
            ratio = 0.5 if len(beats) < hist_w else n_paired_win / hist_w
            if ratio < kick_thr and len(beats) >= 4:
                self._kickstart_log(beats, tag)
            cur = pk[j]
            if j >= n - 1:
                add_beat(j, False)
                tag[j] = _T_LONE
                info[cur] = LONE_S1_LAST
                j += 1
            else:
                ok, why = self._pair(j, ratio, ltb, len(beats))
                if ok:
                    add_beat(j, True)
                    tag[j], tag[j + 1] = _T_S1, _T_S2
                    t = f"PAIRING_SUCCESS_REASON§{why}"
                    info[cur] = f"{S1_PAIRED}§{t}"
                    info[pk[j + 1]] = f"{S2_PAIRED}§{t}"
                    rr_fails = 0
                    j += 2
                else:
                    fail = f"PAIRING_FAIL_REASON§{why.lstrip(' |')}"
                    if not beats:
                        valid, detail, on_rhythm = True, "First beat", False
                    else:
                        valid, detail, on_rhythm = self._lone(j, beats[-1], ltb)
                    if valid:
                        add_beat(j, False)
                        tag[j] = _T_LONE
                        info[cur] = f"{LONE_S1}§{fail}§LONE_S1_VALIDATE_REASON§{detail}"
                        rr_fails = 0
                    else:
                        rr_fails = rr_fails + 1 if on_rhythm else 0
                        rej = f"LONE_S1_REJECT_REASON§{detail}"
                        if rr_fails >= cascade_at:
                            logging.info(f"CASCADE RESET: Forcing peak at {cur / sr:.2f}s as Lone S1 "
                                         f"due to repeated rhythmic failures.")
                            add_beat(j, False)
                            tag[j] = _T_LONE
                            info[cur] = f"{LONE_S1_CASCADE}§{fail}§{rej}"
                            rr_fails = 0
                        else:
                            tag[j] = _T_NOISE
                            info[cur] = f"Noise§{fail}§{rej}"
                    j += 1
            # long-term BPM belief after every decision, from the last two beats (:203-212)
            if len(beats) > 1:
                rr = (pkl[beats[-1]] - pkl[beats[-2]]) / sr
                if rr > 0:
                    ltb = update_long_term_bpm(rr, ltb, p)
            if beats:
                lt_hist.append((pk[beats[-1]] / sr, ltb))

        data = {"dynamic_noise_floor_series": self.noise_floor, "trough_indices": self.troughs,
                "deviation_series": self.deviation_series, "beat_debug_info": info}
        if lt_hist:
            tt, vv = zip(*lt_hist)
            data["long_term_bpm_series"] = pd.Series(vv, index=tt)
        s1 = np.array(sorted(pk[b] for b in beats))
        return s1, pk, data

    def _kickstart_log(self, beats: List[int], tag: np.ndarray) -> None:
        """The reference's kick-start check (:132-168) only logs: the override it
        stores is never read, so it cannot change a decision."""
        lone = [b for b in beats[-4:] if tag[b] == _T_LONE]
        if len(lone) < 3:
            return
        hits = sum(1 for b in lone if b < len(self.peaks) - 1 and tag[b + 1] == _T_NOISE)
        if hits >= 3:
            logging.info(f"KICK-START: Found {hits}/{len(lone)} S1->Noise patterns. Overriding pairing ratio to "
                         f"{self.params.get('kickstart_override_ratio', 0.6)}.")


# ---------------------------------------------------------------- BPM curve
_EPOCH = None


def _epoch():
    global _EPOCH
    if _EPOCH is None:
        _EPOCH = datetime.datetime.fromtimestamp(0)
    return _EPOCH


def bpm_series(peaks: np.ndarray, sample_rate: int, params: Dict) -> Tuple[pd.Series, np.ndarray]:
    """Instantaneous BPM between beats, centered time-window mean (:1463-1484).
    Returns (smoothed pd.Series on a naive-datetime index, beat times in s)."""
    if len(peaks) < 2:
        return pd.Series(dtype=np.float64), np.array([])
    t = peaks / sample_rate
    dt = np.diff(t)
    ok = dt > 1e-6
    if not np.any(ok):
        return pd.Series(dtype=np.float64), np.array([])
    bpm = 60.0 / dt[ok]
    t_ok = t[1:][ok]
    e = _epoch()
    s = pd.Series(bpm, index=[e + datetime.timedelta(seconds=x) for x in t_ok])
    if np.median(bpm) > 0:
        smooth = s.rolling(window=f"{params['output_smoothing_window_sec']}s", min_periods=1, center=True).mean()
    else:
        smooth = pd.Series(dtype=np.float64)
    return smooth, t_ok


calculate_bpm_series = bpm_series


def find_recovery_phase(bpm: pd.Series, t: np.ndarray, params: Dict) -> Tuple[Optional[float], Optional[float]]:
    """Peak-BPM time and the end of the high-contractility window after it (:1612-1620)."""
    if t is None or len(t) < 2:
        logging.warning("Not enough preliminary beats to determine a recovery phase.")
        return None, None
    t_pk = t[np.argmax(bpm.to_numpy())]
    return t_pk, t_pk + params.get("recovery_phase_duration_sec", 120.0)


def run_preliminary_pass(env, sr, params, floor, troughs, start_bpm_hint, raw_peaks=None):
    """Anchor pass at pairing threshold 0.75 -> (start_bpm, peak time, recovery end) (:1623-1652)."""
    p1 = dict(params)
    p1["pairing_confidence_threshold"] = 0.75
    anchors, raw, _ = PeakClassifier(env, sr, p1, start_bpm_hint, floor, troughs, None, None,
                                     raw_peaks=raw_peaks).classify_peaks()
    est = None
    if len(anchors) >= 10:
        med = np.median(np.diff(anchors) / sr)
        if med > 0:
            est = 60.0 / med
    start = start_bpm_hint or est or 80.0
    s, t = bpm_series(anchors, sr, params)
    t_pk, t_end = find_recovery_phase(s, t, params)
    return start, t_pk, t_end


# ---------------------------------------------------------------- refinement
def correct_peaks_by_rhythm(peaks: np.ndarray, audio_envelope: np.ndarray, sample_rate: int, params: Dict):
    """Drop the weaker of two beats closer than rr_correction_threshold_pct x median RR (:1257-1306)."""
    if len(peaks) < 5:
        return peaks
    thr = np.median(np.diff(peaks) / sample_rate) * params.get("rr_correction_threshold_pct", 0.6)
    kept = [peaks[0]]
    for q in peaks[1:]:
        if (q - kept[-1]) / sample_rate < thr:
            if audio_envelope[q] > audio_envelope[kept[-1]]:
                kept[-1] = q
        else:
            kept.append(q)
    return np.array(kept)


def fix_rhythmic_discontinuities(s1, raw, info: Dict, env, floor: np.ndarray, params: Dict, sr: int):
    """One gap-fill + short-interval pass (:1309-1412) -> (peaks, info, n_corrections)."""
    m = 3
    if len(s1) < 2 * m:
        return s1, info, 0
    rr = np.diff(s1) / sr
    q1, q3 = np.percentile(rr, [25, 75])
    iqr = q3 - q1
    stable = rr[(rr > (q1 - 1.5 * iqr)) & (rr < (q3 + 1.5 * iqr))]
    if len(stable) < 1:
        return s1, info, 0
    med = np.median(stable)
    short_thr = med * params["rr_correction_threshold_pct"]
    long_thr = med * params.get("rr_correction_long_interval_pct", 1.7)
    out = dict(info)
    added = set()
    n_fix = 0
    waiver, max_ratio = params["penalty_waiver_strength_ratio"], params["penalty_waiver_max_s2_s1_ratio"]
    for i in range(m, len(s1) - 1 - m):
        a, b = s1[i], s1[i + 1]
        if not (b - a) / sr > long_thr:
            continue
        lo, hi = np.searchsorted(raw, a, side="right"), np.searchsorted(raw, b, side="left")
        for k in range(lo, hi):                              # raw peaks strictly inside the gap
            c1 = raw[k]
            if "Noise" not in info.get(c1, "") or c1 in added or k + 1 >= len(raw):
                continue
            c2 = raw[k + 1]
            if c2 >= b or "Noise" not in info.get(c2, ""):
                continue
            if (max(0, env[c1] - floor[c1]) > waiver * floor[c1]
                    and (env[c2] / (env[c1] + 1e-9)) < max_ratio):
                n_fix += 1
                added.add(c1)
                out[c1] = f"{S1_GAP}§ORIGINAL_REASON§{out.get(c1, 'Noise')}"
                out[c2] = f"{S2_GAP}§ORIGINAL_REASON§{out.get(c2, 'Noise')}"
                break
    merged = sorted(set(s1) | added)
    drop = set()
    for i in range(m, len(merged) - 1 - m):
        a, b = merged[i], merged[i + 1]
        if a in drop or b in drop:
            continue
        if (b - a) / sr < short_thr:
            drop.add(a if env[b] > env[a] else b)
            n_fix += 1
    return np.array(sorted(q for q in merged if q not in drop)), out, n_fix


def refine_peaks(s1, raw, data: Dict, env, sr: int, params: Dict) -> Tuple[np.ndarray, Dict]:
    """Rhythm correction, then up to 5 discontinuity passes until stable (:1655-1698)."""
    floor = np.asarray(data['dynamic_noise_floor_series'].values, dtype=np.float64)
    peaks = correct_peaks_by_rhythm(s1, env, sr, params)
    info = data["beat_debug_info"].copy()
    for _ in range(5):
        peaks, info, n = fix_rhythmic_discontinuities(peaks, raw, info, env, floor, params, sr)
        if n == 0:
            break
    else:
        logging.warning("Correction process reached max iterations without stabilizing.")
    data["beat_debug_info"] = info
    return peaks, data


# ---------------------------------------------------------------- final metrics
def windowed_hrv(s1: np.ndarray, sr: int, params: Dict) -> pd.DataFrame:
    """RMSSDc / SDNN / BPM over sliding beat windows (:1414-1461)."""
    w, step = params['hrv_window_size_beats'], params['hrv_step_size_beats']
    cols = ['time', 'rmssdc', 'sdnn', 'bpm']
    if len(s1) < w:
        return pd.DataFrame(columns=cols)
    rr = np.diff(s1) / sr
    t = s1 / sr
    rows = []
    for i in range(0, len(rr) - w + 1, step):
        ms = rr[i:i + w] * 1000
        mean_s = np.mean(ms) / 1000.0
        rmssd = np.sqrt(np.mean(np.diff(ms) ** 2))
        rows.append({'time': (t[i] + t[i + w]) / 2.0, 'rmssdc': rmssd / mean_s if mean_s > 0 else 0,
                     'sdnn': np.std(ms), 'bpm': 60 / mean_s if mean_s > 0 else 0})
    return pd.DataFrame(rows) if rows else pd.DataFrame(columns=cols)


def _turning_points(s: pd.Series, min_duration_sec: float):
    from scipy.signal import find_peaks
    step = np.nanmean(s.index.to_series().diff().dt.total_seconds())
    dist = 5 if np.isnan(step) or step == 0 else int((min_duration_sec / 2) / step)
    v = s.values
    return find_peaks(v, prominence=5, distance=dist)[0], find_peaks(-v, prominence=5, distance=dist)[0]


def _runs(s: pd.Series, starts, ends, min_duration_sec, min_change, rising: bool) -> List[Dict]:
    out = []
    for a in starts:
        nxt = ends[ends > a]
        if len(nxt) == 0:
            continue
        b = nxt[0]
        t0, t1, v0, v1 = s.index[a], s.index[b], s.values[a], s.values[b]
        dur = (t1 - t0).total_seconds()
        change = v1 - v0 if rising else v0 - v1
        if dur >= min_duration_sec and change >= min_change:
            d = {'start_time': t0, 'end_time': t1, 'start_bpm': v0, 'end_bpm': v1, 'duration_sec': dur}
            d['bpm_increase' if rising else 'bpm_decrease'] = change
            d['slope_bpm_per_sec'] = (v1 - v0) / dur if not rising else change / dur
            out.append(d)
    out.sort(key=lambda x: x['slope_bpm_per_sec'], reverse=rising)
    return out


def find_major_hr_inclines(s: pd.Series, min_duration_sec: int = 10, min_bpm_increase: int = 15) -> List[Dict]:
    """Trough -> next peak runs of the smoothed BPM (:1486-1517)."""
    if s.empty or len(s) < 2:
        return []
    pk, tr = _turning_points(s, min_duration_sec)
    if len(tr) == 0 or len(pk) == 0:
        return []
    return _runs(s, tr, pk, min_duration_sec, min_bpm_increase, True)


def find_major_hr_declines(s: pd.Series, min_duration_sec: int = 10, min_bpm_decrease: int = 15) -> List[Dict]:
    """Peak -> next trough runs of the smoothed BPM (:1519-1550)."""
    if s.empty or len(s) < 2:
        return []
    pk, tr = _turning_points(s, min_duration_sec)
    if len(tr) == 0 or len(pk) == 0:
        return []
    return _runs(s, pk, tr, min_duration_sec, min_bpm_decrease, False)


def _steepest(s: pd.Series, window_sec: float, sign: float) -> Optional[Dict]:
    """Steepest window_sec slope (sign -1: fall, +1: rise); first end index at >= t_i + window."""
    t = np.asarray((s.index - s.index[0]).total_seconds())
    if t[-1] < window_sec:
        return None
    v, best, out = s.values, 0, None
    ends = np.searchsorted(t, t[:-1] + window_sec, side="left")
    for i in range(len(t) - 1):
        e = ends[i]
        if e >= len(t):
            break
        dur = t[e] - t[i]
        if dur > 0:
            sl = (v[e] - v[i]) / dur
            if sign * sl > sign * best:
                best = sl
                out = {'start_time': s.index[i], 'end_time': s.index[e], 'start_bpm': v[i], 'end_bpm': v[e],
                       'slope_bpm_per_sec': sl, 'duration_sec': dur}
    return out


def find_peak_recovery_rate(s: pd.Series, window_sec: int = 20) -> Optional[Dict]:
    """Steepest decline after the BPM maximum (:1552-1574)."""
    if s.empty or len(s) < 2:
        return None
    rec = s[s.idxmax():]
    return None if rec.empty else _steepest(rec, window_sec, -1.0)


def find_peak_exertion_rate(s: pd.Series, window_sec: int = 20) -> Optional[Dict]:
    """Steepest rise over the whole recording (:1576-1595)."""
    if s.empty or len(s) < 2:
        return None
    return _steepest(s, window_sec, 1.0)


def calculate_hrr(s: pd.Series, interval_sec: int = 60) -> Optional[Dict]:
    """Heart-rate recovery interval_sec after the maximum (:1597-1610)."""
    if s.empty or len(s) < 2:
        return None
    top, t_top = s.max(), s.idxmax()
    t_chk = t_top + pd.Timedelta(seconds=interval_sec)
    if t_chk > s.index.max():
        return None
    rec = np.interp(t_chk.timestamp(), (s.index.astype(np.int64) // 10**9).to_numpy(dtype=float),
                    np.asarray(s.values, dtype=float))
    return {'peak_bpm': top, 'peak_time': t_top, 'recovery_bpm': rec, 'recovery_check_time': t_chk,
            'hrr_value_bpm': top - rec, 'interval_sec': interval_sec}


def final_metrics(peaks: np.ndarray, sr: int, params: Dict) -> Dict:
    """BPM curve, slopes, HRR, HRV and the summary dict (:1701-1722)."""
    m: Dict = {}
    m['smoothed_bpm'], m['bpm_times'] = s, _ = bpm_series(peaks, sr, params)
    m['major_inclines'] = find_major_hr_inclines(s)
    m['major_declines'] = find_major_hr_declines(s)
    m['hrr_stats'] = calculate_hrr(s)
    m['peak_recovery_stats'] = find_peak_recovery_rate(s)
    m['peak_exertion_stats'] = find_peak_exertion_rate(s)
    m['windowed_hrv_df'] = h = windowed_hrv(peaks, sr, params)
    summ = {}
    if not s.empty:
        summ.update(avg_bpm=s.mean(), min_bpm=s.min(), max_bpm=s.max())
    if not h.empty:
        summ.update(avg_rmssdc=h['rmssdc'].mean(), avg_sdnn=h['sdnn'].mean())
    m['hrv_summary'] = summ
    return m


# ---------------------------------------------------------------- per-file orchestration
def analyze_recording(env: np.ndarray, sr: int, floor, troughs: np.ndarray, raw_peaks: np.ndarray,
                      params: Dict, start_bpm_hint: Optional[float] = None) -> Dict:
    """Stages 2-6 of analyze_wav_file (:1734-1757) on one recording's GPU outputs.

    Returns dict(final_peaks, s1_peaks, all_raw_peaks, analysis_data, final_metrics,
    start_bpm, peak_time, recovery_time); final_metrics is None when fewer than
    two beats survive (the reference stops there without a report)."""
    if not isinstance(floor, pd.Series):
        floor = pd.Series(np.asarray(floor, dtype=np.float64), index=np.arange(len(floor)))
    env = np.asarray(env, dtype=np.float64)
    start, t_pk, t_end = run_preliminary_pass(env, sr, params, floor, troughs, start_bpm_hint, raw_peaks)
    s1, raw, data = PeakClassifier(env, sr, params, start, floor, troughs, t_pk, t_end,
                                   raw_peaks=raw_peaks).classify_peaks()
    # < 2 raw peaks: classify_peaks returns without the floor, and refinement
    # raises KeyError('dynamic_noise_floor_series') exactly as the reference's does
    final, data = refine_peaks(s1, raw, data, env, sr, params)
    if len(final) < 2:
        logging.warning("Not enough S1 peaks detected to generate full report.")
        metrics = None
    else:
        metrics = final_metrics(final, sr, params)
    return {"final_peaks": final, "s1_peaks": s1, "all_raw_peaks": raw, "analysis_data": data,
            "final_metrics": metrics, "start_bpm": start, "peak_time": t_pk, "recovery_time": t_end}


def write_bpm_csv(path: str, metrics: Dict) -> bool:
    """``<base>_bpm_plot.csv``: 'Time (s)','Average BPM' rows to 3 decimals, NaN rows skipped (:458-473)."""
    s, t = metrics.get('smoothed_bpm'), metrics.get('bpm_times')
    if s is None or s.empty or t is None:
        return False
    with open(path, 'w', newline='', encoding='utf-8') as f:
        w = csv.writer(f)
        w.writerow(['Time (s)', 'Average BPM'])
        for x, b in zip(t, s.values):
            if not np.isnan(b):
                w.writerow([f"{x:.3f}", f"{b:.3f}"])
    return True


def analyze_wav_file(wav_file_path: str, params: Dict, start_bpm_hint: Optional[float], original_file_path: str,
                     output_directory: str, mode: Optional[str] = None, device: int = 0):
    """The reference entry point (:1725) on the GPU path: preprocess + floor + raw
    peaks in one batched run, then the host stages above; writes the filtered
    debug WAVs, ``<base>_bpm_plot.html`` (plot.py), ``<base>_bpm_plot.csv``
    and the ReportGenerator files (reports.py: summary, debug log, settings),
    in the reference's order.  Returns None."""
    from .dropin import analyze_wav_files
    r = analyze_wav_files([wav_file_path], params, output_directory, mode=mode, device=device)[0]
    if "error" in r:
        raise r["error"]
    res = analyze_recording(r["env"], r["sr"], r["floor"], r["troughs"], r["peaks"], params, start_bpm_hint)
    m = res["final_metrics"]
    if m is not None:
        from .plot import write_plot
        from .reports import write_reports
        env = np.asarray(r["env"], dtype=np.float64)
        write_plot(original_file_path, output_directory, params, r["sr"], env, res["all_raw_peaks"],
                   res["analysis_data"], m)
        base = os.path.basename(os.path.splitext(original_file_path)[0])
        write_bpm_csv(os.path.join(output_directory, f"{base}_bpm_plot.csv"), m)
        write_reports(original_file_path, output_directory, env, r["sr"], res["all_raw_peaks"],
                      res["analysis_data"], m, start_bpm_hint)
    return None


def _analyze_one(job):
    r, params, hint = job
    if "error" in r:
        return r
    try:
        return analyze_recording(r["env"], r["sr"], r["floor"], r["troughs"], r["peaks"], params, hint)
    except Exception as exc:                      # per-file, as the GUI's loop catches it (gui.py:247-251)
        return {"error": exc}


def analyze_many(results: Sequence[Dict], params: Dict, start_bpm_hint: Optional[float] = None,
                 workers: int = 1) -> List[Dict]:
    """``analyze_recording`` over the per-file dicts of a batched GPU run
    (dropin.analyze_batch / analyze_wav_files); entries with ``error`` pass
    through, and a file whose stages raise comes back as ``{"error": exc}``.

    The stages are sequential per file but files are independent: with
    ``workers > 1`` they run in that many CPU-only processes (spawned fresh, so
    they never touch the GPU context of this one), ``chunksize`` files at a time."""
    jobs = [({k: r[k] for k in ("env", "sr", "floor", "troughs", "peaks") if k in r} if "error" not in r else r,
             params, start_bpm_hint) for r in results]
    if workers <= 1 or len(jobs) < 2:
        return [_analyze_one(j) for j in jobs]
    import multiprocessing
    from concurrent.futures import ProcessPoolExecutor
    chunk = max(1, len(jobs) // (4 * workers))
    with ProcessPoolExecutor(max_workers=workers, mp_context=multiprocessing.get_context("spawn")) as ex:
        return list(ex.map(_analyze_one, jobs, chunksize=chunk))


def analyze_fast(results: Sequence[Dict], params: Dict, start_bpm_hint: Optional[float] = None,
                 threads: int = 1) -> List[Dict]:
    """The beat stages the batch path needs — preliminary pass, classifier,
    refinement and the smoothed BPM curve — as native code (libbpmx_host.so,
    include/bpmx_host.h) over the per-file dicts of a batched GPU run, on
    ``threads`` host threads (the C++ releases the GIL).  Per file:
    dict(final_peaks, bpm_times, bpm, start_bpm, peak_time, recovery_time,
    tags), or the entry's / the stage's ``error``.  The same beats and curve
    as ``analyze_recording`` (tests/test_host_beats.py); HRV, slopes, reports
    and the plot stay with analyze_recording."""
    from . import _host
    return _host.beats_batch(list(results), params, start_bpm_hint, threads=threads)
