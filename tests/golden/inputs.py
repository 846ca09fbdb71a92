"""Deterministic inputs for the golden vectors and the parity tests.

Every input is built from the integer-only synthetic generator
(``bpm_analysis_amd/csrc/bpmx_synth.h``, exposed through the oracle's
``bpmo_synth``) plus integer numpy transforms, so it is bit-identical in the
build container and on the GPU box.  ``make_goldens.py`` records a sha256 of
each PCM array; the tests regenerate the array and check the hash first.
"""
from __future__ import annotations

import os
import sys

import numpy as np

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _REPO not in sys.path:
    sys.path.insert(0, _REPO)


def _synth(seed, n, fs, ch):
    from oracle import oracle as O
    return O.synth(seed, n, fs, ch)


def _hash_u32(seed: int, n: int) -> np.ndarray:
    z = (np.arange(n, dtype=np.uint64) + np.uint64(seed) * np.uint64(0x9E3779B9)) * np.uint64(0xBF58476D1CE4E5B9)
    z ^= z >> np.uint64(31)
    z *= np.uint64(0x94D049BB133111EB)
    z ^= z >> np.uint64(29)
    return (z & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def make_input(spec: dict):
    """spec -> (pcm ndarray, fs)."""
    fs = int(spec["fs"])
    ch = int(spec.get("channels", 1))
    n = int(spec["n_frames"]) if "n_frames" in spec else int(round(spec["secs"] * fs))
    pcm = _synth(int(spec["seed"]), n, fs, ch)
    t = spec.get("transform", "none")
    if t == "clicks":
        # sparse loud clicks (every ~0.9 s): they lift some troughs far above the
        # local noise floor, so the sanitize step (bpm_analysis.py:1090-1097) rejects them
        p = pcm.astype(np.int32)
        h = _hash_u32(int(spec["seed"]) + 77, n)
        period = int(0.9 * fs)
        for c0 in range(period // 3, n - fs // 5, period):
            c = c0 + int(h[c0] % (fs // 4))
            L = fs // 6
            sl = slice(c, min(n, c + L))
            amp = 9000 + int(h[c] % 9000)
            k = np.arange(sl.stop - sl.start)
            burst = (amp * ((k * 3) % 17 - 8) // 8)
            if p.ndim == 1:
                p[sl] += burst
            else:
                p[sl, :] += burst[:, None]
        pcm = np.clip(p, -32768, 32767).astype(np.int16)
    elif t == "wrap":
        # decimated edge samples near full scale: the odd-extension pad
        # 2*x0 - x[k] overflows int16 and must wrap (scipy _arraytools.py:57-107)
        ds = int(spec["ds"])
        pcm = pcm.copy()
        pcm[0] = 30000
        for k in range(1, 17):
            pcm[k * ds] = -20000 - 500 * k
        pcm[-1] = -31000
        last = n - 1
        for k in range(1, 17):
            pcm[last - k * ds] = 25000 - 100 * k
    elif t == "zeros":
        pcm = np.zeros_like(pcm)
    dt = spec.get("dtype", "int16")
    if dt == "uint8":
        pcm = ((pcm.astype(np.int32) >> 8) + 128).astype(np.uint8)
    elif dt == "int32":
        h = _hash_u32(int(spec["seed"]) + 5, pcm.size).reshape(pcm.shape)
        pcm = ((pcm.astype(np.int64) << 16) | (h & 0xFFFF).astype(np.int64)).astype(np.int32)
    elif dt == "float32":
        pcm = (pcm.astype(np.float32) / np.float32(32768.0)).astype(np.float32)
    elif dt == "float64":
        pcm = pcm.astype(np.float64) / 32768.0
    return np.ascontiguousarray(pcm), fs


# name, spec, mode, param overrides, store pcm in the fixture
CASES = [
    ("ref_44k_60s_mono", dict(seed=0, secs=60, fs=44100), "reference", None, False),
    ("ref_48k_20s_mono", dict(seed=1, secs=20, fs=48000), "reference", None, False),
    ("ref_44k_15s_stereo", dict(seed=2, secs=15, fs=44100, channels=2), "reference", None, False),
    ("ref_96k_20s_stereo", dict(seed=3, secs=20, fs=96000, channels=2), "reference", None, False),
    ("ref_22k_30s_mono", dict(seed=4, secs=30, fs=22050), "reference", None, False),
    ("ref_44k_40s_clicks", dict(seed=5, secs=40, fs=44100, transform="clicks"), "reference", None, False),
    ("ref_44k_20s_wrap", dict(seed=6, secs=20, fs=44100, transform="wrap", ds=146), "reference", None, False),
    ("ref_44k_10s_zeros", dict(seed=7, secs=10, fs=44100, transform="zeros"), "reference", None, False),
    ("ref_44k_12s_u8", dict(seed=8, secs=12, fs=44100, dtype="uint8"), "reference", None, False),
    ("ref_44k_12s_i32", dict(seed=9, secs=12, fs=44100, dtype="int32"), "reference", None, False),
    ("ref_44k_12s_f32", dict(seed=10, secs=12, fs=44100, dtype="float32"), "reference", None, False),
    ("ref_44k_12s_f32_stereo", dict(seed=11, secs=12, fs=44100, dtype="float32", channels=2), "reference", None, False),
    ("ref_44k_12s_f64", dict(seed=12, secs=12, fs=44100, dtype="float64"), "reference", None, False),
    ("ref_44k_short16", dict(seed=13, n_frames=146 * 15 + 1, fs=44100), "reference", None, False),
    ("ref_44k_30s_params", dict(seed=14, secs=30, fs=44100), "reference",
     dict(downsample_factor=100, min_peak_distance_sec=0.08, peak_prominence_quantile=0.2,
          trough_prominence_quantile=0.05, noise_floor_quantile=0.3, noise_window_sec=6,
          trough_rejection_multiplier=2.5), False),
    ("nat_44k_60s_mono", dict(seed=0, secs=60, fs=44100), "native", None, False),
    ("nat_96k_20s_stereo", dict(seed=3, secs=20, fs=96000, channels=2), "native", None, False),
    ("nat_44k_40s_clicks", dict(seed=5, secs=40, fs=44100, transform="clicks"), "native", None, False),
    ("nat_48k_20s_mono", dict(seed=1, secs=20, fs=48000), "native", None, False),
]


def _vshape(knots_pos, knots_val, n):
    return np.interp(np.arange(n), knots_pos, knots_val)


def env_cases() -> dict:
    """Synthetic envelopes that drive the noise-floor branches directly."""
    out = {}
    sr = 302
    # static fallback: fewer than 5 troughs (bpm_analysis.py:1073-1077)
    pos = [0, 200, 400, 600, 800, 999]
    val = [10.0, 900.0, 40.0, 1000.0, 30.0, 800.0]
    out["env_static_fallback"] = (_vshape(pos, val, 1000), sr, None)
    # draft-floor fallback: >= 5 troughs but <= 2 survive sanitisation (:1107-1110)
    pos, val = [0], [5000.0]
    troughs = [(100, 1.0), (600, 1.0), (700, 1000.0), (800, 1000.0), (900, 1000.0), (1000, 1000.0)]
    for (p, v) in troughs:
        pos += [p - 25, p]
        val += [v + 5000.0, v]
        pos += [p + 25]
        val += [v + 5000.0]
    pos += [1099]
    val += [5000.0]
    order = np.argsort(pos, kind="stable")
    out["env_draft_fallback"] = (_vshape(np.array(pos)[order], np.array(val)[order], 1100), sr, None)
    # plateaus (flat tops / flat bottoms) exercising the midpoint rule of _local_maxima_1d
    # (every run has its own height, so no two maxima tie: numpy's argsort order
    # for exactly equal heights is implementation-defined — see DESIGN.md)
    rng = np.random.default_rng(99)
    runs = []
    for r in range(1400):
        runs.append(np.full(int(rng.integers(1, 6)), 50.0 * int(rng.integers(4, 40)) + 1e-3 * r))
    out["env_plateaus"] = (np.concatenate(runs)[:4000], sr, None)
    # random smooth envelope with a long noise window (W > Nd)
    rng = np.random.default_rng(1234)
    r = np.abs(np.convolve(rng.standard_normal(2500), np.ones(25) / 25.0, mode="same")) * 1000.0
    out["env_random_long_window"] = (r, sr, dict(noise_window_sec=20))
    r2 = np.abs(np.convolve(rng.standard_normal(9000), np.ones(9) / 9.0, mode="same")) * 100.0 + 1.0
    out["env_random_rough"] = (r2, sr, None)
    out.update(tie_env_cases())
    return out


def _tie_pairs(seed: int, n_groups: int = 100) -> np.ndarray:
    """Piecewise-linear envelope whose local maxima come in pairs closer than
    find_peaks' distance (15 samples at 302 Hz), and whose minima (the troughs
    find_peaks(-env) sees) come in pairs too.  Within a pair both extrema sit
    on integer knots, and in three groups of four their values are exactly
    equal: the distance filter then meets two equal priorities, and
    numpy's argsort (bpm_analysis.py:1070, :227 -> scipy _peak_finding.py:976-978)
    decides which one stays."""
    h = _hash_u32(seed, 8 * n_groups).astype(np.int64)
    pos, val = [0], [60.0]
    x = 12
    for g in range(n_groups):
        u = h[8 * g: 8 * g + 8]
        hp = 400 + 10 * int(u[0] % 40)                    # peak pair height
        hp2 = hp if u[1] % 4 else hp + 1 + int(u[1] % 7)  # equal in 3 of 4 groups
        sep = 4 + int(u[2] % 10)                          # 4..13 samples apart
        dip = hp - 40 - int(u[3] % 120)
        lo = 20 + int(u[4] % 25)                          # trough pair depth
        lo2 = lo if u[5] % 4 else lo + 1 + int(u[5] % 5)
        tsep = 4 + int(u[6] % 10)
        bump = lo + 15 + int(u[7] % 30)
        pos += [x, x + sep // 2, x + sep]
        val += [float(hp), float(dip), float(hp2)]
        x += sep + 9 + int(u[0] % 7)
        pos += [x, x + tsep // 2, x + tsep]
        val += [float(lo), float(bump), float(lo2)]
        x += tsep + 9 + int(u[3] % 7)
    pos.append(x + 10)
    val.append(60.0)
    return _vshape(np.array(pos), np.array(val), x + 11)


def _quantized_labeler_env(seed: int, secs: int = 40) -> np.ndarray:
    """The labeler's envelope recipe (heartbeat_labeler.py:63-67: centred
    rolling mean of |x| over sr // 10 samples) on coarsely quantized and
    clipped PCM: the synthetic recording picked at 302 Hz, shifted down to
    small integers and clipped at +-12, so every envelope value is k / 30 and
    equal-height extrema within `distance` are common."""
    x = _synth(seed, secs * 44100, 44100, 1)[::146].astype(np.int64)
    q = np.clip(x >> 9, -12, 12).astype(np.float64)
    import pandas as pd
    return pd.Series(np.abs(q)).rolling(window=30, min_periods=1, center=True).mean().values


def tie_env_cases() -> dict:
    """Envelopes with exact height ties inside find_peaks' distance filter, for
    the decisive-tie report (BPMX_F_TROUGH_TIE / BPMX_F_PEAK_TIE)."""
    sr = 302
    return {
        "env_ties_pairs": (_tie_pairs(41), sr, None),
        "env_ties_quantized": (_quantized_labeler_env(42), sr, None),
        "env_ties_quantized_b": (_quantized_labeler_env(43, 60), sr, dict(trough_rejection_multiplier=2.0)),
    }
