"""Host-side derivations for one sample rate: the scalar part of the path.

Mirrors the reference's host logic before any per-sample work
(pixeru/bpm_analysis bpm_analysis.py):

* ``:1018-1029``  the downsample-factor clamp ``max_safe = int(fs/300 - 1)``
  (with the same two warnings);
* ``:1031-1036``  ``sr = fs // ds`` (integer; the true 302.05 Hz is ignored);
* ``:1038-1042``  the Nyquist check and its ``ValueError``;
* ``:1044``       ``butter(2, [20/nyq, 150/nyq], 'band')`` and, inside scipy's
  ``filtfilt``, ``lfilter_zi`` (a LAPACK solve) — computed here with scipy
  exactly as the reference's own call computes them, then handed to the
  kernels as plain doubles;
* ``:1053, :1066, :1084``  envelope window, peak distance, noise window.

Native mode additionally designs the same band-pass as second-order sections
at the native rate (``output='sos'`` + ``sosfilt_zi``) and the block-state
tables its kernels consume (see ``csrc/k_envelope_native.hip``).
"""
from __future__ import annotations

import functools
import logging
from dataclasses import dataclass, field

import numpy as np

from . import _native as N

LOWCUT, HIGHCUT = 20, 150   # hard-coded band, bpm_analysis.py:1018


@dataclass(frozen=True)
class Design:
    fs: int
    ds: int
    sr: int
    env_window: int
    distance: int
    noise_window: int
    b: tuple
    a: tuple
    zi: tuple
    sos: tuple
    sos_zi: tuple
    warnings: tuple = field(default=())


def clamp_downsample(fs: int, downsample_factor: int):
    """bpm_analysis.py:1021-1036 -> (ds, sr, warnings)."""
    ds = downsample_factor
    warns = []
    max_safe = int((fs / (HIGHCUT * 2)) - 1)
    if ds > max_safe:
        warns.append(f"Original 'downsample_factor' of {ds} is too high for a "
                     f"{HIGHCUT}Hz filter with a {fs}Hz sample rate.")
        ds = max(1, max_safe)
        warns.append(f"Adjusting 'downsample_factor' to a safe value of {ds}.")
    if ds > 1:
        sr = fs // ds
    else:
        sr = fs
        ds = 1
    return ds, sr, tuple(warns)


@functools.lru_cache(maxsize=64)
def _design(fs: int, downsample_factor: int, min_peak_distance_sec: float, noise_window_sec: float) -> Design:
    from scipy.signal import butter, lfilter_zi, sosfilt_zi

    ds, sr, warns = clamp_downsample(fs, downsample_factor)
    nyquist = 0.5 * sr
    low, high = LOWCUT / nyquist, HIGHCUT / nyquist
    if high >= 1.0:
        raise ValueError(f"Cannot create a {HIGHCUT}Hz filter. The effective sample rate of {sr}Hz is too low.")
    b, a = butter(2, [low, high], btype="band")
    zi = lfilter_zi(b, a)
    nyq_n = 0.5 * fs
    sos = butter(2, [LOWCUT / nyq_n, HIGHCUT / nyq_n], btype="band", output="sos")
    szi = sosfilt_zi(sos)
    return Design(fs=fs, ds=ds, sr=sr, env_window=sr // 10,
                  distance=int(min_peak_distance_sec * sr), noise_window=int(noise_window_sec * sr),
                  b=tuple(float(v) for v in b), a=tuple(float(v) for v in a), zi=tuple(float(v) for v in zi),
                  sos=tuple(float(v) for v in np.asarray(sos).ravel()),
                  sos_zi=tuple(float(v) for v in np.asarray(szi).ravel()), warnings=warns)


def detect_design(sr: int, params: dict) -> Design:
    """Detection-only derivations for an envelope already at rate `sr`
    (bpm_analysis.py:1066, :1084, :226); no filter is designed."""
    z5, z4, z12 = (0.0,) * 5, (0.0,) * 4, (0.0,) * 12
    return Design(fs=int(sr), ds=1, sr=int(sr), env_window=int(sr) // 10,
                  distance=int(params["min_peak_distance_sec"] * sr),
                  noise_window=int(params["noise_window_sec"] * sr), b=z5, a=z5, zi=z4, sos=z12, sos_zi=z4)


def design(fs: int, params: dict, log: bool = True) -> Design:
    d = _design(int(fs), params["downsample_factor"], params["min_peak_distance_sec"], params["noise_window_sec"])
    if log:
        for w in d.warnings:
            logging.warning(w)
    return d


def dtype_code(dt) -> int:
    dt = np.dtype(dt)
    table = {np.dtype(np.uint8): N.DT_U8, np.dtype(np.int16): N.DT_I16, np.dtype(np.int32): N.DT_I32,
             np.dtype(np.float32): N.DT_F32, np.dtype(np.float64): N.DT_F64}
    if dt not in table:
        raise TypeError(f"unsupported sample format {dt} (scipy.io.wavfile gives u8/i16/i32/f32/f64)")
    return table[dt]


def make_params(d: Design, params: dict, mode: int, stages: int, dtype: int, channels: int) -> N.Params:
    p = N.Params()
    p.mode, p.stages, p.dtype, p.channels = mode, stages, dtype, channels
    p.fs, p.ds, p.sr = d.fs, d.ds, d.sr
    p.env_window, p.distance, p.noise_window = d.env_window, d.distance, d.noise_window
    p.min_periods = 3                                   # bpm_analysis.py:1085, :1105
    p.trough_prom_q = float(params["trough_prominence_quantile"])
    p.peak_prom_q = float(params["peak_prominence_quantile"])
    p.noise_floor_q = float(params["noise_floor_quantile"])
    p.fallback_q = 0.1                                  # bpm_analysis.py:1114
    p.reject_mult = float(params.get("trough_rejection_multiplier", 4.0))
    p.ba_b[:] = d.b
    p.ba_a[:] = d.a
    p.ba_zi[:] = d.zi
    p.sos[:] = d.sos
    p.sos_zi[:] = d.sos_zi
    return p
