"""CPU oracle for the bpm_analysis hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
import this module, and only as the checker / baseline.  The product package
``bpm_analysis_amd`` never imports it.

Python side of the restatement in ``bpmx_oracle.c``.  Host-level logic is
restated from the reference (pixeru/bpm_analysis @ 2025-07-25):

* ``bpm_analysis.py:1018-1044``  ds clamp, decimated rate, Nyquist check, butter design
* ``bpm_analysis.py:1064-1117``  noise floor (C), ``:223-229`` raw peaks (C)
* native mode (north_star ordering): sosfiltfilt at the
  native rate (C) -> ``y[::ds]`` -> ``|scipy.signal.hilbert|`` restated with
  ``numpy.fft`` (``scipy/signal/_signaltools.py:2318``) -> rolling mean (C).

Filter coefficients come from ``scipy.signal.butter`` / ``lfilter_zi`` /
``sosfilt_zi`` exactly as the reference calls them (host scalars).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "libbpmx_oracle.so")

DT = {np.dtype(np.uint8): 0, np.dtype(np.int16): 1, np.dtype(np.int32): 2,
      np.dtype(np.float32): 3, np.dtype(np.float64): 4}

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        P, I64, D, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_int
        L.bpmo_synth.argtypes = [ctypes.c_uint64, I64, ctypes.c_int32, I, P]
        L.bpmo_synth.restype = I
        L.bpmo_preprocess_ref.argtypes = [P, I, I64, I, I64, P, P, P, I64, P, P]
        L.bpmo_preprocess_ref.restype = I64
        L.bpmo_sosfiltfilt.argtypes = [P, I, I64, I, P, P, P]
        L.bpmo_sosfiltfilt.restype = I
        L.bpmo_rolling_mean.argtypes = [P, I64, I64, I64, P]
        L.bpmo_rolling_quantile.argtypes = [P, I64, I64, I64, D, P]
        L.bpmo_interp_dense.argtypes = [P, I64, P, I64, P]
        L.bpmo_quantile.argtypes = [P, I64, D]
        L.bpmo_quantile.restype = D
        L.bpmo_find_peaks.argtypes = [P, I64, D, P, I64, D, P]
        L.bpmo_find_peaks.restype = I64
        L.bpmo_find_peaks_ex.argtypes = [P, I64, D, P, I64, D, P, ctypes.POINTER(I)]
        L.bpmo_find_peaks_ex.restype = I64
        L.bpmo_prominence.argtypes = [P, I64, D, I64]
        L.bpmo_prominence.restype = D
        L.bpmo_raw_peaks_ex.argtypes = [P, I64, P, I64, D, P, ctypes.POINTER(I)]
        L.bpmo_raw_peaks_ex.restype = I64
        L.bpmo_noise_floor.argtypes = [P, I64, P, P, P, ctypes.POINTER(I)]
        L.bpmo_noise_floor.restype = I64
        L.bpmo_raw_peaks.argtypes = [P, I64, P, I64, D, P]
        L.bpmo_raw_peaks.restype = I64
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class _NF(ctypes.Structure):
    _fields_ = [("distance", ctypes.c_int64), ("noise_window", ctypes.c_int64),
                ("min_periods", ctypes.c_int64), ("trough_prom_q", ctypes.c_double),
                ("noise_floor_q", ctypes.c_double), ("reject_mult", ctypes.c_double),
                ("fallback_q", ctypes.c_double)]


# ----------------------------------------------------------------------------
# synthetic input
# ----------------------------------------------------------------------------
def synth(seed: int, n_frames: int, fs: int, channels: int = 1) -> np.ndarray:
    out = np.empty((n_frames, channels) if channels > 1 else (n_frames,), dtype=np.int16)
    lib().bpmo_synth(seed, n_frames, fs, channels, _p(out))
    return out


# ----------------------------------------------------------------------------
# host-level derivations (bpm_analysis.py:1018-1044, :1053, :1066, :1084)
# ----------------------------------------------------------------------------
@dataclass
class Derived:
    fs: int
    ds: int
    sr: int
    env_w: int
    distance: int
    noise_window: int
    b: np.ndarray
    a: np.ndarray
    zi: np.ndarray
    sos: np.ndarray
    sos_zi: np.ndarray


def derive(fs: int, params: dict) -> Derived:
    from scipy.signal import butter, lfilter_zi, sosfilt_zi
    ds = params["downsample_factor"]
    lowcut, highcut = 20, 150
    max_safe = int((fs / (highcut * 2)) - 1)
    if ds > max_safe:
        ds = max(1, max_safe)
    sr = fs // ds if ds > 1 else fs
    nyq = 0.5 * sr
    low, high = lowcut / nyq, highcut / nyq
    if high >= 1.0:
        raise ValueError(f"Cannot create a {highcut}Hz filter. The effective sample rate of {sr}Hz is too low.")
    b, a = butter(2, [low, high], btype="band")
    zi = lfilter_zi(b, a)
    nyq_n = 0.5 * fs
    sos = butter(2, [lowcut / nyq_n, highcut / nyq_n], btype="band", output="sos")
    szi = sosfilt_zi(sos)
    return Derived(fs=fs, ds=max(1, ds), sr=sr, env_w=sr // 10,
                   distance=int(params["min_peak_distance_sec"] * sr),
                   noise_window=int(params["noise_window_sec"] * sr),
                   b=np.ascontiguousarray(b, dtype=np.float64), a=np.ascontiguousarray(a, dtype=np.float64),
                   zi=np.ascontiguousarray(zi, dtype=np.float64),
                   sos=np.ascontiguousarray(sos, dtype=np.float64), sos_zi=np.ascontiguousarray(szi, dtype=np.float64))


# ----------------------------------------------------------------------------
# stages
# ----------------------------------------------------------------------------
def preprocess_ref(pcm: np.ndarray, d: Derived, return_y: bool = False):
    """preprocess_audio minus I/O (bpm_analysis.py:1007-1062) -> env (and y)."""
    pcm = np.ascontiguousarray(pcm)
    ch = 1 if pcm.ndim == 1 else pcm.shape[1]
    n = pcm.shape[0]
    nd = -(-n // d.ds)
    y = np.empty(max(nd, 1))
    env = np.empty(max(nd, 1))
    r = lib().bpmo_preprocess_ref(_p(pcm), DT[pcm.dtype], n, ch, d.ds, _p(d.b), _p(d.a), _p(d.zi), d.env_w,
                                  _p(y), _p(env))
    if r < 0:
        raise ValueError("The length of the input vector x must be greater than padlen, which is 15.")
    return (env[:nd], y[:nd]) if return_y else env[:nd]


def rolling_mean(v: np.ndarray, w: int, minp: int = 1) -> np.ndarray:
    v = np.ascontiguousarray(v, dtype=np.float64)
    out = np.empty_like(v)
    lib().bpmo_rolling_mean(_p(v), v.size, w, minp, _p(out))
    return out


def hilbert_abs(x: np.ndarray) -> np.ndarray:
    """|scipy.signal.hilbert(x)| restated with numpy.fft (_signaltools.py:2318-2400)."""
    n = x.shape[-1]
    xf = np.fft.fft(x, n)
    h = np.zeros(n)
    if n % 2 == 0:
        h[0] = h[n // 2] = 1
        h[1:n // 2] = 2
    else:
        h[0] = 1
        h[1:(n + 1) // 2] = 2
    return np.abs(np.fft.ifft(xf * h))


def preprocess_native(pcm: np.ndarray, d: Derived, return_y: bool = False):
    """north_star ordering: sosfiltfilt @ fs -> [::ds] -> |hilbert| -> rolling mean."""
    pcm = np.ascontiguousarray(pcm)
    ch = 1 if pcm.ndim == 1 else pcm.shape[1]
    n = pcm.shape[0]
    y = np.empty(n)
    r = lib().bpmo_sosfiltfilt(_p(pcm), DT[pcm.dtype], n, ch, _p(d.sos), _p(d.sos_zi), _p(y))
    if r < 0:
        raise ValueError("The length of the input vector x must be greater than padlen, which is 15.")
    yd = np.ascontiguousarray(y[::d.ds])
    env = rolling_mean(hilbert_abs(yd), d.env_w, 1)
    return (env, yd) if return_y else env


def quantile(x: np.ndarray, q: float) -> float:
    x = np.ascontiguousarray(x, dtype=np.float64)
    return lib().bpmo_quantile(_p(x), x.size, q)


# per-file flag bits of the decisive-tie report (include/bpmx.h BPMX_F_TROUGH_TIE / BPMX_F_PEAK_TIE)
F_TROUGH_TIE = 32
F_PEAK_TIE = 64


def find_peaks(x: np.ndarray, height=None, distance: int = 0, prominence=None, negate: bool = False,
               return_tie: bool = False):
    """scipy.signal.find_peaks(sign*x, height, distance, prominence) with the stable
    tie order (bpmx_oracle.c); with return_tie also whether that order decided
    anything in the distance filter (see bpmo_find_peaks_ex)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty(x.size // 2 + 2, dtype=np.int64)
    h = None if height is None else np.ascontiguousarray(height, dtype=np.float64)
    tie = ctypes.c_int(0)
    m = lib().bpmo_find_peaks_ex(_p(x), x.size, -1.0 if negate else 1.0, None if h is None else _p(h),
                                 distance, np.nan if prominence is None else float(prominence), _p(out),
                                 ctypes.byref(tie))
    pk = out[:m].copy()
    return (pk, bool(tie.value)) if return_tie else pk


def find_peaks_numpy_order(x: np.ndarray, height=None, distance: int = 0, prominence=None,
                           negate: bool = False) -> np.ndarray:
    """find_peaks with the distance filter visiting numpy's default argsort
    order, as the reference's own call does on this machine: local maxima and
    height from bpmx_oracle.c, the distance filter by select_by_peak_distance,
    prominences by bpmo_prominence.  Pins the stable-order restatement on tie
    inputs (tests/test_oracle.py); small cases only."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    sg = -1.0 if negate else 1.0
    cand = find_peaks(x, height=height, negate=negate)
    if distance and cand.size:
        cand = cand[select_by_peak_distance(cand, sg * x[cand], distance, "numpy")]
    if prominence is not None:
        cand = np.array([p for p in cand if float(prominence) <= lib().bpmo_prominence(_p(x), x.size, sg, int(p))],
                        dtype=np.int64)
    return cand


def select_by_peak_distance(peaks: np.ndarray, priority: np.ndarray, distance: int, order: str = "numpy"):
    """scipy _peak_finding_utils._select_by_peak_distance restated in Python
    (scipy/signal/_peak_finding.py:976-980 calls it; its loop: visit
    ``np.argsort(priority)`` from the end, a kept peak removes every peak
    closer than ceil(distance) on both sides).  ``order="numpy"`` takes
    numpy's default (unstable) argsort exactly as the reference does, on this
    machine's numpy; ``"stable"`` is the convention of bpmx_oracle.c and the
    kernels.  Pure-Python loop: small cases only (tie pinning tests)."""
    peaks = np.asarray(peaks, dtype=np.int64)
    pr = np.asarray(priority, dtype=np.float64)
    d = int(np.ceil(distance))
    keep = np.ones(peaks.size, dtype=bool)
    idx = np.argsort(pr) if order == "numpy" else np.argsort(pr, kind="stable")
    for i in range(peaks.size - 1, -1, -1):
        j = int(idx[i])
        if not keep[j]:
            continue
        k = j - 1
        while k >= 0 and peaks[j] - peaks[k] < d:
            keep[k] = False
            k -= 1
        k = j + 1
        while k < peaks.size and peaks[k] - peaks[j] < d:
            keep[k] = False
            k += 1
    return keep


def interp_dense(troughs: np.ndarray, env: np.ndarray) -> np.ndarray:
    t = np.ascontiguousarray(troughs, dtype=np.int64)
    env = np.ascontiguousarray(env, dtype=np.float64)
    out = np.empty(env.size)
    lib().bpmo_interp_dense(_p(t), t.size, _p(env), env.size, _p(out))
    return out


def rolling_quantile(v: np.ndarray, w: int, minp: int, q: float) -> np.ndarray:
    """rolling(w, minp, center=True).quantile(q).bfill().ffill()"""
    v = np.ascontiguousarray(v, dtype=np.float64)
    out = np.empty_like(v)
    lib().bpmo_rolling_quantile(_p(v), v.size, w, minp, q, _p(out))
    return out


def noise_floor_from_raw(env: np.ndarray, raw: np.ndarray, d: Derived, params: dict):
    """_calculate_dynamic_noise_floor after its trough search (bpm_analysis.py:1073-1117)
    from a given raw trough list -> (floor, troughs, flags): the static fallback
    (< 5 troughs), the draft floor (interp + centred rolling quantile +
    bfill/ffill), the sanitize loop, the final floor or the draft fallback, the
    all-NaN fallback.  Composes this module's C restatements; used with
    find_peaks_numpy_order's troughs (noise_floor_numpy_order)."""
    env = np.ascontiguousarray(env, dtype=np.float64)
    raw = np.asarray(raw, dtype=np.int64)
    q = params["noise_floor_quantile"]
    if raw.size < 5:                                                          # :1073-1077
        return np.full(env.size, quantile(env, q)), raw, 1
    draft = rolling_quantile(interp_dense(raw, env), d.noise_window, 3, q)   # :1081-1086
    mult = params.get("trough_rejection_multiplier", 4.0)
    kept = np.array([t for t in raw if not np.isnan(draft[t]) and env[t] <= mult * draft[t]], dtype=np.int64)
    flags = 0
    if kept.size > 2:                                                         # :1101-1106
        floor = rolling_quantile(interp_dense(kept, env), d.noise_window, 3, q)
    else:                                                                     # :1107-1110
        floor, flags = draft, 2
    if np.isnan(floor).all():                                                 # :1113-1115
        floor, flags = np.full(env.size, quantile(env, 0.1)), flags | 4
    return floor, kept, flags


def noise_floor_numpy_order(env: np.ndarray, d: Derived, params: dict):
    """_calculate_dynamic_noise_floor with its trough search in numpy's argsort
    order (find_peaks_numpy_order), i.e. the reference's answer on this
    machine when a decisive tie decides the troughs -> (floor, troughs, flags,
    raw troughs).  Small cases only."""
    env = np.ascontiguousarray(env, dtype=np.float64)
    raw = find_peaks_numpy_order(env, distance=d.distance, negate=True,
                                 prominence=quantile(env, params["trough_prominence_quantile"]))
    floor, kept, flags = noise_floor_from_raw(env, raw, d, params)
    return floor, kept, flags, raw


def noise_floor(env: np.ndarray, d: Derived, params: dict):
    """_calculate_dynamic_noise_floor -> (floor f64, troughs i64, flags)."""
    env = np.ascontiguousarray(env, dtype=np.float64)
    n = env.size
    nf = _NF(d.distance, d.noise_window, 3, params["trough_prominence_quantile"], params["noise_floor_quantile"],
             params.get("trough_rejection_multiplier", 4.0), 0.1)
    floor = np.empty(n)
    tr = np.empty(n // 2 + 2, dtype=np.int64)
    flags = ctypes.c_int(0)
    m = lib().bpmo_noise_floor(_p(env), n, ctypes.byref(nf), _p(floor), _p(tr), ctypes.byref(flags))
    return floor, tr[:m].copy(), flags.value


def raw_peaks(env: np.ndarray, floor: np.ndarray, d: Derived, params: dict, return_tie: bool = False):
    env = np.ascontiguousarray(env, dtype=np.float64)
    floor = np.ascontiguousarray(floor, dtype=np.float64)
    out = np.empty(env.size // 2 + 2, dtype=np.int64)
    tie = ctypes.c_int(0)
    m = lib().bpmo_raw_peaks_ex(_p(env), env.size, _p(floor), d.distance, params["peak_prominence_quantile"],
                                _p(out), ctypes.byref(tie))
    return (out[:m].copy(), bool(tie.value)) if return_tie else out[:m].copy()


def detect(pcm: np.ndarray, fs: int, params: dict, mode: str = "reference"):
    """Whole hot path for one recording -> dict(env, floor, troughs, peaks, sr, flags)."""
    d = derive(fs, params)
    if mode == "reference":
        env, y = preprocess_ref(pcm, d, return_y=True)
    else:
        env, y = preprocess_native(pcm, d, return_y=True)
    floor, troughs, flags = noise_floor(env, d, params)
    peaks, ptie = raw_peaks(env, floor, d, params, return_tie=True)
    flags |= F_PEAK_TIE if ptie else 0
    return dict(env=env, y=y, floor=floor, troughs=troughs, peaks=peaks, sr=d.sr, flags=flags)
