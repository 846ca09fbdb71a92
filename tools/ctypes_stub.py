"""The reference-side binding of libbpmx.so: what a bpm_analysis maintainer
would add next to bpm_analysis.py to call the C ABI (include/bpmx.h) directly.
It needs only ctypes, numpy, scipy and the HIP runtime (libamdhip64.so) for
device memory: no torch and no bpm_analysis_amd package.

    import ctypes_stub as bpmx
    env, floor, troughs, peaks, sr = bpmx.analyze(pcm_int16, 44100, DEFAULT_PARAMS)

The ``analyze`` body mirrors bpm_analysis.py:1007-1117 + :223-229 for one
in-memory recording.  It is exercised on the GPU by tests/test_gpu_parity.py.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("BPMX_LIB", os.path.join(HERE, "..", "bpm_analysis_amd", "libbpmx.so"))

DT = {np.dtype(np.uint8): 0, np.dtype(np.int16): 1, np.dtype(np.int32): 2, np.dtype(np.float32): 3,
      np.dtype(np.float64): 4}


class Params(ctypes.Structure):          # bpmx_params
    _fields_ = [(k, ctypes.c_int32) for k in ("mode", "stages", "dtype", "channels", "fs", "ds", "sr",
                                              "env_window", "distance", "noise_window", "min_periods",
                                              "options")] + \
               [(k, ctypes.c_double) for k in ("trough_prom_q", "peak_prom_q", "noise_floor_q", "fallback_q",
                                               "reject_mult")] + \
               [("ba_b", ctypes.c_double * 5), ("ba_a", ctypes.c_double * 5), ("ba_zi", ctypes.c_double * 4),
                ("sos", ctypes.c_double * 12), ("sos_zi", ctypes.c_double * 4)]


class Batch(ctypes.Structure):           # bpmx_batch
    _fields_ = [("n_files", ctypes.c_int32), ("reserved", ctypes.c_int32), ("pcm", ctypes.c_void_p),
                ("frame_offsets", ctypes.POINTER(ctypes.c_int64))]


class Out(ctypes.Structure):             # bpmx_out
    _fields_ = [(k, ctypes.c_void_p) for k in ("env", "floor", "y", "troughs", "peaks", "n_troughs", "n_peaks",
                                               "flags", "n_raw_troughs")]


_hip = _lib = _ctx = None


def _load():
    global _hip, _lib, _ctx
    if _lib is None:
        _hip = ctypes.CDLL("libamdhip64.so")
        _lib = ctypes.CDLL(LIB)
        _lib.bpmx_last_error.restype = ctypes.c_char_p
        _lib.bpmx_decimated_length.restype = ctypes.c_int64
        _lib.bpmx_decimated_length.argtypes = [ctypes.c_int64, ctypes.c_int32]
        ctx = ctypes.c_void_p()
        _check(_lib.bpmx_create(0, ctypes.byref(ctx)))
        _ctx = ctx
    return _hip, _lib, _ctx


def _check(rc):
    if rc != 0:
        msg = _lib.bpmx_last_error().decode()
        raise ValueError(msg) if rc == -1 else RuntimeError(msg)


def _dev(nbytes):
    p = ctypes.c_void_p()
    if _hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(max(nbytes, 8))) != 0:
        raise MemoryError("hipMalloc")
    return p


def _h2d(dst, a):
    _hip.hipMemcpy(dst, a.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(a.nbytes), 1)


def _d2h(a, src):
    _hip.hipMemcpy(a.ctypes.data_as(ctypes.c_void_p), src, ctypes.c_size_t(a.nbytes), 2)


def make_params(fs, params, mode=0, dtype=1, channels=1):
    """bpm_analysis.py:1018-1044 (ds clamp, sr, Nyquist check, butter) -> bpmx_params."""
    from scipy.signal import butter, lfilter_zi, sosfilt_zi
    ds = params["downsample_factor"]
    max_safe = int((fs / (150 * 2)) - 1)
    if ds > max_safe:
        ds = max(1, max_safe)
    sr = fs // ds if ds > 1 else fs
    ds = max(ds, 1)
    nyq = 0.5 * sr
    if 150 / nyq >= 1.0:
        raise ValueError(f"Cannot create a 150Hz filter. The effective sample rate of {sr}Hz is too low.")
    b, a = butter(2, [20 / nyq, 150 / nyq], btype="band")
    sos = butter(2, [20 / (0.5 * fs), 150 / (0.5 * fs)], btype="band", output="sos")
    p = Params(mode=mode, stages=7, dtype=dtype, channels=channels, fs=fs, ds=ds, sr=sr, env_window=sr // 10,
               distance=int(params["min_peak_distance_sec"] * sr), noise_window=int(params["noise_window_sec"] * sr),
               min_periods=3, trough_prom_q=params["trough_prominence_quantile"],
               peak_prom_q=params["peak_prominence_quantile"], noise_floor_q=params["noise_floor_quantile"],
               fallback_q=0.1, reject_mult=params.get("trough_rejection_multiplier", 4.0))
    p.ba_b[:], p.ba_a[:], p.ba_zi[:] = list(b), list(a), list(lfilter_zi(b, a))
    p.sos[:], p.sos_zi[:] = list(np.ravel(sos)), list(np.ravel(sosfilt_zi(sos)))
    return p


def analyze(pcm: np.ndarray, fs: int, params: dict, native: bool = False):
    """One recording -> (env, floor, troughs, peaks, sr), all stages on the GPU."""
    hip, lib, ctx = _load()
    pcm = np.ascontiguousarray(pcm)
    ch = 1 if pcm.ndim == 1 else pcm.shape[1]
    p = make_params(fs, params, 1 if native else 0, DT[pcm.dtype], ch)
    n = pcm.shape[0]
    nd = lib.bpmx_decimated_length(n, p.ds)
    fo = np.array([0, n], dtype=np.int64)
    d_pcm = _dev(pcm.nbytes)
    _h2d(d_pcm, pcm)
    bufs = {k: _dev(nd * 8) for k in ("env", "floor", "troughs", "peaks")}
    cnt = {k: _dev(4) for k in ("n_troughs", "n_peaks", "flags", "n_raw_troughs")}
    out = Out(y=None, **bufs, **cnt)
    batch = Batch(n_files=1, pcm=d_pcm, frame_offsets=fo.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
    _check(lib.bpmx_run(ctx, ctypes.byref(p), ctypes.byref(batch), ctypes.byref(out), None))
    hip.hipDeviceSynchronize()
    env, floor = np.empty(nd), np.empty(nd)
    _d2h(env, bufs["env"])
    _d2h(floor, bufs["floor"])
    ntr, npk = np.zeros(1, np.int32), np.zeros(1, np.int32)
    _d2h(ntr, cnt["n_troughs"])
    _d2h(npk, cnt["n_peaks"])
    tr, pk = np.empty(int(ntr[0]), np.int64), np.empty(int(npk[0]), np.int64)
    if len(tr):
        _d2h(tr, bufs["troughs"])
    if len(pk):
        _d2h(pk, bufs["peaks"])
    for v in (d_pcm, *bufs.values(), *cnt.values()):
        hip.hipFree(v)
    return env, floor, tr, pk, p.sr
