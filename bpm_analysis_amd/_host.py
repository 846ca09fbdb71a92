"""ctypes binding of libbpmx_host.so (include/bpmx_host.h): the per-file beat
stages as native code for host threads.  Built in-tree by
``make -C bpm_analysis_amd/host`` (``__graft_entry__.build()``); raises if the
library is missing."""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libbpmx_host.so")
ABI_VERSION = 1
OK, E_ARG, E_FEW_PEAKS = 0, -1, -2
TAG_NONE, TAG_S1, TAG_S2, TAG_LONE_S1, TAG_NOISE = 0, 1, 2, 3, 4

_D, _I = ctypes.c_double, ctypes.c_int64
# (field, type, params key, default when the key is absent: beats.py's params.get defaults)
_FIELDS = [
    ("pairing_confidence_threshold", _D, None), ("s1_s2_interval_cap_sec", _D, None),
    ("s1_s2_interval_rr_fraction", _D, None), ("deviation_smoothing_factor", _D, None),
    ("stability_history_window", _I, 20), ("stability_confidence_floor", _D, 0.85),
    ("stability_confidence_ceiling", _D, 1.10), ("s1_s2_boost_ratio", _D, 1.2), ("boost_amount_min", _D, 0.10),
    ("boost_amount_max", _D, 0.35), ("penalty_amount_min", _D, 0.15), ("penalty_amount_max", _D, 0.40),
    ("s2_s1_ratio_low_bpm", _D, None), ("s2_s1_ratio_high_bpm", _D, None), ("contractility_bpm_low", _D, None),
    ("contractility_bpm_high", _D, None), ("recovery_phase_duration_sec", _D, 120.0),
    ("interval_penalty_start_factor", _D, 1.0), ("interval_penalty_full_factor", _D, 1.4),
    ("interval_max_penalty", _D, 0.75), ("enable_interval_penalty", _I, True), ("cascade_reset_trigger_count", _I, 3),
    ("min_bpm", _D, None), ("max_bpm", _D, None), ("lone_s1_forward_check_pct", _D, 0.6),
    ("lone_s1_confidence_threshold", _D, 0.6), ("lone_s1_rhythm_weight", _D, 0.65),
    ("lone_s1_amplitude_weight", _D, 0.35), ("rr_correction_threshold_pct", _D, 0.6),
    ("rr_correction_long_interval_pct", _D, 1.7), ("penalty_waiver_strength_ratio", _D, None),
    ("penalty_waiver_max_s2_s1_ratio", _D, None), ("output_smoothing_window_sec", _D, None),
]


class BeatParams(ctypes.Structure):
    _fields_ = [(n, t) for n, t, _ in _FIELDS]


def beat_params(params: dict) -> BeatParams:
    p = BeatParams()
    for name, typ, default in _FIELDS:
        v = params[name] if default is None else params.get(name, default)
        setattr(p, name, int(bool(v)) if name == "enable_interval_penalty" else (int(v) if typ is _I else float(v)))
    return p


_lib = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not found: build it with `make -C bpm_analysis_amd/host`")
    L = ctypes.CDLL(LIB_PATH)
    L.bpmx_host_abi_version.restype = ctypes.c_int
    P = ctypes.c_void_p
    L.bpmx_beats.argtypes = [P, _I, P, P, _I, ctypes.c_int32, ctypes.POINTER(BeatParams), _D, P, P, P, P, P, P, P]
    L.bpmx_beats.restype = ctypes.c_int
    L.bpmx_beats_batch.argtypes = [ctypes.c_int32, P, P, P, P, P, P, ctypes.POINTER(BeatParams), _D, ctypes.c_int32,
                                   P, P, P, P, P, P, P, P]
    L.bpmx_beats_batch.restype = ctypes.c_int
    if L.bpmx_host_abi_version() != ABI_VERSION:
        raise RuntimeError("libbpmx_host ABI mismatch; rebuild")
    _lib = L
    return L


def beats(env: np.ndarray, sr: int, floor, raw_peaks: np.ndarray, params, hint=None) -> dict:
    """Beat stages of one recording (bpm_analysis.py:1734-1757 minus metrics
    and reports) -> dict(final_peaks, bpm_times, bpm, start_bpm, peak_time,
    recovery_time, tags) or dict(error=KeyError) for < 2 raw peaks, as the
    reference's refinement raises.  ``params`` may be a prepared BeatParams."""
    L = load()
    env = np.ascontiguousarray(env, dtype=np.float64)
    floor = np.ascontiguousarray(getattr(floor, "values", floor), dtype=np.float64)
    pk = np.ascontiguousarray(raw_peaks, dtype=np.int64)
    bp = params if isinstance(params, BeatParams) else beat_params(params)
    n = max(len(pk), 1)
    fin = np.empty(n, np.int64)
    bt, bv = np.empty(n), np.empty(n)
    nf, nb = ctypes.c_int64(0), ctypes.c_int64(0)
    pas = np.empty(3)
    tags = np.empty(n, np.int8)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = L.bpmx_beats(p(env), env.size, p(floor), p(pk), len(pk), int(sr), ctypes.byref(bp),
                      float("nan") if hint is None else float(hint), p(fin), ctypes.byref(nf), p(bt), p(bv),
                      ctypes.byref(nb), p(pas), p(tags))
    if rc == E_FEW_PEAKS:
        return {"error": KeyError("dynamic_noise_floor_series")}
    if rc != OK:
        raise ValueError(f"bpmx_beats failed ({rc})")
    nan2none = lambda x: None if x != x else float(x)  # noqa: E731
    return {"final_peaks": fin[:nf.value].copy(), "bpm_times": bt[:nb.value].copy(), "bpm": bv[:nb.value].copy(),
            "start_bpm": float(pas[0]), "peak_time": nan2none(pas[1]), "recovery_time": nan2none(pas[2]),
            "tags": tags[:len(pk)].copy()}


def beats_batch(results, params, hint=None, threads: int = 1) -> list:
    """bpmx_beats_batch over per-file dicts (env, floor, peaks, sr) on
    ``threads`` native host threads; one call, no per-file Python work beyond
    collecting pointers.  Entries with ``error`` pass through."""
    L = load()
    bp = params if isinstance(params, BeatParams) else beat_params(params)
    idx = [k for k, r in enumerate(results) if "error" not in r]
    out = list(results)
    F = len(idx)
    if F == 0:
        return out
    keep, envp, flp, pkp, ne, npk, srs = [], [], [], [], [], [], []
    finb, btb, bvb, tagb = [], [], [], []
    for k in idx:
        r = results[k]
        e = np.ascontiguousarray(r["env"], dtype=np.float64)
        fl = np.ascontiguousarray(getattr(r["floor"], "values", r["floor"]), dtype=np.float64)
        pk = np.ascontiguousarray(r["peaks"], dtype=np.int64)
        m = max(len(pk), 1)
        bufs = (np.empty(m, np.int64), np.empty(m), np.empty(m), np.empty(m, np.int8))
        keep += [e, fl, pk]
        envp.append(e.ctypes.data); flp.append(fl.ctypes.data); pkp.append(pk.ctypes.data)
        ne.append(e.size); npk.append(len(pk)); srs.append(int(r["sr"]))
        finb.append(bufs[0]); btb.append(bufs[1]); bvb.append(bufs[2]); tagb.append(bufs[3])
    ptr = lambda lst: (ctypes.c_void_p * F)(*lst)  # noqa: E731
    data = lambda bl: ptr([b.ctypes.data for b in bl])  # noqa: E731
    ne_a, npk_a = np.array(ne, np.int64), np.array(npk, np.int64)
    sr_a = np.array(srs, np.int32)
    nf, nb, st = np.zeros(F, np.int64), np.zeros(F, np.int64), np.zeros(F, np.int32)
    pas = np.empty((F, 3))
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = L.bpmx_beats_batch(F, ptr(envp), p(ne_a), ptr(flp), ptr(pkp), p(npk_a), p(sr_a), ctypes.byref(bp),
                            float("nan") if hint is None else float(hint), int(threads), data(finb), p(nf),
                            data(btb), data(bvb), p(nb), p(pas), data(tagb), p(st))
    if rc != OK:
        raise ValueError(f"bpmx_beats_batch failed ({rc})")
    nan2none = lambda x: None if x != x else float(x)  # noqa: E731
    for j, k in enumerate(idx):
        if st[j] == E_FEW_PEAKS:
            out[k] = {"error": KeyError("dynamic_noise_floor_series")}
        elif st[j] != OK:
            raise ValueError(f"bpmx_beats failed ({st[j]}) for recording {k}")
        else:
            out[k] = {"final_peaks": finb[j][:nf[j]], "bpm_times": btb[j][:nb[j]], "bpm": bvb[j][:nb[j]],
                      "start_bpm": float(pas[j, 0]), "peak_time": nan2none(pas[j, 1]),
                      "recovery_time": nan2none(pas[j, 2]), "tags": tagb[j][:npk[j]]}
    return out
