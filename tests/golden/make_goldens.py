"""Generate the golden vectors in tests/golden/*.npz from the REFERENCE itself.

Runs only in the build container, where ``/root/reference`` (pixeru/bpm_analysis
@ 2025-07-25) is importable.  It imports the reference's own functions —
``preprocess_audio`` (bpm_analysis.py:1007), ``_calculate_dynamic_noise_floor``
(:1064) and ``PeakClassifier._find_raw_peaks`` (:223) — and records their outputs
on seeded inputs.  Native-mode goldens use the scipy composition SURVEY.md §8(c)
defines (sosfiltfilt @ fs -> [::ds] -> |hilbert| -> rolling mean -> the
reference's own floor and peak calls).  Fixtures are data only: inputs (or the
recipe + sha256 to regenerate them) and expected outputs.

    python tests/golden/make_goldens.py
"""
from __future__ import annotations

import hashlib
import json
import logging
import os
import sys
import tempfile

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from tests.golden import inputs as I  # noqa: E402

REF = "/root/reference"
sys.path.insert(0, REF)
import bpm_analysis as R  # noqa: E402
import config as RC  # noqa: E402
from scipy.io import wavfile  # noqa: E402
from scipy.signal import butter, hilbert, sosfiltfilt  # noqa: E402

HOT_KEYS = ["downsample_factor", "min_peak_distance_sec", "peak_prominence_quantile",
            "trough_prominence_quantile", "noise_floor_quantile", "noise_window_sec",
            "trough_rejection_multiplier"]


class _Flags(logging.Handler):
    def __init__(self):
        super().__init__(logging.WARNING)
        self.msgs = []

    def emit(self, record):
        self.msgs.append(record.getMessage())


def _flags(msgs):
    f = 0
    if any("Not enough troughs found" in m for m in msgs):
        f |= 1
    if any("Not enough sanitized troughs" in m for m in msgs):
        f |= 2
    return f


def _raw_peaks(env, sr, params, floor):
    pc = R.PeakClassifier.__new__(R.PeakClassifier)
    pc.audio_envelope, pc.sample_rate, pc.params = env, sr, params
    return pc._find_raw_peaks(floor)


def _floor_and_peaks(env, sr, params):
    h = _Flags()
    logging.getLogger().addHandler(h)
    try:
        floor, troughs = R._calculate_dynamic_noise_floor(env, sr, params)
    finally:
        logging.getLogger().removeHandler(h)
    fl = _flags(h.msgs)
    floor_v = floor.values.astype(np.float64)
    peaks = _raw_peaks(env, sr, params, floor.values)
    return floor_v, np.asarray(troughs).astype(np.int64), np.asarray(peaks, dtype=np.int64), fl


def _params(over=None):
    p = dict(RC.DEFAULT_PARAMS)
    p["save_filtered_wav"] = False
    if over:
        p.update(over)
    return p


def make_pcm_case(name, spec, mode="reference", over=None, store_pcm=False):
    params = _params(over)
    pcm, fs = I.make_input(spec)
    if mode == "reference":
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "in.wav")
            wavfile.write(path, fs, pcm)
            env, sr = R.preprocess_audio(path, params, td)
        floor, troughs, peaks, fl = _floor_and_peaks(env, sr, params)
        # y = the reference's filtfilt output (bpm_analysis.py:1044-1045), for the filter kernel check
        x = pcm if pcm.ndim == 1 else np.mean(pcm, axis=1)
        ds = params["downsample_factor"]
        ms = int((fs / (150 * 2)) - 1)
        if ds > ms:
            ds = max(1, ms)
        from scipy.signal import filtfilt
        xd = x[::ds] if ds > 1 else x
        b, a = butter(2, [20 / (0.5 * sr), 150 / (0.5 * sr)], btype="band")
        y = filtfilt(b, a, xd)
    else:
        x = pcm if pcm.ndim == 1 else np.mean(pcm, axis=1)
        ds = params["downsample_factor"]
        ms = int((fs / (150 * 2)) - 1)
        if ds > ms:
            ds = max(1, ms)
        sr = fs // ds if ds > 1 else fs
        sos = butter(2, [20 / (0.5 * fs), 150 / (0.5 * fs)], btype="band", output="sos")
        y = sosfiltfilt(sos, x)[::ds]
        env = pd.Series(np.abs(hilbert(y))).rolling(window=sr // 10, min_periods=1, center=True).mean().values
        floor, troughs, peaks, fl = _floor_and_peaks(env, sr, params)
    out = dict(kind="pcm", mode=mode, fs=fs, sr=sr, spec=json.dumps(spec),
               params=json.dumps({k: params[k] for k in HOT_KEYS}),
               pcm_sha256=hashlib.sha256(np.ascontiguousarray(pcm).tobytes()).hexdigest(),
               env=env, floor=floor, troughs=troughs, peaks=peaks, y=np.asarray(y, dtype=np.float64), flags=fl)
    if store_pcm:
        out["pcm"] = pcm
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(f"{name:28s} mode={mode:9s} fs={fs} sr={sr} Nd={len(env)} troughs={len(troughs)} peaks={len(peaks)} flags={fl}")


def make_env_case(name, env, sr, over=None):
    params = _params(over)
    env = np.ascontiguousarray(env, dtype=np.float64)
    floor, troughs, peaks, fl = _floor_and_peaks(env, sr, params)
    extra = {}
    if name.startswith("env_ties"):
        # the raw troughs before sanitisation, by the reference's own call
        # (bpm_analysis.py:1066-1070), so the tie tests can pin the trough
        # search separately from the floor
        from scipy.signal import find_peaks
        d = int(params["min_peak_distance_sec"] * sr)
        q = np.quantile(env, params["trough_prominence_quantile"])
        extra["raw_troughs"] = find_peaks(-env, distance=d, prominence=q)[0].astype(np.int64)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), kind="env", mode="env", sr=sr, fs=sr,
                        params=json.dumps({k: params[k] for k in HOT_KEYS}), env=env, floor=floor,
                        troughs=troughs, peaks=peaks, flags=fl, **extra)
    print(f"{name:28s} env-level sr={sr} Nd={len(env)} troughs={len(troughs)} peaks={len(peaks)} flags={fl}")


def make_vulpine():
    """Known-answer test: the reference's committed outputs for vulpine.wav.

    samples/vulpine_filtered_debug.wav (the 302 Hz filtered signal the reference wrote)
    and the raw-peak / sanitized-trough times from samples/vulpine_Debug_Log.md.
    """
    import re
    fs, w = wavfile.read(os.path.join(REF, "samples", "vulpine_filtered_debug.wav"))
    txt = open(os.path.join(REF, "samples", "vulpine_Debug_Log.md")).read()
    ents = re.findall(r"## Time: `([0-9.]+)s`\n\*\*([^*]+)\*\*", txt)
    peaks = sorted(int(round(float(t) * fs)) for t, k in ents if k.strip() != "Trough Detected")
    troughs = sorted(int(round(float(t) * fs)) for t, k in ents if k.strip() == "Trough Detected")
    # the reference pipeline run on the committed WAV (ds clamps to 1 at 302 Hz)
    params = _params()
    env, sr = R.preprocess_audio(os.path.join(REF, "samples", "vulpine_filtered_debug.wav"), params, "/tmp")
    floor, tr, pk, fl = _floor_and_peaks(env, sr, params)
    np.savez_compressed(os.path.join(HERE, "vulpine.npz"), kind="vulpine", fs=fs, sr=sr, pcm=w,
                        params=json.dumps({k: params[k] for k in HOT_KEYS}),
                        log_peaks=np.array(peaks, dtype=np.int64), log_troughs=np.array(troughs, dtype=np.int64),
                        env=env, floor=floor, troughs=tr, peaks=pk, flags=fl)
    print(f"vulpine: log peaks={len(peaks)} log troughs={len(troughs)}; pipeline troughs={len(tr)} peaks={len(pk)}")


def main(only=None):
    """Every fixture, or only those whose names start with one of `only`
    (e.g. ``python tests/golden/make_goldens.py env_ties``)."""
    np.seterr(all="ignore")
    logging.getLogger().setLevel(logging.WARNING)
    want = (lambda n: any(n.startswith(o) for o in only)) if only else (lambda n: True)
    for name, spec, mode, over, store in I.CASES:
        if want(name):
            make_pcm_case(name, spec, mode, over, store)
    for name, (env, sr, over) in I.env_cases().items():
        if want(name):
            make_env_case(name, env, sr, over)
    if want("vulpine"):
        make_vulpine()


if __name__ == "__main__":
    main(sys.argv[1:] or None)
