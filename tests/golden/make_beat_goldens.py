"""Golden vectors for the host beat stages (bpm_analysis_amd/beats.py) from the REFERENCE.

Runs only in the build container, where ``/root/reference`` is importable.  For
every hot-path golden (tests/golden/*.npz holding env / floor / troughs) and for
two long synthetic recordings (regenerated bit-exactly by
``tests/golden/inputs.make_input`` and run through the reference's own
``preprocess_audio`` + ``_calculate_dynamic_noise_floor``), it runs the
reference's stages 2-6 of ``analyze_wav_file`` (bpm_analysis.py:1734-1757):
``_run_preliminary_pass`` (:1623), ``PeakClassifier.classify_peaks`` (:113),
``_refine_and_correct_peaks`` (:1655), ``_calculate_final_metrics`` (:1701),
the ``Plotter`` figure (its plotly JSON, :429-780), the BPM CSV it writes
(:458-473) and the
``ReportGenerator`` files (summary, debug log, settings; :782-985).  It records
the outputs as data in ``tests/golden/beats/<name>.npz``.

    python tests/golden/make_beat_goldens.py
"""
from __future__ import annotations

import glob
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
OUT = os.path.join(HERE, "beats")
sys.path.insert(0, REPO)
from tests.golden import inputs as I  # noqa: E402

sys.path.insert(0, "/root/reference")
import bpm_analysis as R  # noqa: E402
import config as RC  # noqa: E402
from scipy.io import wavfile  # noqa: E402

# long recordings: the BPM ramp of the generator spans the file, so the
# slope / HRR / HRV metrics all have data (name, spec, start_bpm_hint)
LONG = [
    ("long_6k_8min", dict(seed=21, secs=480, fs=6000), None),
    ("long_8k_5min_hint", dict(seed=22, secs=300, fs=8000), 95.0),
]
HINTS = {"ref_44k_60s_mono": 70.0}      # one hot-path case also with a start-BPM hint


def _ts(v):
    """Timestamps -> int64 ns; numpy scalars -> python numbers (JSON-exact)."""
    if isinstance(v, pd.Timestamp):
        return {"ns": int(v.value)}
    if isinstance(v, (np.floating, float)):
        return float(v)
    if isinstance(v, (np.integer, int)):
        return int(v)
    return v


def _metrics_json(m):
    d = {}
    for k in ("major_inclines", "major_declines"):
        d[k] = [{kk: _ts(vv) for kk, vv in x.items()} for x in m[k]]
    for k in ("hrr_stats", "peak_recovery_stats", "peak_exertion_stats"):
        d[k] = None if m[k] is None else {kk: _ts(vv) for kk, vv in m[k].items()}
    d["hrv_summary"] = {k: float(v) for k, v in m["hrv_summary"].items()}
    return json.dumps(d)


def run_case(name, env, sr, floor, troughs, params, hint):
    floor_s = pd.Series(floor, index=np.arange(len(floor)))
    out = dict(name=name, sr=sr, params=json.dumps({k: params[k] for k in params if k in RC.DEFAULT_PARAMS}),
               hint=np.nan if hint is None else hint)
    start, t_pk, t_end = R._run_preliminary_pass(env, sr, params, floor_s, troughs, hint)
    out.update(start_bpm=start, peak_time=np.nan if t_pk is None else t_pk,
               recovery_time=np.nan if t_end is None else t_end)
    clf = R.PeakClassifier(env, sr, params, start, floor_s, troughs, t_pk, t_end)
    s1, raw, data = clf.classify_peaks()
    out.update(s1_peaks=np.asarray(s1), all_raw_peaks=np.asarray(raw))
    try:
        final, data = R._refine_and_correct_peaks(s1, raw, data, env, sr, params)
    except KeyError as exc:
        out["error"] = f"KeyError:{exc.args[0]}"
        return out
    out["final_peaks"] = np.asarray(final)
    info = data["beat_debug_info"]
    keys = sorted(info)
    out.update(info_keys=np.array(keys, dtype=np.int64), info_vals=np.array([info[k] for k in keys], dtype=str))
    if "long_term_bpm_series" in data:
        out.update(lt_t=data["long_term_bpm_series"].index.to_numpy(float),
                   lt_v=data["long_term_bpm_series"].to_numpy(float))
    out.update(dev_t=data["deviation_series"].index.to_numpy(float), dev_v=data["deviation_series"].to_numpy(float))
    if len(final) < 2:
        return out
    m = R._calculate_final_metrics(final, sr, params)
    sb = m["smoothed_bpm"]
    out.update(bpm_times=np.asarray(m["bpm_times"], dtype=float), bpm_v=sb.to_numpy(float),
               bpm_ns=sb.index.asi8.astype(np.int64) if len(sb) else np.zeros(0, np.int64),
               metrics=_metrics_json(m))
    h = m["windowed_hrv_df"]
    for c in ("time", "rmssdc", "sdnn", "bpm"):
        out["hrv_" + c] = h[c].to_numpy(float) if len(h) else np.zeros(0)
    with tempfile.TemporaryDirectory() as td:
        p = R.Plotter(os.path.join(td, name + ".wav"), params, sr, td)
        fig_json = p.plot_and_save(env, raw, data, m).to_json()
        out["fig_sha256"] = hashlib.sha256(fig_json.encode()).hexdigest()
        if len(fig_json) < 600_000:
            out["fig_json"] = fig_json
        csv_path = os.path.join(td, name + "_bpm_plot.csv")
        out["csv"] = open(csv_path).read() if os.path.exists(csv_path) else ""
        # ReportGenerator (:782-985); the one timestamp line of each markdown file is dropped
        rep = R.ReportGenerator(os.path.join(td, name + ".wav"), td)
        rep.save_analysis_summary(m)
        rep.create_chronological_log(env, sr, raw, data, m)
        rep.save_analysis_settings(hint)
        for key, suffix in (("summary_md", "_Analysis_Summary.md"), ("debug_log_md", "_Debug_Log.md"),
                            ("settings_json", "_Analysis_Settings.json")):
            text = open(os.path.join(td, name + suffix), encoding="utf-8").read()
            if suffix.endswith(".md"):
                lines = text.split("\n")
                text = "\n".join(lines[:1] + lines[2:])
            out[key] = text
    return out


def main():
    np.seterr(all="ignore")
    logging.getLogger().setLevel(logging.ERROR)
    os.makedirs(OUT, exist_ok=True)
    for path in sorted(glob.glob(os.path.join(HERE, "*.npz"))):
        g = np.load(path)
        if "troughs" not in g or "env" not in g or "floor" not in g:
            continue
        name = os.path.splitext(os.path.basename(path))[0]
        params = dict(RC.DEFAULT_PARAMS)
        params.update(json.loads(str(g["params"])))
        for hint in [None] + ([HINTS[name]] if name in HINTS else []):
            tag = name if hint is None else f"{name}_hint"
            o = run_case(tag, g["env"], int(g["sr"]), g["floor"], g["troughs"], params, hint)
            o["source"] = name
            np.savez_compressed(os.path.join(OUT, tag + ".npz"), **o)
            print(tag, len(o.get("final_peaks", [])), o.get("error", ""))
    for name, spec, hint in LONG:
        pcm, fs = I.make_input(spec)
        params = dict(RC.DEFAULT_PARAMS)
        params["save_filtered_wav"] = False
        with tempfile.TemporaryDirectory() as td:
            wav = os.path.join(td, name + ".wav")
            wavfile.write(wav, fs, pcm)
            env, sr = R.preprocess_audio(wav, params, td)
        floor, troughs = R._calculate_dynamic_noise_floor(env, sr, params)
        o = run_case(name, env, sr, floor.to_numpy(float), troughs, params, hint)
        o.update(source="synth", spec=json.dumps(spec))
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **o)
        print(name, len(o.get("final_peaks", [])), o.get("error", ""))


if __name__ == "__main__":
    main()
