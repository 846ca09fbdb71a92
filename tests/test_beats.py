"""Host beat stages (bpm_analysis_amd/beats.py) against goldens made by the reference.

tests/golden/beats/*.npz were written by tests/golden/make_beat_goldens.py from
the reference's own ``_run_preliminary_pass``, ``PeakClassifier``,
``_refine_and_correct_peaks``, ``_calculate_final_metrics`` and BPM CSV
(bpm_analysis.py:1623-1757, :458-473).  Inputs are the hot-path goldens'
env / floor / troughs / raw peaks, or — for the long recordings — the C
oracle's outputs on the regenerated synthetic PCM (the oracle is pinned bit
for bit against the reference in test_oracle.py).  Beat indices, labels and
debug strings are compared exactly; the BPM curve, HRV and slope metrics to
1e-12 relative (they come out bit-identical today; the north_star bar is 1e-5).

The CPU tests feed the stages from the goldens; test_gpu_parity.py runs the
same stages on the GPU's outputs (marked gpu).
"""
from __future__ import annotations

import glob
import json
import os

import numpy as np
import pandas as pd
import pytest

from bpm_analysis_amd import beats as B
from bpm_analysis_amd.config import DEFAULT_PARAMS

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
CASES = sorted(os.path.splitext(os.path.basename(p))[0] for p in glob.glob(os.path.join(GOLD, "beats", "*.npz")))
RTOL = 1e-12


def load_case(name):
    g = np.load(os.path.join(GOLD, "beats", name + ".npz"))
    params = dict(DEFAULT_PARAMS)
    params.update(json.loads(str(g["params"])))
    hint = None if np.isnan(g["hint"]) else float(g["hint"])
    src = str(g["source"])
    if src == "synth":
        from oracle import oracle as O
        from tests.golden import inputs as I
        pcm, fs = I.make_input(json.loads(str(g["spec"])))
        r = O.detect(pcm, fs, params, "reference")
        inp = dict(env=r["env"], floor=r["floor"], troughs=r["troughs"], peaks=r["peaks"], sr=r["sr"])
    else:
        h = np.load(os.path.join(GOLD, src + ".npz"))
        inp = dict(env=h["env"], floor=h["floor"], troughs=h["troughs"], peaks=h["peaks"], sr=int(h["sr"]))
    return g, params, hint, inp


def _close(a, b, what):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    assert a.shape == b.shape, f"{what}: shape {a.shape} vs {b.shape}"
    np.testing.assert_allclose(a, b, rtol=RTOL, atol=0, equal_nan=True, err_msg=what)


def _cmp_obj(ours, ref, what):
    if ref is None:
        assert ours is None, what
        return
    assert ours is not None, what
    assert list(ours) == list(ref), f"{what}: keys"
    for k, v in ref.items():
        o = ours[k]
        if isinstance(v, dict):
            assert pd.Timestamp(o).value == v["ns"], f"{what}.{k}"
        else:
            _close(o, v, f"{what}.{k}")


def check_against_golden(g, res):
    assert np.array_equal(res["all_raw_peaks"], g["all_raw_peaks"])
    assert res["start_bpm"] == float(g["start_bpm"])
    for k in ("peak_time", "recovery_time"):
        v = res[k]
        assert (np.isnan(g[k]) and v is None) or v == float(g[k]), k
    assert np.array_equal(res["s1_peaks"], g["s1_peaks"])
    assert np.array_equal(res["final_peaks"], g["final_peaks"])
    info = res["analysis_data"]["beat_debug_info"]
    assert sorted(info) == list(g["info_keys"])
    for k, v in zip(g["info_keys"], g["info_vals"]):
        assert info[k] == str(v), f"debug string of peak {k}"
    data = res["analysis_data"]
    if "lt_t" in g:
        _close(data["long_term_bpm_series"].index, g["lt_t"], "long-term BPM times")
        _close(data["long_term_bpm_series"].values, g["lt_v"], "long-term BPM")
    _close(data["deviation_series"].index, g["dev_t"], "deviation times")
    _close(data["deviation_series"].values, g["dev_v"], "smoothed deviations")
    m = res["final_metrics"]
    if "metrics" not in g:
        assert m is None
        return
    _close(m["bpm_times"], g["bpm_times"], "bpm times")
    _close(m["smoothed_bpm"].values, g["bpm_v"], "smoothed BPM")
    assert np.array_equal(m["smoothed_bpm"].index.asi8, g["bpm_ns"])
    for c in ("time", "rmssdc", "sdnn", "bpm"):
        h = m["windowed_hrv_df"]
        _close(h[c].to_numpy(float) if len(h) else np.zeros(0), g["hrv_" + c], "hrv " + c)
    ref = json.loads(str(g["metrics"]))
    for k in ("major_inclines", "major_declines"):
        assert len(m[k]) == len(ref[k]), k
        for i, (o, r) in enumerate(zip(m[k], ref[k])):
            _cmp_obj(o, r, f"{k}[{i}]")
    for k in ("hrr_stats", "peak_recovery_stats", "peak_exertion_stats"):
        _cmp_obj(m[k], ref[k], k)
    assert list(m["hrv_summary"]) == list(ref["hrv_summary"])
    for k, v in ref["hrv_summary"].items():
        _close(m["hrv_summary"][k], v, "hrv_summary " + k)


@pytest.mark.parametrize("name", CASES)
def test_beats_match_reference(name, tmp_path):
    g, params, hint, inp = load_case(name)
    assert np.array_equal(inp["peaks"], g["all_raw_peaks"]), "hot-path raw peaks differ from the reference's"
    if "error" in g:
        with pytest.raises(KeyError):
            B.analyze_recording(inp["env"], inp["sr"], inp["floor"], inp["troughs"], inp["peaks"], params, hint)
        return
    res = B.analyze_recording(inp["env"], inp["sr"], inp["floor"], inp["troughs"], inp["peaks"], params, hint)
    check_against_golden(g, res)
    if res["final_metrics"] is not None:
        p = tmp_path / "bpm.csv"
        assert B.write_bpm_csv(str(p), res["final_metrics"]) == bool(str(g["csv"]))
        if str(g["csv"]):
            assert p.read_text() == str(g["csv"]), "BPM CSV differs byte-wise"


def test_goldens_cover_the_branches():
    """The fixtures exercise every label and each metric family at least once."""
    seen, metrics = set(), {"major_inclines": 0, "major_declines": 0, "hrr_stats": 0,
                            "peak_recovery_stats": 0, "peak_exertion_stats": 0}
    for name in CASES:
        g = np.load(os.path.join(GOLD, "beats", name + ".npz"))
        if "info_vals" in g:
            seen |= {str(v).split("§")[0] for v in g["info_vals"]}
        if "metrics" in g:
            for k, v in json.loads(str(g["metrics"])).items():
                if k in metrics and v:
                    metrics[k] += 1
    assert {B.S1_PAIRED, B.S2_PAIRED, B.LONE_S1, B.LONE_S1_LAST, B.LONE_S1_CASCADE, B.S1_GAP, B.S2_GAP,
            "Noise"} <= seen, seen
    assert all(metrics.values()), metrics


def test_update_long_term_bpm_limits():
    p = dict(DEFAULT_PARAMS)
    assert B.update_long_term_bpm(1.0, 80.0, p) == pytest.approx(79.0)          # EMA: 0.95 * 80 + 0.05 * 60
    assert B.update_long_term_bpm(0.5, 80.0, p) == pytest.approx(81.5)          # EMA says 82, slew limit 3 * 0.5
    assert B.update_long_term_bpm(0.1, 80.0, p) == pytest.approx(80.3)          # slew-limited to 3 * 0.1
    assert B.update_long_term_bpm(10.0, p["min_bpm"], p) == p["min_bpm"]         # clamped


def _drop_stamp(text: str) -> str:
    lines = text.split("\n")
    return "\n".join(lines[:1] + lines[2:])


@pytest.mark.parametrize("name", [c for c in CASES])
def test_reports_match_reference(name, tmp_path):
    """Analysis_Summary.md, Debug_Log.md (minus the timestamp line) and
    Analysis_Settings.json byte-equal to the reference's ReportGenerator."""
    from bpm_analysis_amd import reports as RP
    g, params, hint, inp = load_case(name)
    if "summary_md" not in g:
        pytest.skip("the reference writes no reports for this case")
    res = B.analyze_recording(inp["env"], inp["sr"], inp["floor"], inp["troughs"], inp["peaks"], params, hint)
    fname = os.path.join(str(tmp_path), name + ".wav")
    RP.write_reports(fname, str(tmp_path), inp["env"], inp["sr"], res["all_raw_peaks"], res["analysis_data"],
                     res["final_metrics"], hint)
    got = lambda suffix: (tmp_path / (name + suffix)).read_text(encoding="utf-8")  # noqa: E731
    assert _drop_stamp(got("_Analysis_Summary.md")) == str(g["summary_md"])
    assert _drop_stamp(got("_Debug_Log.md")) == str(g["debug_log_md"])
    assert got("_Analysis_Settings.json") == str(g["settings_json"])


@pytest.mark.parametrize("name", [c for c in CASES])
def test_plot_matches_reference(name, tmp_path):
    """The analysis figure's plotly JSON equals the reference Plotter's (hash for
    every case; the JSON itself is kept for the small ones to show a diff)."""
    import hashlib
    from bpm_analysis_amd import plot as PL
    g, params, hint, inp = load_case(name)
    if "fig_sha256" not in g:
        pytest.skip("the reference draws no figure for this case")
    res = B.analyze_recording(inp["env"], inp["sr"], inp["floor"], inp["troughs"], inp["peaks"], params, hint)
    fig = PL.write_plot(os.path.join(str(tmp_path), name + ".wav"), str(tmp_path), params, inp["sr"], inp["env"],
                        res["all_raw_peaks"], res["analysis_data"], res["final_metrics"])
    js = fig.to_json()
    if "fig_json" in g:
        want = json.loads(str(g["fig_json"]))
        got = json.loads(js)
        assert len(got["data"]) == len(want["data"])
        for i, (a, b) in enumerate(zip(got["data"], want["data"])):
            assert a == b, f"trace {i} ({b.get('name')})"
        assert got["layout"] == want["layout"]
    assert hashlib.sha256(js.encode()).hexdigest() == str(g["fig_sha256"])
    assert (tmp_path / f"{name}_bpm_plot.html").stat().st_size > 0


def test_analyze_many_worker_processes():
    """The per-file stages over worker processes give what the sequential loop gives."""
    names = ["ref_44k_60s_mono", "ref_44k_40s_clicks", "ref_44k_10s_zeros", "vulpine"]
    runs, params = [], None
    for n in names:
        g, params, hint, inp = load_case(n)
        runs.append(dict(inp))
    seq = B.analyze_many(runs, params)
    par = B.analyze_many(runs, params, workers=2)
    for a, b in zip(seq, par):
        assert ("error" in a) == ("error" in b)
        if "error" in a:
            assert type(a["error"]) is type(b["error"])
            continue
        assert np.array_equal(a["final_peaks"], b["final_peaks"])
        assert a["analysis_data"]["beat_debug_info"] == b["analysis_data"]["beat_debug_info"]
        pd.testing.assert_series_equal(a["final_metrics"]["smoothed_bpm"], b["final_metrics"]["smoothed_bpm"])
