"""libbpmx_host.so (the beat stages in C++) against the reference's beat
goldens (tests/golden/beats, made by the reference itself): final beats,
preliminary-pass values and labels exact, the smoothed BPM curve to 1e-12
relative (north_star: 1e-5)."""
import numpy as np
import pytest

from bpm_analysis_amd import _host as H
from bpm_analysis_amd import beats as B
from tests import test_beats as TB

LABEL = {H.TAG_S1: B.S1_PAIRED, H.TAG_S2: B.S2_PAIRED, H.TAG_NOISE: "Noise"}


@pytest.mark.parametrize("name", TB.CASES)
def test_native_beats_match_reference(name):
    g, params, hint, inp = TB.load_case(name)
    r = H.beats(inp["env"], inp["sr"], inp["floor"], inp["peaks"], params, hint)
    if "error" in g:
        assert isinstance(r["error"], KeyError)
        return
    assert np.array_equal(r["final_peaks"], g["final_peaks"])
    assert r["start_bpm"] == float(g["start_bpm"])
    for k in ("peak_time", "recovery_time"):
        assert (np.isnan(g[k]) and r[k] is None) or r[k] == float(g[k]), k
    # labels: the first field of every debug string
    labels = dict(zip((int(k) for k in g["info_keys"]), (str(v).split("§")[0] for v in g["info_vals"])))
    for k, tg in zip(g["all_raw_peaks"], r["tags"]):
        want = labels[int(k)]
        if want in (B.LONE_S1, B.LONE_S1_LAST, B.LONE_S1_CASCADE):
            assert tg == H.TAG_LONE_S1, (k, want)
        elif want in (B.S1_GAP, B.S2_GAP):
            assert tg == H.TAG_NOISE, (k, want)          # gap corrections relabel Noise peaks
        else:
            assert LABEL[int(tg)] == want, (k, want)
    if "metrics" not in g:
        return
    np.testing.assert_allclose(r["bpm_times"], g["bpm_times"], rtol=TB.RTOL, atol=0)
    np.testing.assert_allclose(r["bpm"], g["bpm_v"], rtol=TB.RTOL, atol=0)


def test_native_beats_agree_with_python_stages_on_random_inputs():
    """Beyond the goldens: random envelopes through the oracle's hot path, the
    C++ stages and beats.analyze_recording give the same beats and curves."""
    from oracle import oracle as O
    from bpm_analysis_amd import DEFAULT_PARAMS
    params = dict(DEFAULT_PARAMS, save_filtered_wav=False)
    for seed in range(6):
        o = O.detect(O.synth(300 + seed, 44100 * (20 + 7 * seed), 44100, 1), 44100, params, mode="native")
        a = B.analyze_recording(o["env"], o["sr"], o["floor"], o["troughs"], o["peaks"], params)
        r = H.beats(o["env"], o["sr"], o["floor"], o["peaks"], params)
        assert np.array_equal(r["final_peaks"], a["final_peaks"])
        m = a["final_metrics"]
        np.testing.assert_array_equal(r["bpm_times"], m["bpm_times"])
        np.testing.assert_allclose(r["bpm"], m["smoothed_bpm"].values, rtol=1e-12, atol=0)


def test_host_library_exports_every_declared_symbol():
    import os
    import re
    txt = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                            "bpmx_host.h")).read()
    names = set(re.findall(r"^\s*int\s+(bpmx_\w+)\s*\(", txt, re.M))
    assert names == {"bpmx_host_abi_version", "bpmx_beats", "bpmx_beats_batch"}
    L = H.load()
    for n in names:
        assert hasattr(L, n)
    assert L.bpmx_host_abi_version() == H.ABI_VERSION


def test_analyze_fast_threads_match_sequential():
    names = ["ref_44k_60s_mono", "ref_44k_40s_clicks", "ref_44k_10s_zeros", "vulpine", "ref_44k_short16"]
    runs, params = [], None
    for n in names:
        g, params, hint, inp = TB.load_case(n)
        runs.append(dict(inp))
    a = B.analyze_fast(runs, params)
    b = B.analyze_fast(runs, params, threads=3)
    for x, y in zip(a, b):
        assert ("error" in x) == ("error" in y)
        if "error" not in x:
            assert np.array_equal(x["final_peaks"], y["final_peaks"]) and np.array_equal(x["bpm"], y["bpm"])
