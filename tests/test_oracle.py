"""The CPU oracle against the reference's golden vectors (pins the oracle)."""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests import goldens as G


@pytest.mark.parametrize("name", G.names(kind="pcm"))
def test_oracle_pcm_goldens(name):
    g = G.load(name)
    mode = str(g["mode"])
    o = O.detect(g["pcm"], int(g["fs"]), g["params"], mode=mode)
    assert o["sr"] == int(g["sr"])
    if mode == "reference":
        # bit-exact: preprocess_audio, filtfilt, noise floor
        assert np.array_equal(o["y"], g["y"])
        assert np.array_equal(o["env"], g["env"])
        assert np.array_equal(o["floor"], g["floor"], equal_nan=True)
    else:
        # native mode oracle: sosfiltfilt bit-exact, hilbert via numpy.fft (<= 1e-12 rel)
        assert np.array_equal(o["y"], g["y"])
        scale = np.max(np.abs(g["env"]))
        assert np.max(np.abs(o["env"] - g["env"])) <= 1e-12 * scale
        assert np.allclose(o["floor"], g["floor"], rtol=1e-10, atol=0)
    assert np.array_equal(o["troughs"], g["troughs"])
    assert np.array_equal(o["peaks"], g["peaks"])
    assert o["flags"] == int(g["flags"])


@pytest.mark.parametrize("name", G.names(kind="env"))
def test_oracle_env_goldens(name):
    g = G.load(name)
    d = O.derive(302 * 146, dict(g["params"]))  # derive() only supplies distance/window here
    sr = int(g["sr"])
    d.sr = sr
    d.distance = int(g["params"]["min_peak_distance_sec"] * sr)
    d.noise_window = int(g["params"]["noise_window_sec"] * sr)
    floor, tr, flags = O.noise_floor(g["env"], d, g["params"])
    assert np.array_equal(floor, g["floor"], equal_nan=True)
    assert np.array_equal(tr, g["troughs"])
    assert flags == int(g["flags"])
    pk = O.raw_peaks(g["env"], floor, d, g["params"])
    assert np.array_equal(pk, g["peaks"])


def test_oracle_vulpine_known_answer():
    """Labeler-recipe envelope of the committed filtered WAV reproduces every raw
    peak index of samples/vulpine_Debug_Log.md (heartbeat_labeler.py:63-67)."""
    g = G.load("vulpine")
    w = g["pcm"]
    env = O.rolling_mean(np.abs(w).astype(np.float64), int(g["fs"]) // 10, 1)
    d = O.derive(302 * 146, dict(g["params"]))
    d.sr, d.distance, d.noise_window = 302, 15, 3020
    floor, tr, _ = O.noise_floor(env, d, g["params"])
    pk = O.raw_peaks(env, floor, d, g["params"])
    assert np.array_equal(pk, g["log_peaks"])
    assert len(np.intersect1d(tr, g["log_troughs"])) >= 1345  # 4 off by int16 quantisation
    # and the reference pipeline run on the same WAV
    o = O.detect(w, int(g["fs"]), g["params"])
    assert np.array_equal(o["env"], g["env"])
    assert np.array_equal(o["troughs"], g["troughs"])
    assert np.array_equal(o["peaks"], g["peaks"])


def test_short_input_raises():
    pcm = O.synth(1, 146 * 15, 44100, 1)
    with pytest.raises(ValueError):
        O.detect(pcm, 44100, G.BASE_PARAMS)


def test_oracle_under_sanitizers(tmp_path):
    """SURVEY.md section 5 (race detection / sanitizers): the C restatement under
    ASan + UBSan on synthetic recordings (reference and native ordering,
    stereo, padlen rejects) and envelope edge cases (constant, ramps, windows
    longer than the recording).  Any invalid access, leak or UB fails."""
    import shutil
    import subprocess
    cc = shutil.which("gcc")
    if cc is None:
        pytest.skip("gcc not available")
    here = os.path.dirname(os.path.abspath(__file__))
    exe = str(tmp_path / "sanitize_driver")
    cmd = [cc, "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1",
           "-ffp-contract=off", "-std=c11", "-o", exe, os.path.join(here, "sanitize_driver.c"), "-lm"]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "sanitize" in (b.stderr or ""):
        pytest.skip("sanitizer runtime not available: " + b.stderr[-200:])
    assert b.returncode == 0, b.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0"))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "SANITIZE OK" in r.stdout
