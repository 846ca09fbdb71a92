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


@pytest.mark.parametrize("name", [n for n in G.names(kind="env") if not n.startswith("env_ties")])
def test_oracle_env_goldens(name):
    g = G.load(name)
    d = G.env_derived(g)
    floor, tr, flags = O.noise_floor(g["env"], d, g["params"])
    assert np.array_equal(floor, g["floor"], equal_nan=True)
    assert np.array_equal(tr, g["troughs"])
    assert flags == int(g["flags"])
    pk, tie = O.raw_peaks(g["env"], floor, d, g["params"], return_tie=True)
    assert np.array_equal(pk, g["peaks"])
    assert not tie


@pytest.mark.parametrize("name", G.names(kind="env", prefix="env_ties"))
def test_oracle_tie_goldens(name):
    """Envelopes with equal-height extrema closer than find_peaks' distance.
    (1) The restatement with numpy's own argsort order in the distance filter
    reproduces the reference's raw troughs and raw peaks exactly, which pins
    every other step of the oracle's find_peaks on these inputs.  (2) The
    stable order (the oracle's and the kernels' convention) differs from it
    here, and the decisive-tie report is set: on every tie golden, for the
    troughs and for the peaks wherever their answers differ."""
    g = G.load(name)
    d = G.env_derived(g)
    env, p = g["env"], g["params"]
    qt = O.quantile(env, p["trough_prominence_quantile"])
    qp = O.quantile(env, p["peak_prominence_quantile"])
    assert np.array_equal(O.find_peaks_numpy_order(env, distance=d.distance, prominence=qt, negate=True),
                          g["raw_troughs"])
    assert np.array_equal(O.find_peaks_numpy_order(env, height=g["floor"], distance=d.distance, prominence=qp),
                          g["peaks"])
    raw, ttie = O.find_peaks(env, distance=d.distance, prominence=qt, negate=True, return_tie=True)
    assert ttie and not np.array_equal(raw, g["raw_troughs"])
    _, _, flags = O.noise_floor(env, d, p)
    assert flags & O.F_TROUGH_TIE
    pk, ptie = O.raw_peaks(env, g["floor"], d, p, return_tie=True)
    assert ptie or np.array_equal(pk, g["peaks"])
    # (3) the whole noise floor in numpy's order (the GPU tie resolution's
    # checker): the reference's troughs and floor, bit for bit
    nf, nt, nfl, nraw = O.noise_floor_numpy_order(env, d, p)
    assert np.array_equal(nraw, g["raw_troughs"])
    assert np.array_equal(nt, g["troughs"])
    assert np.array_equal(nf, g["floor"], equal_nan=True)
    assert (nfl & 3) == (int(g["flags"]) & 3)


def test_noise_floor_from_raw_matches_c_restatement():
    """noise_floor_from_raw (the Python composition behind the numpy-order
    floor) equals bpmx_oracle.c's noise floor when both start from the same raw
    troughs (the stable order's, on every golden envelope without a tie)."""
    for name in [n for n in G.names(kind="env") if not n.startswith("env_ties")]:
        g = G.load(name)
        d = G.env_derived(g)
        env, p = g["env"], g["params"]
        raw = O.find_peaks(env, distance=d.distance, negate=True,
                           prominence=O.quantile(env, p["trough_prominence_quantile"]))
        f1, t1, fl1 = O.noise_floor(env, d, p)
        f2, t2, fl2 = O.noise_floor_from_raw(env, raw, d, p)
        assert np.array_equal(f1, f2, equal_nan=True), name
        assert np.array_equal(t1, t2), name
        assert (fl1 & 7) == fl2, name


def test_tie_report_is_exact():
    """The report is set iff some argsort order of the equal heights changes the
    distance filter's outcome: checked against every tie order (permutations
    of each equal-height block) on small random quantized envelopes."""
    import itertools
    import math
    rng = np.random.default_rng(7)
    for trial in range(300):
        n = int(rng.integers(20, 60))
        x = rng.integers(0, 4, n).astype(np.float64)
        cand = O.find_peaks(x)
        if cand.size < 2:
            continue
        dist = int(rng.integers(2, 8))
        _, tie = O.find_peaks(x, distance=dist, return_tie=True)
        pr = x[cand]
        outcomes = set()
        levels = sorted(set(pr.tolist()))
        blocks = [np.flatnonzero(pr == v) for v in levels]
        if np.prod([float(math.factorial(len(b))) for b in blocks]) > 5000:
            continue
        for perms in itertools.product(*[itertools.permutations(b) for b in blocks]):
            order = np.concatenate([np.array(pp, dtype=np.int64) for pp in perms])   # ascending priority
            keep = np.ones(cand.size, dtype=bool)
            for i in range(cand.size - 1, -1, -1):
                j = order[i]
                if not keep[j]:
                    continue
                for k in range(cand.size):
                    if k != j and abs(int(cand[k]) - int(cand[j])) < dist:
                        keep[k] = False
            outcomes.add(tuple(cand[keep].tolist()))
        assert tie == (len(outcomes) > 1), (x.tolist(), dist)


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
