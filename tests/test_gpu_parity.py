"""GPU parity: libbpmx.so (through the C ABI) against the oracle and the
reference's golden vectors.  Bit-exact for every index array and for the
reference-mode envelope, filtered signal and floor."""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests import goldens as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def det():
    from bpm_analysis_amd.engine import Detector
    return Detector(0)


def _same(a, b):
    return np.array_equal(np.asarray(a), np.asarray(b), equal_nan=True)


def _check_file(r, g, exact_env=True):
    if exact_env:
        assert _same(r["env"], g["env"])
        assert _same(r["floor"], g["floor"])
    else:
        scale = np.max(np.abs(g["env"])) or 1.0
        assert np.max(np.abs(r["env"] - g["env"])) <= 1e-9 * scale
        assert np.allclose(r["floor"], g["floor"], rtol=1e-9, atol=1e-9 * scale)
    assert _same(r["troughs"], g["troughs"])
    assert _same(r["peaks"], g["peaks"])
    _check_flags(r["flags"], int(g["flags"]))


FALLBACK_BITS = 3      # the flags the reference's log lines pin (static / draft fallback, :1074, :1109)
TIE_BITS = O.F_TROUGH_TIE | O.F_PEAK_TIE


def _check_flags(got, want):
    """Both sides masked the same way: the fallback bits equal, and no decisive
    find_peaks tie on an input the reference's output pins (tie cases have
    their own test)."""
    assert (got & FALLBACK_BITS) == (want & FALLBACK_BITS)
    assert got & TIE_BITS == 0


def test_device_synth_matches_host(det):
    import torch
    for fs, ch, lens in [(44100, 1, [44100 * 3, 44100 * 2 + 5, 1000]), (96000, 2, [96000 * 2, 77777])]:
        fo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        pcm = det.synth(fo, fs, ch, seed0=11).cpu().numpy()
        torch.cuda.synchronize()
        for f, n in enumerate(lens):
            want = O.synth(11 + f, n, fs, ch).reshape(-1)
            assert np.array_equal(pcm[fo[f] * ch:fo[f + 1] * ch], want)


@pytest.mark.parametrize("name", G.names(kind="pcm", mode="reference"))
def test_reference_mode_golden(det, name):
    g = G.load(name)
    r = det.run_host([g["pcm"]], int(g["fs"]), g["params"], mode="reference", want_y=True)[0]
    assert r["sr"] == int(g["sr"])
    assert _same(r["y"], g["y"])
    _check_file(r, g)


def test_ragged_batch_matches_single(det):
    names = ["ref_44k_60s_mono", "ref_44k_40s_clicks", "ref_44k_20s_wrap", "ref_44k_10s_zeros", "ref_44k_short16"]
    gs = [G.load(n) for n in names]
    short = O.synth(99, 146 * 15, 44100, 1)          # Nd = 15: filtfilt would raise -> flagged, batch survives
    recs = [g["pcm"] for g in gs[:2]] + [short] + [g["pcm"] for g in gs[2:]]
    res = det.run_host(recs, 44100, G.BASE_PARAMS, mode="reference")
    assert res[2]["flags"] & 8
    assert res[2]["n_raw_troughs"] == 0
    d = O.derive(44100, G.BASE_PARAMS)
    for r, g in zip(res[:2] + res[3:], gs):
        _check_file(r, g)
        # the "Kept X of Y initial troughs" count (bpm_analysis.py:1067-1069, :1099)
        prom = O.quantile(g["env"], G.BASE_PARAMS["trough_prominence_quantile"])
        assert r["n_raw_troughs"] == len(O.find_peaks(g["env"], distance=d.distance, prominence=prom, negate=True))


@pytest.mark.parametrize("name", [n for n in G.names(kind="env") if not n.startswith("env_ties")])
def test_env_level_golden(det, name):
    from bpm_analysis_amd import _native as N
    g = G.load(name)
    sr = int(g["sr"])
    r = det.run_env_host([g["env"]], sr, g["params"], N.STAGE_FLOOR)[0]
    assert _same(r["floor"], g["floor"])
    assert _same(r["troughs"], g["troughs"])
    _check_flags(r["flags"], int(g["flags"]))
    p = det.run_env_host([g["env"]], sr, g["params"], N.STAGE_PEAKS, floors=[g["floor"]])[0]
    assert _same(p["peaks"], g["peaks"])
    assert p["flags"] & TIE_BITS == 0


@pytest.mark.parametrize("name", G.names(kind="env", prefix="env_ties"))
def test_tie_goldens_flagged(det, name):
    """Equal-height extrema within find_peaks' distance (reference-made goldens:
    pairs of equal maxima / minima, the labeler envelope of quantized PCM).
    The kernels keep the stable order, so they equal the oracle; they set
    BPMX_F_TROUGH_TIE / BPMX_F_PEAK_TIE exactly where the oracle does, and
    wherever the reference's (numpy argsort) answer differs from theirs."""
    from bpm_analysis_amd import _native as N
    g = G.load(name)
    sr = int(g["sr"])
    d = G.env_derived(g)
    of, ot, ofl = O.noise_floor(g["env"], d, g["params"])
    r = det.run_env_host([g["env"]], sr, g["params"], N.STAGE_FLOOR)[0]
    assert _same(r["floor"], of) and _same(r["troughs"], ot)
    assert r["flags"] == ofl
    assert r["flags"] & N.F_TROUGH_TIE
    assert r["n_raw_troughs"] == len(O.find_peaks(g["env"], distance=d.distance, negate=True,
                                                  prominence=O.quantile(g["env"], g["params"]["trough_prominence_quantile"])))
    raw = O.find_peaks(g["env"], distance=d.distance, negate=True,
                       prominence=O.quantile(g["env"], g["params"]["trough_prominence_quantile"]))
    assert not _same(raw, g["raw_troughs"])           # the tie order decided something here
    # peaks on the reference's own floor: flagged, equal to the oracle's stable answer
    p = det.run_env_host([g["env"]], sr, g["params"], N.STAGE_PEAKS, floors=[g["floor"]])[0]
    opk, otie = O.raw_peaks(g["env"], g["floor"], d, g["params"], return_tie=True)
    assert _same(p["peaks"], opk)
    assert bool(p["flags"] & N.F_PEAK_TIE) == otie
    if not otie:
        assert _same(p["peaks"], g["peaks"])
    # the same envelopes through the one-workgroup global-memory kernel
    # (k_find_peaks): same outputs and flags
    for opt in (N.OPT_PEAKS_GLOBAL,):
        r2 = det.run_env_host([g["env"]], sr, g["params"], N.STAGE_FLOOR, options=opt)[0]
        assert _same(r2["troughs"], ot) and r2["flags"] == ofl
        p2 = det.run_env_host([g["env"]], sr, g["params"], N.STAGE_PEAKS, floors=[g["floor"]], options=opt)[0]
        assert _same(p2["peaks"], opk) and p2["flags"] == p["flags"]
    # FLOOR | PEAKS in one run: the peak launch of k_find_peaks_lds takes the
    # trough launch's extrema lists (bpmx_fpscan.h) on these plateau- and
    # tie-heavy envelopes; peaks and PEAK_TIE as the oracle's on its own floor
    opk2, otie2 = O.raw_peaks(g["env"], of, d, g["params"], return_tie=True)
    for opt in (0, N.OPT_PEAKS_GLOBAL):
        c = det.run_env_host([g["env"]], sr, g["params"], N.STAGE_FLOOR | N.STAGE_PEAKS, options=opt)[0]
        assert _same(c["floor"], of) and _same(c["troughs"], ot) and _same(c["peaks"], opk2)
        assert c["flags"] == ofl | (N.F_PEAK_TIE if otie2 else 0)


def _numpy_order_answer(env, d, params, floor=None):
    """The reference's answer on this machine (oracle restatement with numpy's
    own argsort order in find_peaks' distance filter)."""
    nf, nt, nfl, nraw = O.noise_floor_numpy_order(env, d, params)
    h = nf if floor is None else floor
    pk = O.find_peaks_numpy_order(env, height=h, distance=d.distance,
                                  prominence=O.quantile(env, params["peak_prominence_quantile"]))
    return nf, nt, nfl, nraw, pk


@pytest.mark.parametrize("name", G.names(kind="env", prefix="env_ties"))
def test_tie_goldens_resolved(det, name):
    """Decisive ties re-decided in numpy's argsort order (engine.resolve_ties,
    bpmx_run_ordered): the reference-made tie goldens' troughs, floor and raw
    peaks come out exactly, through the engine and through the drop-in."""
    from bpm_analysis_amd import _native as N, dropin
    g = G.load(name)
    sr = int(g["sr"])
    d = G.env_derived(g)
    nf, nt, nfl, nraw, npk = _numpy_order_answer(g["env"], d, g["params"])
    r = det.run_env_host([g["env"]], sr, g["params"], N.STAGE_FLOOR, resolve_ties=True)[0]
    assert _same(r["troughs"], nt) and _same(r["floor"], nf)
    assert r["n_raw_troughs"] == len(nraw)
    assert r["flags"] & TIE_BITS == 0 and r["flags"] & N.F_TROUGH_ORDERED
    p = det.run_env_host([g["env"]], sr, g["params"], N.STAGE_PEAKS, floors=[g["floor"]], resolve_ties=True)[0]
    c = det.run_env_host([g["env"]], sr, g["params"], N.STAGE_FLOOR | N.STAGE_PEAKS, resolve_ties=True)[0]
    assert _same(c["troughs"], nt) and _same(c["floor"], nf) and _same(c["peaks"], npk)
    assert p["flags"] & TIE_BITS == 0 and c["flags"] & TIE_BITS == 0
    # the reference's own outputs (made in the build container, whose numpy
    # argsort orders these heights as this box's does: the oracle's numpy-order
    # raw troughs equal the reference's here too)
    assert _same(nraw, g["raw_troughs"])
    assert _same(r["troughs"], g["troughs"]) and _same(r["floor"], g["floor"])
    assert _same(p["peaks"], g["peaks"]) and _same(c["peaks"], g["peaks"])
    # the drop-in (bpm_analysis.py:1064-1117, :223-229 signatures)
    fs, tr = dropin._calculate_dynamic_noise_floor(g["env"], sr, g["params"])
    assert _same(tr, nt) and _same(fs.values, nf)
    assert _same(dropin.find_raw_peaks(g["env"], sr, g["params"], g["floor"]), p["peaks"])


def test_tie_resolution_in_a_batch(det):
    """Many quantised (tie-heavy) envelopes with untied neighbours in one batch:
    the flagged recordings re-run as a sub-batch and are written back in place;
    every recording equals the numpy-order oracle, untied ones are untouched."""
    from bpm_analysis_amd import _native as N
    rng = np.random.default_rng(5)
    params = dict(G.BASE_PARAMS)
    sr = 302
    d = G.env_derived({"params": params, "sr": sr})
    envs = []
    for k in range(24):
        n = int(rng.integers(2500, 7000))
        t = np.arange(n)
        base = 5 + 100 * np.sin(t / 40.0) ** 2
        e = np.round(base + rng.random(n) * 6) / 3.0 if k % 3 else base + rng.random(n)
        envs.append(np.ascontiguousarray(e, dtype=np.float64))
    plain = det.run_env_host(envs, sr, params, N.STAGE_FLOOR | N.STAGE_PEAKS)
    res = det.run_env_host(envs, sr, params, N.STAGE_FLOOR | N.STAGE_PEAKS, resolve_ties=True)
    n_flagged = 0
    for e, a, r in zip(envs, plain, res):
        nf, nt, nfl, nraw, npk = _numpy_order_answer(e, d, params)
        assert _same(r["troughs"], nt) and _same(r["floor"], nf) and _same(r["peaks"], npk)
        assert r["n_raw_troughs"] == len(nraw)
        assert r["flags"] & TIE_BITS == 0
        if a["flags"] & TIE_BITS:
            n_flagged += 1
        else:
            assert _same(a["troughs"], r["troughs"]) and _same(a["peaks"], r["peaks"]) and a["flags"] == r["flags"]
    assert n_flagged >= 8


def test_vulpine_reference_pipeline_and_known_answer(det):
    from bpm_analysis_amd import _native as N
    g = G.load("vulpine")
    r = det.run_host([g["pcm"]], int(g["fs"]), g["params"], mode="reference")[0]
    _check_file(r, g)
    # labeler-recipe envelope (heartbeat_labeler.py:63-67) -> every Debug_Log raw peak;
    # its trough search meets a decisive tie (int16 |x| means are multiples of 1/30)
    env = O.rolling_mean(np.abs(g["pcm"]).astype(np.float64), int(g["fs"]) // 10, 1)
    fl = det.run_env_host([env], 302, g["params"], N.STAGE_FLOOR | N.STAGE_PEAKS)[0]
    assert _same(fl["peaks"], g["log_peaks"])
    assert fl["flags"] & TIE_BITS == N.F_TROUGH_TIE
    assert len(np.intersect1d(fl["troughs"], g["log_troughs"])) >= 1345
    # resolved in numpy's order: the reference's troughs and floor on this
    # machine (oracle numpy-order restatement), raw peaks still the log's
    d = O.derive(int(g["fs"]), g["params"])
    assert d.sr == 302
    nf, nt, nfl, nraw, npk = _numpy_order_answer(env, d, g["params"])
    rs = det.run_env_host([env], 302, g["params"], N.STAGE_FLOOR | N.STAGE_PEAKS, resolve_ties=True)[0]
    assert _same(rs["troughs"], nt) and _same(rs["floor"], nf) and _same(rs["peaks"], npk)
    assert rs["flags"] & TIE_BITS == 0 and rs["flags"] & N.F_TROUGH_ORDERED
    assert _same(rs["peaks"], g["log_peaks"])


def test_synthetic_batch_vs_oracle(det):
    """64 x 60 s recordings generated in HBM; 6 of them re-derived by the oracle
    bit for bit, all of them checked for structural invariants."""
    import torch
    fs, F, n = 44100, 64, 44100 * 60
    fo = np.arange(F + 1, dtype=np.int64) * n
    pcm = det.synth(fo, fs, 1, seed0=1000)
    params = dict(G.BASE_PARAMS)
    res = det.run(pcm, fo, fs, params, mode="reference")
    torch.cuda.synchronize()
    host = res.to_host()
    for f in [0, 1, 17, 31, 48, 63]:
        o = O.detect(O.synth(1000 + f, n, fs, 1), fs, params)
        assert _same(host[f]["env"], o["env"])
        assert _same(host[f]["floor"], o["floor"])
        assert _same(host[f]["troughs"], o["troughs"])
        assert _same(host[f]["peaks"], o["peaks"])
    for h in host:
        pk, env, fl = h["peaks"], h["env"], h["floor"]
        assert len(pk) > 100 and np.all(np.diff(pk) >= 15)
        assert np.all(env[pk] >= fl[pk])


def test_dropin_functions(det, tmp_path):
    import pandas as pd
    from scipy.io import wavfile

    import bpm_analysis_amd as B
    g = G.load("ref_48k_20s_mono")
    wav = tmp_path / "rec.wav"
    wavfile.write(str(wav), int(g["fs"]), g["pcm"])
    params = dict(B.DEFAULT_PARAMS)
    env, sr = B.preprocess_audio(str(wav), params, str(tmp_path))
    assert sr == int(g["sr"]) and _same(env, g["env"])
    assert (tmp_path / "rec_filtered_debug.wav").exists()
    floor, troughs = B._calculate_dynamic_noise_floor(env, sr, params)
    assert isinstance(floor, pd.Series) and _same(floor.values, g["floor"])
    assert troughs.dtype == np.int64 and _same(troughs, g["troughs"])
    peaks = B.find_raw_peaks(env, sr, params, floor.values)
    assert _same(peaks, g["peaks"])
    with pytest.raises(ValueError):
        short = tmp_path / "short.wav"
        wavfile.write(str(short), 44100, O.synth(1, 146 * 15, 44100, 1))
        B.preprocess_audio(str(short), params, str(tmp_path))


@pytest.mark.parametrize("name", G.names(kind="pcm", mode="native"))
def test_native_mode_golden(det, name):
    """north_star ordering (sosfiltfilt @ fs -> [::ds] -> |hilbert| -> rolling mean):
    envelope within 1e-9 relative of the scipy composition, indices exact."""
    g = G.load(name)
    r = det.run_host([g["pcm"]], int(g["fs"]), g["params"], mode="native", want_y=True)[0]
    assert r["sr"] == int(g["sr"])
    scale = np.max(np.abs(g["y"]))
    assert np.max(np.abs(r["y"] - g["y"])) <= 1e-9 * scale
    _check_file(r, g, exact_env=False)


def test_native_ragged_batch(det):
    names = ["nat_44k_60s_mono", "nat_44k_40s_clicks"]
    gs = [G.load(n) for n in names]
    res = det.run_host([g["pcm"] for g in gs], 44100, G.BASE_PARAMS, mode="native")
    for r, g in zip(res, gs):
        _check_file(r, g, exact_env=False)


@pytest.mark.parametrize("fs,lens,shift,ch", [
    (44100, [44100 * 7 + 3, 44100 * 5 + 1, 146 * 16 + 7, 44100 * 3], 0, 1),   # odd file offsets, tiny file
    (96000, [96000 * 6 + 5, 96000 * 4], 0, 1),                               # ds = 300: 34-block tiles
    (44100, [44100 * 6 + 1, 44100 * 4 + 2], 1, 1),                           # pcm not 16-B aligned: generic path
    (48000, [48000 * 5 + 3, 48000 * 3 + 1], 1, 2),                           # stereo, not 4-B aligned: generic path
    (44100, [44100 * 4 + 2, 44100 * 3 + 5], 0, 3),                           # three channels: generic path
])
def test_native_tile_geometries(det, fs, lens, shift, ch):
    import torch
    recs = [O.synth(500 + i, n, fs, ch) for i, n in enumerate(lens)]
    flat = np.concatenate([np.zeros(shift, np.int16)] + [r.reshape(-1) for r in recs])
    dev = torch.from_numpy(flat).to(det.device)[shift:]
    fo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    params = dict(G.BASE_PARAMS)
    res = det.run(dev, fo, fs, params, mode="native", want_y=True, channels=ch)
    torch.cuda.synchronize()
    for h, pcm in zip(res.to_host(), recs):
        o = O.detect(pcm, fs, params, mode="native")
        scale = np.max(np.abs(o["y"]))
        assert np.max(np.abs(h["y"] - o["y"])) <= 1e-9 * scale
        _check_file(h, o, exact_env=False)


@pytest.mark.parametrize("mode", ["native", "reference"])
def test_config_c2_ten_minute_recording(det, mode):
    """BASELINE config C2: one 10-min 44.1 kHz mono recording (Nd = 181,233:
    the long-recording kernels — sorted-union rolling quantile, global block
    tables, multi-pass quantile) against the oracle."""
    fs, n = 44100, 44100 * 600
    pcm = O.synth(4242, n, fs, 1)
    params = dict(G.BASE_PARAMS)
    r = det.run_host([pcm], fs, params, mode=mode, want_y=True)[0]
    o = O.detect(pcm, fs, params, mode=mode)
    if mode == "native":
        scale = np.max(np.abs(o["y"]))
        assert np.max(np.abs(r["y"] - o["y"])) <= 1e-9 * scale
    _check_file(r, o, exact_env=(mode == "reference"))
    assert len(r["peaks"]) > 1000


def test_config_c5_96k_stereo_ragged(det):
    """BASELINE config C5 (scaled down in length): 96 kHz stereo recordings of
    ragged lengths in one batch (ds = 300, two channels averaged on device),
    native mode, against the oracle."""
    import torch
    fs = 96000
    lens = [96000 * 150 + 17, 96000 * 61, 96000 * 247 + 3]
    recs = [O.synth(700 + i, n, fs, 2) for i, n in enumerate(lens)]
    dev = torch.from_numpy(np.concatenate([r.reshape(-1) for r in recs])).to(det.device)
    fo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    params = dict(G.BASE_PARAMS)
    res = det.run(dev, fo, fs, params, mode="native", channels=2, want_y=True)
    torch.cuda.synchronize()
    for h, pcm in zip(res.to_host(), recs):
        o = O.detect(pcm, fs, params, mode="native")
        assert h["sr"] == o["sr"] == 320
        scale = np.max(np.abs(o["y"]))
        assert np.max(np.abs(h["y"] - o["y"])) <= 1e-9 * scale
        _check_file(h, o, exact_env=False)


def test_config_c5_full_length_recording(det):
    """BASELINE config C5 at its maximum size: one 30-min 96 kHz stereo
    recording (172.8 M frames, 691 MB of PCM, Nd = 576,000: rocFFT Hilbert
    fallback, sorted-union rolling quantile, global find_peaks tables)."""
    import torch
    fs, n = 96000, 96000 * 1800
    fo = np.array([0, n], dtype=np.int64)
    dev = det.synth(fo, fs, 2, seed0=777)
    params = dict(G.BASE_PARAMS)
    res = det.run(dev, fo, fs, params, mode="native", channels=2, want_y=True)
    torch.cuda.synchronize()
    h = res.to_host()[0]
    del dev
    o = O.detect(O.synth(777, n, fs, 2), fs, params, mode="native")
    assert h["sr"] == o["sr"] == 320 and len(h["env"]) == 576000
    scale = np.max(np.abs(o["y"]))
    assert np.max(np.abs(h["y"] - o["y"])) <= 1e-9 * scale
    _check_file(h, o, exact_env=False)


def test_analyze_wav_files_batched_ingest(det, tmp_path):
    """WAV files of mixed formats in one call — grouped by
    (rate, format, channels), each group one ragged batch — against the
    oracle bit for bit (reference mode), both debug WAVs as the reference
    writes them, and the padlen ValueError for a too-short file."""
    from scipy.io import wavfile
    from bpm_analysis_amd import dropin
    params = dict(G.BASE_PARAMS, save_filtered_wav=True)
    cases = [("a_i16.wav", 44100, O.synth(31, 44100 * 20, 44100, 1)),
             ("b_i16_stereo.wav", 48000, O.synth(32, 48000 * 15, 48000, 2)),
             ("c_f32.wav", 44100, (O.synth(33, 44100 * 12, 44100, 1) / 32768.0).astype(np.float32)),
             ("d_i16.wav", 44100, O.synth(34, 44100 * 9 + 5, 44100, 1)),
             ("e_short.wav", 44100, O.synth(35, 146 * 15, 44100, 1))]
    paths = []
    for name, fs, pcm in cases:
        paths.append(str(tmp_path / name))
        wavfile.write(paths[-1], fs, pcm)
    outdir = tmp_path / "out"
    outdir.mkdir()
    res = dropin.analyze_wav_files(paths, params, str(outdir), mode="reference")
    for (name, fs, pcm), path, r in zip(cases, paths, res):
        if name.startswith("e_"):
            assert isinstance(r["error"], ValueError) and "padlen" in str(r["error"])
            continue
        o = O.detect(wavfile.read(path)[1], fs, params, mode="reference")
        assert _same(r["env"], o["env"]) and _same(r["floor"], o["floor"])
        assert _same(r["troughs"], o["troughs"]) and _same(r["peaks"], o["peaks"])
        want = np.int16(o["y"] / np.max(np.abs(o["y"])) * 32767)
        for dbg in (path[:-4] + "_filtered_debug.wav", str(outdir / (name[:-4] + "_filtered_debug.wav"))):
            sr, got = wavfile.read(dbg)
            assert sr == o["sr"] and _same(got, want)


def test_reference_side_ctypes_stub():
    """INTEGRATION.md's torch-free ctypes binding of the C ABI, on a golden."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ctypes_stub", os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "ctypes_stub.py"))
    stub = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(stub)
    import bpm_analysis_amd as B
    g = G.load("ref_44k_60s_mono")
    env, floor, tr, pk, sr = stub.analyze(g["pcm"], int(g["fs"]), dict(B.DEFAULT_PARAMS))
    assert sr == int(g["sr"])
    assert _same(env, g["env"]) and _same(floor, g["floor"])
    assert _same(tr, g["troughs"]) and _same(pk, g["peaks"])


@pytest.mark.parametrize("name", ["ref_44k_60s_mono", "ref_44k_40s_clicks", "ref_96k_20s_stereo"])
def test_rolling_quantile_kernels_agree(det, name):
    """The wavelet-matrix rolling quantile (default), the sorted-union kernel
    (BPMX_OPT_ROLLQ_MERGE) and its global-memory form (BPMX_OPT_ROLLQ_GLOBAL)
    all reproduce the golden floor bit for bit."""
    from bpm_analysis_amd import _native as N
    g = G.load(name)
    for opt in (0, N.OPT_ROLLQ_MERGE, N.OPT_ROLLQ_GLOBAL):
        r = det.run_host([g["pcm"]], int(g["fs"]), g["params"], mode="reference", options=opt)[0]
        _check_file(r, g)


def _floor_envelopes():
    """Envelopes that stress the final-floor pruning: golden env cases, the
    vulpine labeler envelope, near-constant floors (ulp-level differences),
    steep trends, random roughness, > WM_TRMAX troughs (unpruned path) and
    short recordings dominated by edge windows."""
    rng = np.random.default_rng(7)
    out = [(G.load(n)["env"], int(G.load(n)["sr"])) for n in G.names(kind="env")]
    g = G.load("vulpine")
    out.append((O.rolling_mean(np.abs(g["pcm"]).astype(np.float64), int(g["fs"]) // 10, 1), 302))
    n = 18124
    t = np.arange(n)
    beat = np.maximum(0.0, np.sin(2 * np.pi * t / 250.0)) ** 8
    out.append((10.0 + np.spacing(10.0) * rng.integers(0, 5, n) + 300 * beat, 302))         # ulp-level floor
    out.append((10.0 + 0.05 * t + 3000 * beat + rng.random(n), 302))                           # ramp
    out.append((rng.random(n) ** 3 * 1000 + 50 * beat, 302))                                   # rough
    out.append((np.abs(np.sin(t / 9.0)) * 100 + rng.random(n), 302))                           # > 512 troughs
    out.append((200 + 80 * np.sin(t / 700.0) + 300 * beat + rng.random(n), 302))              # slow wander
    out.append((300 * beat[:4000] + rng.random(4000) + 20, 302))                               # short
    return out


def test_rollq_pruning_exact(det):
    """The pruned wavelet-matrix floor (default) equals the unpruned one
    (BPMX_OPT_ROLLQ_NOPRUNE) and the oracle bit for bit on every envelope."""
    from bpm_analysis_amd import _native as N
    params = dict(G.BASE_PARAMS)
    for env, sr in _floor_envelopes():
        a = det.run_env_host([env], sr, params, N.STAGE_FLOOR)[0]
        b = det.run_env_host([env], sr, params, N.STAGE_FLOOR, options=N.OPT_ROLLQ_NOPRUNE)[0]
        assert _same(a["floor"], b["floor"])
        assert _same(a["troughs"], b["troughs"])
        d = O.derive(sr, params)
        of, ot, _ = O.noise_floor(env, d, params)
        assert _same(a["floor"], of)
        assert _same(a["troughs"], ot)


def test_long_quantiles_adversarial(det):
    """Long recordings' quantiles (k_qv_*: key bins over the recording's own
    range, the target bin's keys gathered, an exact select among them) on
    envelopes that put many keys in one bin or spread them over the whole
    double range: floor, troughs, raw peaks and flags equal to the oracle
    (np.quantile, bit for bit), in one ragged batch with short recordings."""
    from bpm_analysis_amd import _native as N
    params = dict(G.BASE_PARAMS)
    rng = np.random.default_rng(23)
    m = 60_000
    t = np.arange(m)
    beat = np.maximum(0.0, np.sin(2 * np.pi * t / 250.0)) ** 8
    envs = [
        np.full(m, 7.0) + 300 * (t % 911 == 0),                              # one value nearly everywhere
        np.geomspace(1e-300, 1e300, m)[rng.permutation(m)] + 0.0,              # every octave of the range
        np.round(10.0 + 0.001 * t, 1) + 300 * beat,                            # long runs of equal values
        np.where(t % 3 == 0, 0.0, 1e-12 * rng.random(m)) + 50 * beat,          # zeros and tiny values
        rng.pareto(1.5, m) + 30 * beat,                                        # heavy tail
        300 * beat[:20_000] + rng.random(20_000),                              # short: k_quantile_reg
    ]
    sr = 302
    d = O.derive(sr, params)
    got = det.run_env_host(envs, sr, params, N.STAGE_FLOOR | N.STAGE_PEAKS)
    for env, r in zip(envs, got):
        of, ot, ofl = O.noise_floor(env, d, params)
        opk = O.raw_peaks(env, of, d, params)
        assert _same(r["floor"], of)
        assert _same(r["troughs"], ot)
        assert _same(r["peaks"], opk)
        mask = FALLBACK_BITS | 4 | O.F_TROUGH_TIE       # decisive-tie reports: the oracle's are exact too
        assert (r["flags"] & mask) == (ofl & mask)


def test_find_peaks_kernels_agree(det):
    """find_peaks with prominences from the LDS-resident local extrema
    (k_find_peaks_lds, default) equals the sample walks over global memory
    (k_find_peaks, BPMX_OPT_PEAKS_GLOBAL) bit for bit, troughs and peaks, on
    every floor-stress envelope plus plateau-heavy and > 3072-maxima ones
    (those the LDS kernel hands over), all in one ragged batch."""
    from bpm_analysis_amd import _native as N
    params = dict(G.BASE_PARAMS)
    rng = np.random.default_rng(11)
    envs = [e for e, sr in _floor_envelopes() if sr == 302]
    n = 18124
    envs.append(np.round(rng.random(n) * 4) + 100 * (np.arange(n) % 300 == 0))     # plateaus, ties
    envs.append(rng.random(n) * 10)                                                 # ~6000 maxima
    envs.append(np.repeat(rng.random(n // 8), 8))                                   # flat runs
    stages = N.STAGE_FLOOR | N.STAGE_PEAKS
    a = det.run_env_host(envs, 302, params, stages)
    b = det.run_env_host(envs, 302, params, stages, options=N.OPT_PEAKS_GLOBAL)
    for x, y in zip(a, b):
        assert _same(x["troughs"], y["troughs"])
        assert _same(x["peaks"], y["peaks"])
        assert _same(x["floor"], y["floor"])
        assert x["flags"] == y["flags"]                 # decisive-tie reports included
    assert any(x["flags"] & TIE_BITS for x in a)
    # with recordings beyond 65536 samples in the batch, the long ones and the
    # short ones with > 3072 maxima take the multi-workgroup k_fpl_* path
    m = 200_000
    t = np.arange(m)
    beat = np.maximum(0.0, np.sin(2 * np.pi * t / 250.0)) ** 8
    long_envs = [
        10.0 + 0.001 * t + 3000 * beat + rng.random(m),                     # rising: long prominence walks
        np.concatenate([np.full(70_000, 5.0), 300 * beat[:70_000] + 20]),    # flat head: edge gaps
        np.round(rng.random(m) * 3) + 200 * (t % 700 == 0),                 # plateaus and ties everywhere
        300 * beat[:66_000] + rng.random(66_000),
        # sparse maxima (k_fpl_dist_ch cuts them into chunks) then dense noise
        # (one component past the chunk halo: k_fpl_distance finishes the rest)
        np.concatenate([300 * beat[:100_000] + 20, rng.random(100_000) * 10 + 5]),
    ]
    envs2 = long_envs + envs[-3:]
    a = det.run_env_host(envs2, 302, params, stages)
    b = det.run_env_host(envs2, 302, params, stages, options=N.OPT_PEAKS_GLOBAL)
    for x, y in zip(a, b):
        assert _same(x["troughs"], y["troughs"])
        assert _same(x["peaks"], y["peaks"])
        assert _same(x["floor"], y["floor"])
        assert x["flags"] == y["flags"]
    d = O.derive(302, params)
    for k in (0, 2):                   # 2: ties everywhere, through k_fpl_prom's tie check
        of, ot, ofl = O.noise_floor(long_envs[k], d, params)
        opk, ptie = O.raw_peaks(long_envs[k], of, d, params, return_tie=True)
        assert _same(a[k]["troughs"], ot)
        assert _same(a[k]["peaks"], opk)
        assert a[k]["flags"] == ofl | (O.F_PEAK_TIE if ptie else 0)
    assert a[2]["flags"] & TIE_BITS
    # a tied recording beyond 65536 samples through engine.resolve_ties (the
    # ordered sub-batch takes the single-workgroup k_find_peaks with the run's
    # own options forwarded), beside a tied short one: numpy's order exactly
    for opt in (0, N.OPT_PEAKS_GLOBAL):
        pair = [long_envs[2], envs[-3]]
        rs = det.run_env_host(pair, 302, params, stages, options=opt, resolve_ties=True)
        for e, r in zip(pair, rs):
            nf, nt, nfl, nraw, npk = _numpy_order_answer(e, d, params)
            assert _same(r["troughs"], nt) and _same(r["floor"], nf) and _same(r["peaks"], npk)
            assert r["n_raw_troughs"] == len(nraw)
            assert r["flags"] & TIE_BITS == 0


@pytest.mark.parametrize("fs", [44100, 22050, 48000])
def test_native_block_kernels_agree(det, fs):
    """The exact-integer matrix-core block projections (default for int16 mono,
    ds + 1 <= 160) are at least as close to the oracle's sosfiltfilt as the f64
    VALU kernel (BPMX_OPT_NATIVE_F64), and both give the oracle's indices."""
    import torch
    from bpm_analysis_amd import _native as N
    lens = [fs * 9 + 77, fs * 6, fs * 4 + 3]
    recs = [O.synth(900 + i, n, fs, 1) for i, n in enumerate(lens)]
    dev = torch.from_numpy(np.concatenate(recs)).to(det.device)
    fo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    params = dict(G.BASE_PARAMS)
    outs = []
    for opt in (0, N.OPT_NATIVE_F64):
        res = det.run(dev, fo, fs, params, mode="native", want_y=True, options=opt)
        torch.cuda.synchronize()
        outs.append(res.to_host())
    for a, b, pcm in zip(outs[0], outs[1], recs):
        o = O.detect(pcm, fs, params, mode="native")
        scale = np.max(np.abs(o["y"]))
        ea, eb = np.max(np.abs(a["y"] - o["y"])), np.max(np.abs(b["y"] - o["y"]))
        print(f"fs={fs} n={len(pcm)}: |y_mfma - y_oracle| = {ea / scale:.3e}, |y_f64 - y_oracle| = {eb / scale:.3e} (rel)")
        assert ea <= max(2 * eb, 1e-12 * scale)
        assert ea <= 1e-9 * scale
        _check_file(a, o, exact_env=False)
        _check_file(b, o, exact_env=False)


def test_fused_hilbert_matches_rocfft_and_oracle(det):
    """k_hilbert_env (in-LDS mixed-radix transform + rolling mean) against the
    batched Bluestein transform (BPMX_OPT_HILBERT_ROCFFT: every recording),
    the per-length rocFFT R2C/C2R path (+ BPMX_OPT_HILBERT_R2C) and the oracle,
    on a ragged batch whose Nd exercise radix 2 / 3 / 5 / 23 / 197 / 401 plans,
    a tiny plan, and odd or large-prime Nd that fall back inside the same
    batch (packed and unpacked Bluestein groups)."""
    import torch
    from bpm_analysis_amd import _native as N
    fs, ds = 44100, 146
    nds = [18124, 9000, 2406, 1000, 18, 402, 12083, 6038]
    lens = [nd * ds - (i % 3) for i, nd in enumerate(nds)]
    recs = [O.synth(700 + i, n, fs, 1) for i, n in enumerate(lens)]
    dev = torch.from_numpy(np.concatenate(recs)).to(det.device)
    fo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    params = dict(G.BASE_PARAMS)
    outs = []
    # default (fused where it plans, batched Bluestein elsewhere), Bluestein for
    # all (BPMX_OPT_HILBERT_ROCFFT), per-length rocFFT R2C/C2R for all
    for opt in (0, N.OPT_HILBERT_ROCFFT, N.OPT_HILBERT_ROCFFT | N.OPT_HILBERT_R2C):
        res = det.run(dev, fo, fs, params, mode="native", want_y=True, options=opt)
        torch.cuda.synchronize()
        outs.append(res.to_host())
    for a, b, c, pcm in zip(outs[0], outs[1], outs[2], recs):
        scale = np.max(np.abs(c["env"]))
        assert np.max(np.abs(a["env"] - c["env"])) <= 1e-12 * scale
        assert np.max(np.abs(b["env"] - c["env"])) <= 1e-12 * scale
        if len(pcm) > 5000 * ds:
            o = O.detect(pcm, fs, params, mode="native")
            _check_file(a, o, exact_env=False)
            _check_file(b, o, exact_env=False)


@pytest.mark.parametrize("name", ["ref_44k_60s_mono", "ref_44k_40s_clicks", "vulpine", "env_random_rough",
                                  "env_plateaus", "env_draft_fallback", "env_random_long_window", "env_static_fallback"])
def test_draft_bounds_match_full_draft(det, name):
    """k_draft_bounds (keep decisions from the draft's bracket, the full draft
    only where one is undecided) gives the golden floor, troughs, flags and
    peaks, bit for bit, as does computing the draft in full (BPMX_OPT_DRAFT_FULL)."""
    from bpm_analysis_amd import _native as N
    g = G.load(name)
    for opt in (0, N.OPT_DRAFT_FULL):
        r = det.run_env_host([g["env"]], int(g["sr"]), g["params"], N.STAGE_FLOOR | N.STAGE_PEAKS, options=opt)[0]
        assert _same(r["floor"], g["floor"])
        assert _same(r["troughs"], g["troughs"])
        _check_flags(r["flags"], int(g["flags"]))
        assert _same(r["peaks"], g["peaks"])


def test_beat_stages_on_gpu_outputs(tmp_path):
    """the host beat stages (classifier, refinement,
    BPM curve, slopes/HRR/HRV) on the GPU path's outputs of a batched run, against
    goldens made by the reference (tests/golden/beats); the long recordings are
    regenerated PCM, so everything upstream of the classifier ran on the GPU."""
    import json
    from scipy.io import wavfile
    from bpm_analysis_amd import beats as B, dropin
    from tests import test_beats as TB
    from tests.golden import inputs as I
    names = ["long_6k_8min", "long_8k_5min_hint"]
    for name in names:
        g, params, hint, _ = TB.load_case(name)
        spec = json.loads(str(g["spec"]))
        pcm, fs = I.make_input(spec)
        r = dropin.analyze_batch([pcm], fs, params, mode="reference")[0]
        assert np.array_equal(r["peaks"], g["all_raw_peaks"])
        res = B.analyze_many([r], params, hint)[0]
        TB.check_against_golden(g, res)
        # the reference entry point end to end: WAV in, <base>_bpm_plot.csv out
        wav = tmp_path / f"{name}.wav"
        wavfile.write(str(wav), fs, pcm)
        p = dict(params, save_filtered_wav=False)
        assert B.analyze_wav_file(str(wav), p, hint, str(wav), str(tmp_path)) is None
        assert (tmp_path / f"{name}_bpm_plot.csv").read_text() == str(g["csv"])
        assert TB._drop_stamp((tmp_path / f"{name}_Analysis_Summary.md").read_text()) == str(g["summary_md"])
        assert TB._drop_stamp((tmp_path / f"{name}_Debug_Log.md").read_text()) == str(g["debug_log_md"])
        assert (tmp_path / f"{name}_Analysis_Settings.json").read_text() == str(g["settings_json"])
        assert (tmp_path / f"{name}_bpm_plot.html").stat().st_size > 0


def test_beat_stages_batch_of_hot_path_goldens():
    """Every regenerable hot-path golden in one ragged GPU batch per rate, then
    the beat stages per file against the reference's beat goldens."""
    from bpm_analysis_amd import beats as B, dropin
    from tests import test_beats as TB
    for name in ["ref_44k_60s_mono", "ref_44k_60s_mono_hint", "ref_44k_40s_clicks", "ref_44k_20s_wrap"]:
        g, params, hint, inp = TB.load_case(name)
        h = G.load(str(g["source"]))
        r = dropin.analyze_batch([h["pcm"]], int(h["fs"]), params, mode="reference")[0]
        assert np.array_equal(r["env"], inp["env"]) and np.array_equal(r["peaks"], inp["peaks"])
        TB.check_against_golden(g, B.analyze_many([r], params, hint)[0])


def test_longest_first_order_is_transparent(det):
    """run_host's longest-first dispatch order (shard.py) returns the caller's order, unchanged results."""
    names = ["ref_44k_20s_wrap", "ref_44k_60s_mono", "ref_44k_short16", "ref_44k_40s_clicks"]
    gs = [G.load(n) for n in names]
    a = det.run_host([g["pcm"] for g in gs], 44100, G.BASE_PARAMS, mode="reference")
    b = det.run_host([g["pcm"] for g in gs], 44100, G.BASE_PARAMS, mode="reference", longest_first=False)
    for g, ra, rb in zip(gs, a, b):
        for k in ("env", "floor", "troughs", "peaks"):
            assert _same(ra[k], rb[k]), k
        assert ra["flags"] == rb["flags"]
        if not (ra["flags"] & 8):
            _check_file(ra, g)


@pytest.mark.parametrize("secs", [0, 420, 1500])
def test_draft_bounds_window_ranking(det, secs):
    """k_draft_bounds ranks each window's segments in place for recordings of
    > 512 troughs; the recording-wide order (BPMX_OPT_DRAFT_GLOBAL_RANK) and the
    full draft give the same floor, troughs and peaks (vulpine: 1456 raw
    troughs; a 7-min recording: ~1700; a 25-min one: ~6000, staged per chunk),
    and the oracle agrees."""
    from bpm_analysis_amd import _native as N
    if secs == 0:
        g = G.load("vulpine")
        env, sr, params = g["env"], int(g["sr"]), g["params"]
        want = g
    else:
        pcm = O.synth(123, 44100 * secs, 44100, 1)
        o = O.detect(pcm, 44100, G.BASE_PARAMS, mode="reference")
        env, sr, params, want = o["env"], o["sr"], G.BASE_PARAMS, o
    runs = [det.run_env_host([env], sr, params, N.STAGE_FLOOR | N.STAGE_PEAKS, options=opt)[0]
            for opt in (0, N.OPT_DRAFT_GLOBAL_RANK, N.OPT_DRAFT_FULL)]
    for r in runs:
        assert _same(r["floor"], want["floor"])
        assert _same(r["troughs"], want["troughs"])
        assert _same(r["peaks"], want["peaks"])


def _stand_in_reference():
    """A minimal stand-in for the reference module: the three hot-path names
    (unpatched they raise) and a PeakClassifier whose constructor runs
    _initialize_state the way bpm_analysis.py:80-91 does, plus the first stages
    of analyze_wav_file (:1731-1740)."""
    import types
    mod = types.ModuleType("bpm_analysis_stand_in")

    def unpatched(*a, **k):
        raise AssertionError("reference hot path called: patch_reference did not rebind it")

    class PeakClassifier:
        def __init__(self, audio_envelope, sample_rate, params, start_bpm_hint, precomputed_noise_floor,
                     precomputed_troughs, peak_bpm_time_sec, recovery_end_time_sec):
            self.audio_envelope = audio_envelope
            self.sample_rate = sample_rate
            self.params = params
            self.state = self._initialize_state(start_bpm_hint, precomputed_noise_floor, precomputed_troughs)

        def _initialize_state(self, start_bpm_hint, precomputed_noise_floor, precomputed_troughs):
            state = {"analysis_data": {}}
            state["dynamic_noise_floor"], state["trough_indices"] = precomputed_noise_floor, precomputed_troughs
            state["all_peaks"] = self._find_raw_peaks(state["dynamic_noise_floor"].values)
            return state

        _find_raw_peaks = unpatched

    def analyze_wav_file(wav_file_path, params, start_bpm_hint, original_file_path, output_directory):
        env, sr = mod.preprocess_audio(wav_file_path, params, output_directory)
        floor, troughs = mod._calculate_dynamic_noise_floor(env, sr, params)
        pc = mod.PeakClassifier(env, sr, params, start_bpm_hint, floor, troughs, None, None)
        return env, floor, troughs, pc.state["all_peaks"]

    mod.preprocess_audio = unpatched
    mod._calculate_dynamic_noise_floor = unpatched
    mod.PeakClassifier = PeakClassifier
    mod.analyze_wav_file = analyze_wav_file
    return mod


def test_patch_reference_runs_the_reference_entry_on_the_gpu(det, tmp_path):
    """dropin.patch_reference rebinds a reference module's hot path; the
    module's own entry point then runs it through libbpmx.so (bit-exact)."""
    from scipy.io import wavfile
    from bpm_analysis_amd import dropin
    mod = _stand_in_reference()
    dropin.patch_reference(mod)
    g = G.load("ref_44k_60s_mono")
    wav = tmp_path / "rec.wav"
    wavfile.write(str(wav), int(g["fs"]), g["pcm"])
    params = dict(g["params"], save_filtered_wav=False)
    env, floor, troughs, peaks = mod.analyze_wav_file(str(wav), params, None, str(wav), str(tmp_path))
    assert _same(env, g["env"]) and _same(floor.values, g["floor"])
    assert _same(troughs, g["troughs"]) and _same(peaks, g["peaks"])


def test_reference_value_errors(det, tmp_path):
    """The reference's ValueErrors at the boundary: scipy's distance check, and
    pandas' rolling-window check, which fires only for recordings that reach
    the rolling quantile (>= 5 troughs); per file in the batched entry."""
    from scipy.io import wavfile
    import bpm_analysis_amd as B
    from bpm_analysis_amd import dropin
    g = G.load("ref_44k_60s_mono")
    env, sr = g["env"], int(g["sr"])
    with pytest.raises(ValueError, match="min_periods 3 must be <= window 1"):
        B._calculate_dynamic_noise_floor(env, sr, dict(g["params"], noise_window_sec=0.005))
    with pytest.raises(ValueError, match="min_periods 3 must be <= window -302"):
        B._calculate_dynamic_noise_floor(env, sr, dict(g["params"], noise_window_sec=-1.0))
    with pytest.raises(ValueError, match="`distance` must be greater or equal to 1"):
        B._calculate_dynamic_noise_floor(env, sr, dict(g["params"], min_peak_distance_sec=0.001))
    # < 5 troughs: the static floor is returned before the window is used
    s = G.load("env_static_fallback")
    fl, tr = B._calculate_dynamic_noise_floor(s["env"], int(s["sr"]), dict(s["params"], noise_window_sec=0.005))
    assert _same(fl.values, s["floor"]) and _same(tr, s["troughs"])
    # a library E_ARG is a ValueError too
    from bpm_analysis_amd import _native as N
    with pytest.raises(ValueError):
        det.run_env_host([env], sr, dict(g["params"], min_peak_distance_sec=0.001), N.STAGE_PEAKS, floors=[env])
    paths = []
    for name, pcm in [("a.wav", g["pcm"]), ("b.wav", O.synth(3, 146 * 15, 44100, 1))]:
        paths.append(str(tmp_path / name))
        wavfile.write(paths[-1], 44100, pcm)
    res = dropin.analyze_wav_files(paths, dict(g["params"], noise_window_sec=0.005), str(tmp_path))
    assert "min_periods 3" in str(res[0]["error"]) and "padlen" in str(res[1]["error"])
    res = dropin.analyze_wav_files(paths, dict(g["params"], min_peak_distance_sec=0.001), str(tmp_path))
    assert "distance" in str(res[0]["error"]) and "padlen" in str(res[1]["error"])


def test_native_batch_at_c3_scale(det):
    """BASELINE config C3: 256 x 60 s 44.1 kHz mono recordings in one native-mode
    batch generated in HBM; 16 of them re-derived by the oracle (indices exact,
    envelope/floor within 1e-9 of max|env|), all of them checked for the
    find_peaks invariants."""
    import torch
    fs, F, n = 44100, 256, 44100 * 60
    fo = np.arange(F + 1, dtype=np.int64) * n
    pcm = det.synth(fo, fs, 1, seed0=5000)
    params = dict(G.BASE_PARAMS)
    res = det.run(pcm, fo, fs, params, mode="native")
    torch.cuda.synchronize()
    host = res.to_host()
    del pcm
    for f in np.linspace(0, F - 1, 16).astype(int):
        o = O.detect(O.synth(5000 + int(f), n, fs, 1), fs, params, mode="native")
        _check_file(host[f], o, exact_env=False)
    for h in host:
        pk, env, fl, tr = h["peaks"], h["env"], h["floor"], h["troughs"]
        assert len(pk) > 100 and np.all(np.diff(pk) >= 15) and np.all(np.diff(tr) >= 15)
        assert np.all(env[pk] >= fl[pk]) and h["flags"] == 0


@pytest.mark.parametrize("secs,window", [(600, 30.0), (180, 90.0), (75, 45.0)])
def test_long_noise_window_on_long_recording(det, secs, window):
    """noise_window_sec beyond the LDS kernels on recordings longer than the
    wavelet-matrix limit (bpm_analysis.py:1083-1085 takes any window): the
    global-memory sorted union, bit-exact against the oracle (reference mode)."""
    params = dict(G.BASE_PARAMS, noise_window_sec=window)
    pcm = O.synth(31337 + secs, 44100 * secs, 44100, 1)
    r = det.run_host([pcm], 44100, params, mode="reference")[0]
    o = O.detect(pcm, 44100, params, mode="reference")
    _check_file(r, o)
    assert len(r["peaks"]) > 50


@pytest.mark.parametrize("fs,ds_param,ch", [(192000, 600, 1), (192000, 600, 2), (384000, 1270, 1)])
def test_native_large_decimation(det, fs, ds_param, ch):
    """Native mode beyond ds = 300 (a 192/384 kHz recording with downsample_factor
    raised: bpm_analysis.py:1021-1029 accepts it up to fs/300 - 1) against the oracle."""
    import torch
    params = dict(G.BASE_PARAMS, downsample_factor=ds_param)
    lens = [fs * 12 + 5, fs * 7]
    recs = [O.synth(800 + i, n, fs, ch) for i, n in enumerate(lens)]
    dev = torch.from_numpy(np.concatenate([r.reshape(-1) for r in recs])).to(det.device)
    fo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    res = det.run(dev, fo, fs, params, mode="native", channels=ch, want_y=True)
    torch.cuda.synchronize()
    for h, pcm in zip(res.to_host(), recs):
        o = O.detect(pcm, fs, params, mode="native")
        assert h["sr"] == o["sr"] == fs // ds_param
        scale = np.max(np.abs(o["y"]))
        assert np.max(np.abs(h["y"] - o["y"])) <= 1e-9 * scale
        _check_file(h, o, exact_env=False)


@pytest.mark.parametrize("fs,ch,opt", [(96000, 2, 0), (48000, 2, 0), (44100, 2, 0), (96000, 1, 0), (192000, 1, 0),
                                      (192000, 2, 0), (96000, 2, 128), (44100, 2, 128), (96000, 1, 128)])
def test_native_dma_block_kernel(det, fs, ch, opt):
    """The block kernels for int16 beyond the K <= 160 mono matrix-core path:
    the big-K matrix-core kernel (default for stereo up to ds = 303 and mono up
    to ds = 607: K = channels x (ds + 1) <= 608, the channels' products
    accumulated exactly and halved once) and the LDS-DMA f64 kernel (beyond
    that, e.g. 192 kHz stereo, or BPMX_OPT_NATIVE_DMA) agree with the f64 VALU
    kernels (BPMX_OPT_NATIVE_F64) and give the oracle's indices, on a ragged
    batch whose last recording ends on a partial 16-byte chunk."""
    import torch
    from bpm_analysis_amd import _native as N
    lens = [fs * 9 + 77, fs * 4, fs * 6 + 3]
    recs = [O.synth(960 + i, n, fs, ch) for i, n in enumerate(lens)]
    dev = torch.from_numpy(np.concatenate([r.reshape(-1) for r in recs])).to(det.device)
    fo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    params = dict(G.BASE_PARAMS)
    outs = []
    for o in (opt, N.OPT_NATIVE_F64):
        res = det.run(dev, fo, fs, params, mode="native", channels=ch, want_y=True, options=o)
        torch.cuda.synchronize()
        outs.append(res.to_host())
    for a, b, pcm in zip(outs[0], outs[1], recs):
        # the tile length differs between the kernels (64 vs fewer blocks), so the
        # tile scans round differently: agreement to 1e-12 of the signal's scale
        sy, se = np.max(np.abs(b["y"])), np.max(np.abs(b["env"]))
        assert np.max(np.abs(a["y"] - b["y"])) <= 1e-12 * sy and np.max(np.abs(a["env"] - b["env"])) <= 1e-12 * se
        o = O.detect(pcm, fs, params, mode="native")
        _check_file(a, o, exact_env=False)


def test_run_sharded_single_rank_on_the_gpu(det, tmp_path):
    """shard.run_sharded with the GPU detector (one rank, no process group):
    WAV paths of mixed rates in chunks, native beat stages on host threads;
    raw peaks bit-exact against the oracle, beats and BPM curve equal to the
    Python stages on the same outputs."""
    from scipy.io import wavfile
    from bpm_analysis_amd import beats as B
    from bpm_analysis_amd import DEFAULT_PARAMS
    from bpm_analysis_amd.shard import run_sharded
    params = dict(DEFAULT_PARAMS, save_filtered_wav=False)
    specs = [(44100, 44100 * 40, 1), (48000, 48000 * 25, 2), (44100, 44100 * 33 + 7, 1), (96000, 96000 * 20, 2)]
    paths = []
    for i, (fs, n, ch) in enumerate(specs):
        paths.append(str(tmp_path / f"r{i}.wav"))
        wavfile.write(paths[-1], fs, O.synth(60 + i, n, fs, ch))
    res = run_sharded(paths, params, mode="native", detector=det, host_threads=2, chunk_frames=44100 * 50)
    for (fs, n, ch), path, r in zip(specs, paths, res):
        pcm = wavfile.read(path)[1]
        o = O.detect(pcm, fs, params, mode="native")
        assert _same(r["raw_peaks"], o["peaks"])
        a = B.analyze_recording(o["env"], o["sr"], o["floor"], o["troughs"], o["peaks"], params)
        assert _same(r["final_peaks"], a["final_peaks"])
        np.testing.assert_allclose(r["bpm"], a["final_metrics"]["smoothed_bpm"].values, rtol=1e-12, atol=0)


@pytest.mark.gpu
def test_quantile_kernel_paths(det):
    """qr_select (bpmx_qsel.h, in k_floor_wm's static floor and
    k_quantile_reg): the gather once <= 64 keys share the prefix, long runs of
    tied values (no bin ever that small), a constant envelope (no varying key
    bit), the q = 0 / 1 ends and the (r+1)-th order statistic above the
    gathered keys, through the static noise floor of envelopes without troughs
    (floor = np.quantile(env, q), bpm_analysis.py:1075) and against the
    oracle's troughs and peaks."""
    from bpm_analysis_amd import _native as N
    rng = np.random.default_rng(11)
    n = 18124
    envs = {
        "smooth": np.sort(np.abs(rng.normal(300.0, 80.0, n))),
        "wide_range": np.sort(np.exp(rng.uniform(-12.0, 9.0, n))),
        "ties": np.sort(np.repeat(rng.uniform(1.0, 2.0, 24), (n + 23) // 24)[:n]),
        "constant": np.full(n, 7.25),
        "short": np.sort(rng.uniform(0.0, 1.0, 41)),
    }
    for q in (0.0, 0.2, 0.5, 0.999, 1.0):
        params = dict(G.BASE_PARAMS)
        params["noise_floor_quantile"] = q
        got = det.run_env_host(list(envs.values()), 302, params, N.STAGE_FLOOR)
        for (name, env), r in zip(envs.items(), got):
            want = np.quantile(env, q)
            assert np.all(r["floor"] == want), (name, q, r["floor"][:3], want)
    # the select's (r+1)-th order statistic outside the keys it gathered: r
    # the last key of its 16-bit key prefix on a wide-range envelope, and a
    # step (r + 1 equal values, then a jump) where no bin ever drops to 64 keys
    wide = envs["wide_range"]
    top16 = (wide.view(np.uint64) ^ np.uint64(1 << 63)) >> np.uint64(48)
    edges = np.flatnonzero(top16[1:] != top16[:-1])
    for r in (int(edges[len(edges) // 5]), int(edges[len(edges) // 2]), int(edges[-2])):
        q = (r + 0.5) / (n - 1)
        params = dict(G.BASE_PARAMS)
        params["noise_floor_quantile"] = q
        step = np.where(np.arange(n) <= r, 1.0, 1.0e6)
        got = det.run_env_host([wide, step], 302, params, N.STAGE_FLOOR)
        for env, res in zip((wide, step), got):
            want = np.quantile(env, q)
            assert np.all(res["floor"] == want), (r, q, res["floor"][:3], want)
    # the prominence quantiles (0.1 of the envelope) on bumpy envelopes
    params = dict(G.BASE_PARAMS)
    t = np.arange(n)
    bumpy = [np.abs(np.sin(t / 37.0)) * 100 + np.round(rng.uniform(0, 3, n)),      # many ties
             np.abs(np.sin(t / 23.0)) * np.exp(rng.uniform(-6, 6, n))]
    got = det.run_env_host(bumpy, 302, params, N.STAGE_FLOOR | N.STAGE_PEAKS)
    d = O.derive(302, params)
    for env, r in zip(bumpy, got):
        of, ot, _ = O.noise_floor(env, d, params)
        assert _same(r["troughs"], ot)
        assert _same(r["floor"], of)
        assert _same(r["peaks"], O.raw_peaks(env, of, d, params))


@pytest.mark.gpu
def test_chunked_wavelet_matrix_on_long_recordings(det):
    """Long recordings (n > WM_MMAX) take the pruned wavelet matrix over chunks
    of outputs (default); the sorted-union kernel (BPMX_OPT_ROLLQ_NOPRUNE
    sends them there) and the oracle give the same floor bit for bit.  Cases:
    a late first trough (whole NaN chunks), a ramp, ulp-level floors, a
    recording whose every chunk holds > WM_TRMAX troughs (falls back), and a
    batch mixing short and long recordings."""
    from bpm_analysis_amd import _native as N
    rng = np.random.default_rng(21)
    params = dict(G.BASE_PARAMS)
    d = O.derive(302, params)

    def beat(n, period):
        t = np.arange(n)
        return np.maximum(0.0, np.sin(2 * np.pi * t / period)) ** 8

    n = 96_000                                                   # 5.3 min at 302 Hz
    envs = [
        200 + 80 * np.sin(np.arange(n) / 700.0) + 300 * beat(n, 250) + rng.random(n),
        10.0 + 0.01 * np.arange(n) + 3000 * beat(n, 300) + rng.random(n),
        10.0 + np.spacing(10.0) * rng.integers(0, 5, n) + 300 * beat(n, 250),
        np.abs(np.sin(np.arange(n) / 9.0)) * 100 + rng.random(n),  # > 512 troughs per chunk
        np.concatenate([np.linspace(500.0, 100.0, 40_000), 100 + 300 * beat(n - 40_000, 250) + rng.random(n - 40_000)]),
        300 * beat(12_000, 250) + rng.random(12_000) + 20,          # short, same batch
    ]
    a = det.run_env_host(envs, 302, params, N.STAGE_FLOOR)
    b = det.run_env_host(envs, 302, params, N.STAGE_FLOOR, options=N.OPT_ROLLQ_NOPRUNE)
    for env, ra, rb in zip(envs, a, b):
        assert _same(ra["floor"], rb["floor"])
        assert _same(ra["troughs"], rb["troughs"])
        of, ot, _ = O.noise_floor(env, d, params)
        assert _same(ra["floor"], of)
        assert _same(ra["troughs"], ot)


@pytest.mark.parametrize("mult", [4.0, 2.0, 1.5, 1.0, 0.7])
def test_draft_point_resolves_undecided_troughs(det, mult):
    """Troughs the draft bracket leaves open are decided from the exact draft
    value at the trough (draft_point: one wave per trough), not by computing the
    whole draft floor: bit-identical floors, troughs and peaks to
    BPMX_OPT_DRAFT_FULL and to the oracle, with no recording sent to the full
    draft.  Lower rejection multipliers put many troughs near the threshold
    (vulpine leaves 241 of 1456 undecided at the default 4.0)."""
    from bpm_analysis_amd import _native as N
    params = dict(G.BASE_PARAMS, trough_rejection_multiplier=mult)
    und = raw = 0
    for env, sr in _floor_envelopes():
        a = det.run_env_host([env], sr, params, N.STAGE_FLOOR | N.STAGE_PEAKS, options=N.OPT_STATS)[0]
        st = det.stats()
        und += st["undecided"]
        raw += st["raw_troughs"]
        assert st["full_draft_chunks"] == 0
        b = det.run_env_host([env], sr, params, N.STAGE_FLOOR | N.STAGE_PEAKS, options=N.OPT_DRAFT_FULL)[0]
        for k in ("floor", "troughs", "peaks"):
            assert _same(a[k], b[k]), k
        assert a["flags"] == b["flags"]
        d = O.derive(sr, params)
        of, ot, ofl = O.noise_floor(env, d, params)
        assert _same(a["floor"], of) and _same(a["troughs"], ot) and (a["flags"] & ~O.F_PEAK_TIE) == ofl
    assert raw > 0
    if mult <= 2.0:
        assert und > 0.05 * raw            # the pointwise path is really exercised


def _golden_wav(tmp_path, name):
    from scipy.io import wavfile
    g = G.load(name)
    wav = tmp_path / f"{name}.wav"
    wavfile.write(str(wav), int(g["fs"]), g["pcm"])
    return g, str(wav)


def test_dropin_one_gpu_run_per_file(det, tmp_path, monkeypatch):
    """analyze_wav_file's call sequence (preprocess_audio -> noise floor ->
    _find_raw_peaks twice, bpm_analysis.py:1731-1740, :89) costs one GPU run:
    the floor and peak calls are answered from the run preprocess_audio made,
    bit-exact; a changed envelope or height goes to the GPU again."""
    from bpm_analysis_amd import dropin
    from bpm_analysis_amd.engine import Detector
    g, wav = _golden_wav(tmp_path, "ref_44k_60s_mono")
    params = dict(g["params"], save_filtered_wav=False)
    env, sr = dropin.preprocess_audio(wav, params, str(tmp_path))
    calls = []
    orig = Detector.run_env_host
    monkeypatch.setattr(Detector, "run_env_host", lambda self, *a, **k: calls.append(1) or orig(self, *a, **k))
    floor, troughs = dropin._calculate_dynamic_noise_floor(env, sr, params)
    p1 = dropin.find_raw_peaks(env, sr, params, floor.values)
    p2 = dropin.find_raw_peaks(env, sr, dict(params, pairing_confidence_threshold=0.75), floor.values)
    assert calls == []
    assert _same(env, g["env"]) and _same(floor.values, g["floor"]) and _same(troughs, g["troughs"])
    assert _same(p1, g["peaks"]) and _same(p2, g["peaks"])
    # a different height or envelope is computed on the GPU
    p3 = dropin.find_raw_peaks(env, sr, params, floor.values * 1.5)
    env2 = env.copy()
    env2[100] += 1.0
    dropin._calculate_dynamic_noise_floor(env2, sr, params)
    assert len(calls) == 2
    want = O.raw_peaks(g["env"], g["floor"] * 1.5, O.derive(sr, params), params)
    assert _same(p3, want)


def test_dropin_first_detector_on_a_daemon_thread(tmp_path):
    """gui.py:181-187 imports and runs analyze_wav_file on a daemon thread, so the
    first GPU context is created there: the patched reference entry point runs
    there bit-exact, and the main thread never touches the GPU (own process)."""
    import subprocess
    import sys
    g, wav = _golden_wav(tmp_path, "ref_44k_60s_mono")
    np.savez(str(tmp_path / "want.npz"), env=g["env"], floor=g["floor"], troughs=g["troughs"], peaks=g["peaks"])
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import sys, threading
import numpy as np
sys.path.insert(0, {repo!r})
from tests.test_gpu_parity import _stand_in_reference
from tests import goldens as G
from bpm_analysis_amd import dropin, engine
mod = _stand_in_reference()
dropin.patch_reference(mod)
params = dict(G.load("ref_44k_60s_mono")["params"], save_filtered_wav=False)
res = {{}}
def work():
    try:
        res["out"] = mod.analyze_wav_file({wav!r}, params, None, {wav!r}, {str(tmp_path)!r})
        res["dets"] = len(engine._default.dets)
    except BaseException as exc:
        res["err"] = repr(exc)
t = threading.Thread(target=work, daemon=True)
t.start()
t.join(300)
assert "err" not in res, res.get("err")
assert res["dets"] == 1 and len(engine._default.dets) == 0
w = np.load({str(tmp_path / "want.npz")!r})
env, floor, troughs, peaks = res["out"]
for a, b in ((env, w["env"]), (floor.values, w["floor"]), (troughs, w["troughs"]), (peaks, w["peaks"])):
    assert np.array_equal(np.asarray(a), b, equal_nan=True)
print("daemon-thread ok")
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "daemon-thread ok" in r.stdout, r.stderr[-3000:]


def test_dropin_two_threads_at_once(det, tmp_path):
    """Two threads run the patched reference entry point at the same time on
    different files (Gradio may call concurrently; each thread gets its own
    context and stream), several times each: every result bit-exact."""
    import threading
    from bpm_analysis_amd import dropin
    mod = _stand_in_reference()
    dropin.patch_reference(mod)
    cases = [_golden_wav(tmp_path, n) for n in ("ref_44k_60s_mono", "ref_48k_20s_mono")]
    bar = threading.Barrier(2)
    errs = []

    def work(g, wav):
        try:
            params = dict(g["params"], save_filtered_wav=False)
            for _ in range(4):
                bar.wait(timeout=120)
                env, floor, troughs, peaks = mod.analyze_wav_file(wav, params, None, wav, str(tmp_path))
                assert _same(env, g["env"]) and _same(floor.values, g["floor"])
                assert _same(troughs, g["troughs"]) and _same(peaks, g["peaks"])
                # and the batched entry on the other file's rate group at the same time
                r = dropin.analyze_batch([g["pcm"]], int(g["fs"]), params)[0]
                assert _same(r["peaks"], g["peaks"])
        except BaseException as exc:          # noqa: BLE001 - reported below
            errs.append(repr(exc))
            bar.abort()

    ts = [threading.Thread(target=work, args=c) for c in cases]
    for t in ts:
        t.start()
    for t in ts:
        t.join(600)
    assert not errs, errs


def test_config_c5_shard_of_eight(det):
    """BASELINE config C5 at its stated recording shape: a shard of 8 ragged
    U[10, 30] min 96 kHz stereo int16 recordings (bench.c5_lengths, the
    bench's own seeds) in one device batch, longest first, native mode; every
    recording checked against the oracle (indices and flags exact, envelope
    and floor within 1e-9 of scale; ~30 s of oracle time on 8 threads)."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    import bench
    fs, ch = 96000, 2
    lengths = bench.c5_lengths(8, fs)
    order = np.argsort(-lengths, kind="stable")
    lens = lengths[order]
    fo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    seeds = [100_000 + int(i) for i in order]
    pcm = det.synth(fo, fs, ch, seeds=seeds)
    params = dict(G.BASE_PARAMS)
    res = det.run(pcm, fo, fs, params, mode="native", channels=ch)
    torch.cuda.synchronize()
    host = res.to_host()
    del pcm
    check = list(range(len(lens)))
    with ThreadPoolExecutor(8) as ex:
        outs = list(ex.map(lambda k: O.detect(O.synth(seeds[k], int(lens[k]), fs, ch), fs, params, mode="native"),
                           check))
    for k, o in zip(check, outs):
        _check_file(host[k], o, exact_env=False)
    for h, n in zip(host, lens):
        assert len(h["env"]) == -(-int(n) // 300) and len(h["peaks"]) > 10 * (n // fs // 60)


def test_longfft_hilbert_matches_bluestein_and_oracle(det):
    """Long recordings' Hilbert transform by exact-length four-step DFTs
    (k_longfft.hip) against the rocFFT Bluestein path (BPMX_OPT_HILBERT_BLUESTEIN)
    and the oracle: lengths with a large prime row (s = 601, 1201: Bluestein
    rows inside the workgroup; s = 1742 = 2 x 13 x 67: 4160-point rows), a
    smooth one (s = 1800) and an odd Nd (unpacked transform), 96 kHz mono."""
    import torch
    from bpm_analysis_amd import _native as N
    fs = 96000
    lens = [96000 * 601, 96000 * 1742 // 2, 300 * 95_993, 96000 * 1200 // 2]
    fo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    pcm = det.synth(fo, fs, 1, seed0=321)
    params = dict(G.BASE_PARAMS)
    a = det.run(pcm, fo, fs, params, mode="native").to_host()
    b = det.run(pcm, fo, fs, params, mode="native", options=N.OPT_HILBERT_BLUESTEIN).to_host()
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        scale = np.max(np.abs(y["env"]))
        assert np.max(np.abs(x["env"] - y["env"])) <= 1e-12 * scale
        assert _same(x["peaks"], y["peaks"]) and _same(x["troughs"], y["troughs"])
    o = O.detect(O.synth(321 + 2, lens[2], fs, 1), fs, params, mode="native")     # odd Nd = 95,993 = 59 x 1627
    assert len(a[2]["env"]) == 95_993
    _check_file(a[2], o, exact_env=False)


def test_reference_split_passes_bit_identical(det):
    """Reference mode runs the forward pass in row chunks beside the gather of
    the next chunks (k_ref_fwd), and the Kahan pass in row chunks beside the
    finished chunks' means (k_ref_kahan, k_ref_env_mean on a side stream).
    Those splits equal the single-kernel passes (BPMX_OPT_REF_NOSPLIT) and the
    fully serial rolling mean (BPMX_OPT_REF_SERIAL_MEAN) bit for bit, on a
    ragged f32 batch over two waves of recordings, one of them holding a NaN
    (its wave leaves chain mode and keeps the in-pass means), y included; and
    the clean recordings equal the oracle."""
    from bpm_analysis_amd import _native as N
    fs = 44100
    rng = np.random.default_rng(17)
    lens = [int(fs * s) for s in rng.uniform(14.0, 24.0, 70)]
    recs = [O.synth(400 + f, n, fs, 1).astype(np.float32) for f, n in enumerate(lens)]
    recs[3][len(recs[3]) // 2] = np.nan                     # wave 0 leaves chain mode
    params = dict(G.BASE_PARAMS)
    a = det.run_host(recs, fs, params, mode="reference", want_y=True)
    b = det.run_host(recs, fs, params, mode="reference", want_y=True, options=N.OPT_REF_NOSPLIT)
    c = det.run_host(recs, fs, params, mode="reference", want_y=True, options=N.OPT_REF_SERIAL_MEAN)
    for x, y, z in zip(a, b, c):
        for k in ("env", "y", "floor", "troughs", "peaks"):
            assert _same(x[k], y[k]) and _same(x[k], z[k]), k
        assert x["flags"] == y["flags"] == z["flags"]
    for f in (0, 1, 40, 69):
        o = O.detect(recs[f], fs, params, mode="reference")
        assert _same(a[f]["env"], o["env"]) and _same(a[f]["peaks"], o["peaks"]), f


@pytest.mark.parametrize("mode", ["native", "reference"])
def test_pipelined_run_identical(mode):
    """bpmx_set_pipeline (envelope of chunk k beside the detection of chunk
    k - 1, include/bpmx.h) gives the unpipelined run's outputs: troughs, peaks,
    counts, raw-trough counts, flags and the path counters (BPMX_OPT_STATS)
    identical, env, y and floor bit for bit in both modes (a chunk's PCM base
    that is not 16-byte aligned is realigned by the library), on a ragged
    batch with a too-short recording, with and without CU masks."""
    import torch
    from bpm_analysis_amd import _native as N
    from bpm_analysis_amd.engine import Detector
    fs = 44100
    lens = [fs * 20, fs * 7 + 13, 146 * 15, fs * 31, fs * 12 + 5, fs * 9, fs * 25, fs * 3 + 77, fs * 16]
    seeds = [300 + i for i in range(len(lens))]
    fo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    params = dict(G.BASE_PARAMS, trough_rejection_multiplier=1.5)   # some undecided troughs: draft_point runs
    ref_det = Detector(0)
    pcm = ref_det.synth(fo, fs, 1, seeds=seeds)

    def run(det):
        r = det.run(pcm, fo, fs, params, mode=mode, want_y=True, options=N.OPT_STATS)
        torch.cuda.synchronize()
        return r.to_host(), det.stats(), r.n_raw_troughs.cpu().numpy().copy()

    base, bst, braw = run(ref_det)
    assert base[2]["flags"] & N.F_TOO_SHORT
    for shape in ((2, 0, 0), (3, 0, 0), (2, 192, 64)):
        det = Detector(0)
        det.set_pipeline(*shape)
        got, gst, graw = run(det)
        assert gst == bst, shape
        assert np.array_equal(graw, braw), shape
        for a, b in zip(got, base):
            assert a["flags"] == b["flags"]
            assert a["n_raw_troughs"] == b["n_raw_troughs"]
            for k in ("env", "y", "floor", "troughs", "peaks"):
                if b["flags"] & N.F_TOO_SHORT:           # no outputs (include/bpmx.h): to_host gives empty slices
                    assert a[k] is None or a[k].size == 0, k
                    assert b[k] is None or b[k].size == 0, k
                    continue
                if a[k] is None or b[k] is None:
                    assert a[k] is None and b[k] is None
                else:
                    assert _same(a[k], b[k]), (shape, k)
        det.close()
    ref_det.close()


@pytest.mark.parametrize("mode", ["reference", "native"])
def test_batch_pipeline_identical(det, mode):
    """engine.BatchPipeline (batch k + 1's envelope on one context and stream
    beside batch k's detection on another) gives, for every batch of a
    stream, the single all-stage run's outputs: env and floor bit for bit,
    troughs, peaks and flags identical; four different ragged batches through
    two result sets, so the result-set reuse and the cross-stream events are
    exercised."""
    from bpm_analysis_amd.engine import BatchPipeline
    fs = 44100
    lens = [fs * 20, fs * 7 + 13, fs * 31, fs * 12 + 5, fs * 16]
    fo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    params = dict(G.BASE_PARAMS)
    pcms = [det.synth(fo, fs, 1, seed0=900 + 10 * b) for b in range(4)]
    want = []
    for p in pcms:
        r = det.run(p, fo, fs, params, mode=mode)
        det.resolve_ties(r, params)
        want.append(r.to_host())
    pipe = BatchPipeline(0, fo, fs, params, mode=mode)
    got = []
    for b, p in enumerate(pcms):
        got.append(pipe.submit(p))
        if b % 2 == 1:                   # read back before the set is reused
            pipe.finish()
            got = got[:-2] + [x.to_host() for x in got[-2:]]
    pipe.finish()
    pipe.close()
    assert len(got) == 4
    for g, w in zip(got, want):
        for a, b in zip(g, w):
            assert a["flags"] == b["flags"]
            for k in ("env", "floor", "troughs", "peaks"):
                assert _same(a[k], b[k]), k


@pytest.mark.gpu
def test_native_fused_yd_identical(det):
    """k_hilbert_env making yd of the full decimation tiles itself (HilbArgs::fy:
    no y output requested, every recording on the fused Hilbert plan) gives the
    same env, floor, troughs, peaks and flags bit for bit as k_native_yd
    followed by the kernel (y requested), on a ragged batch with odd decimated
    offsets, partial last tiles and a recording shorter than one tile, and on
    a ragged batch mixing fused (even Nd) and unfused (odd Nd) recordings."""
    fs = 44100                                       # ds = 146: Nd = ceil(n / 146), 62-block tiles
    # even Nd for every recording (an odd Nd takes another transform, and the
    # whole batch the unfused path): 3322 / 1800 (odd decimated offsets after
    # the first) / 58 (shorter than one tile) / 18124 samples
    lens = [146 * 3322 - 5, 146 * 1800, 146 * 58 - 1, 146 * 18124 - 77]
    fo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    params = dict(G.BASE_PARAMS)
    pcm = det.synth(fo, fs, 1, seed0=314)
    det.profile_only("")
    det.profile(True)
    fused = det.run(pcm, fo, fs, params, mode="native").to_host()
    det.profile(False)
    assert "k_native_yd" not in det.profile_read()       # yd made inside k_hilbert_env
    det.profile(True)
    plain = det.run(pcm, fo, fs, params, mode="native", want_y=True).to_host()
    det.profile(False)
    assert "k_native_yd" in det.profile_read()
    assert [r["env"].size for r in plain] == [3322, 1800, 58, 18124]
    for a, b in zip(fused, plain):
        for k in ("env", "floor", "troughs", "peaks"):
            assert _same(a[k], b[k]), k
        assert a["flags"] == b["flags"]
    # a ragged batch mixing odd Nd (another transform, yd from k_native_yd,
    # which skips the fused recordings' tiles) with even Nd (fused)
    lens2 = [146 * 3321 - 9, 146 * 1800, 146 * 2401, 146 * 58 - 1, 146 * 5000 - 3]
    fo2 = np.concatenate([[0], np.cumsum(lens2)]).astype(np.int64)
    pcm2 = det.synth(fo2, fs, 1, seed0=2718)
    det.profile(True)
    mixed = det.run(pcm2, fo2, fs, params, mode="native").to_host()
    det.profile(False)
    assert "k_native_yd" in det.profile_read()
    plain2 = det.run(pcm2, fo2, fs, params, mode="native", want_y=True).to_host()
    assert [r["env"].size % 2 for r in plain2] == [1, 0, 1, 0, 0]
    for a, b in zip(mixed, plain2):
        for k in ("env", "floor", "troughs", "peaks"):
            assert _same(a[k], b[k]), k
        assert a["flags"] == b["flags"]


def test_native_envelope_independent_of_placement(det):
    """A recording's native envelope (and everything after it) is bit-identical
    wherever its PCM lies: a batch started 1..8 frames into an aligned buffer
    (the library realigns the base, bpmx_api.hip run_impl), and the recording
    at different positions of a ragged batch."""
    import torch
    from bpm_analysis_amd import _native as N
    fs = 44100
    lens = [fs * 11 + 3, fs * 6 + 1, fs * 9]
    fo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    params = dict(G.BASE_PARAMS)
    big = det.synth(np.array([0, int(fo[-1]) + 16], dtype=np.int64), fs, 1, seed0=77)
    ref = det.run(big, fo, fs, params, mode="native", want_y=True).to_host()
    for sh in (1, 2, 3, 5, 8):
        view = big[sh:]                                    # base 2*sh bytes past the allocation's
        got = det.run(view, fo, fs, params, mode="native", want_y=True).to_host()
        want = det.run(torch.clone(view), fo, fs, params, mode="native", want_y=True).to_host()
        for a, b in zip(got, want):
            for k in ("env", "y", "floor", "troughs", "peaks"):
                assert _same(a[k], b[k]), (sh, k)
            assert a["flags"] == b["flags"]
    # recording 1 of `ref` alone, and behind an odd-length prefix recording
    r1 = big[int(fo[1]):int(fo[2])]
    alone = det.run(torch.clone(r1), np.array([0, lens[1]]), fs, params, mode="native", want_y=True).to_host()[0]
    pre = torch.cat([big[:fs * 2 + 7], r1])
    behind = det.run(pre, np.array([0, fs * 2 + 7, fs * 2 + 7 + lens[1]]), fs, params, mode="native",
                     want_y=True).to_host()[1]
    for k in ("env", "y", "floor", "troughs", "peaks"):
        assert _same(alone[k], ref[1][k]), k
        assert _same(behind[k], ref[1][k]), k
