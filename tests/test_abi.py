"""C ABI: the library loads, exports every symbol include/bpmx.h declares, and
its host-only entry points behave (no GPU needed)."""
import ctypes
import os
import re

import numpy as np
import pytest

from bpm_analysis_amd import _native as N
from oracle import oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(REPO, "include", "bpmx.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|int64_t|const char \*)\s*\**\s*(bpmx_\w+)\s*\(", txt, re.M)))


def test_header_matches_binding_list():
    assert _declared() == sorted(N.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = N.load()
    for name in _declared():
        assert hasattr(L, name), name
    assert L.bpmx_abi_version() == N.ABI_VERSION


def test_struct_layouts():
    # offsets the C side relies on (bpmx_params: 12 int32, then doubles)
    assert N.Params.trough_prom_q.offset == 48
    assert N.Params.ba_b.offset == 48 + 5 * 8
    assert ctypes.sizeof(N.Params) == 48 + 5 * 8 + (5 + 5 + 4 + 12 + 4) * 8
    assert ctypes.sizeof(N.Batch) == 24
    assert ctypes.sizeof(N.Out) == 9 * 8


@pytest.mark.parametrize("n,ds,want", [(2646000, 146, 18124), (146 * 15, 146, 15), (1, 300, 1), (0, 5, 0)])
def test_decimated_length(n, ds, want):
    assert N.load().bpmx_decimated_length(n, ds) == want


@pytest.mark.parametrize("seed,fs,ch", [(0, 44100, 1), (3, 96000, 2), (9, 22050, 1)])
def test_synth_host_matches_oracle_generator(seed, fs, ch):
    n = fs * 2 + 17
    out = np.empty(n * ch, dtype=np.int16)
    N.load().bpmx_synth_host(seed, n, fs, ch, out.ctypes.data)
    assert np.array_equal(out, O.synth(seed, n, fs, ch).reshape(-1))


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    c = ctypes.c_void_p()
    rc = N.load().bpmx_create(0, ctypes.byref(c))
    assert rc == N.E_NODEV
    assert b"device" in N.load().bpmx_last_error()


def test_reference_side_stub_matches_package():
    """tools/ctypes_stub.py declares the same C structs and
    derives byte-identical bpmx_params to the package's host code."""
    import ctypes
    import importlib.util
    import os

    from bpm_analysis_amd import DEFAULT_PARAMS
    from bpm_analysis_amd import _native as N
    from bpm_analysis_amd.design import design, make_params
    spec = importlib.util.spec_from_file_location("ctypes_stub", os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "ctypes_stub.py"))
    stub = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(stub)
    for a, b in [(stub.Params, N.Params), (stub.Batch, N.Batch), (stub.Out, N.Out)]:
        assert ctypes.sizeof(a) == ctypes.sizeof(b)
        assert [f[0] for f in a._fields_] == [f[0] for f in b._fields_]
    for fs in (44100, 48000, 96000, 22050):
        p1 = stub.make_params(fs, DEFAULT_PARAMS)
        p2 = make_params(design(fs, DEFAULT_PARAMS, log=False), DEFAULT_PARAMS, 0, 7, 1, 1)
        assert bytes(p1) == bytes(p2)


def test_patch_reference_rebinds_the_hot_path_names():
    """patch_reference points a reference module's three hot-path names at the
    drop-ins (what runs behind them is the GPU test's business)."""
    import types

    from bpm_analysis_amd import dropin

    class PeakClassifier:
        def _find_raw_peaks(self, height_threshold):
            raise AssertionError("unpatched")

    mod = types.ModuleType("stand_in")
    mod.preprocess_audio = mod._calculate_dynamic_noise_floor = None
    mod.PeakClassifier = PeakClassifier
    dropin.patch_reference(mod)
    assert mod.preprocess_audio is dropin.preprocess_audio
    assert mod._calculate_dynamic_noise_floor is dropin._calculate_dynamic_noise_floor
    assert PeakClassifier._find_raw_peaks.__name__ == "_find_raw_peaks"
    assert PeakClassifier._find_raw_peaks is not None and "unpatched" not in str(PeakClassifier._find_raw_peaks)


def test_arg_errors_are_value_errors():
    """BPMX_E_ARG surfaces as ValueError (the reference's exception type)."""
    assert issubclass(N.BpmxArgError, ValueError) and issubclass(N.BpmxArgError, N.BpmxError)
    from bpm_analysis_amd import dropin
    e = dropin._window_error({"noise_window_sec": 0.005}, 302)
    assert isinstance(e, ValueError) and str(e) == "min_periods 3 must be <= window 1"
    import pandas as pd
    with pytest.raises(ValueError, match=str(e)):
        pd.Series(np.arange(10.0)).rolling(window=1, min_periods=3, center=True)
    with pytest.raises(ValueError, match=str(dropin._window_error({"noise_window_sec": -1.0}, 302))):
        pd.Series(np.arange(10.0)).rolling(window=-302, min_periods=3, center=True)
    from scipy.signal import find_peaks
    with pytest.raises(ValueError, match=dropin.DISTANCE_MSG):
        find_peaks(np.arange(10.0), distance=0)
