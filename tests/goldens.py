"""Loading helpers for tests/golden/*.npz (data-only fixtures)."""
import glob
import hashlib
import json
import os

import numpy as np

from tests.golden import inputs as I

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

BASE_PARAMS = {"downsample_factor": 300, "save_filtered_wav": False, "min_peak_distance_sec": 0.05,
               "peak_prominence_quantile": 0.1, "trough_prominence_quantile": 0.1,
               "noise_floor_quantile": 0.20, "noise_window_sec": 10, "trough_rejection_multiplier": 4.0}


def names(kind=None, mode=None, prefix=None):
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))):
        name = os.path.splitext(os.path.basename(p))[0]
        if prefix and not name.startswith(prefix):
            continue
        with np.load(p, allow_pickle=False) as z:
            if kind and str(z["kind"]) != kind:
                continue
            if mode and str(z["mode"]) != mode:
                continue
        out.append(name)
    return out


def env_derived(g):
    """oracle.Derived for an env-level fixture (only sr / distance / noise window matter)."""
    from oracle import oracle as O
    d = O.derive(302 * 146, dict(g["params"]))
    sr = int(g["sr"])
    d.sr = sr
    d.distance = int(g["params"]["min_peak_distance_sec"] * sr)
    d.noise_window = int(g["params"]["noise_window_sec"] * sr)
    return d


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    p = dict(BASE_PARAMS)
    p.update(json.loads(str(g["params"])))
    g["params"] = p
    if str(g["kind"]) == "pcm":
        spec = json.loads(str(g["spec"]))
        pcm, fs = I.make_input(spec)
        assert hashlib.sha256(pcm.tobytes()).hexdigest() == str(g["pcm_sha256"]), name
        g["pcm"] = pcm
    return g
