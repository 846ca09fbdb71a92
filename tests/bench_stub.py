"""TESTS ONLY: an oracle-backed stand-in for engine.Detector, so that
`bench.py --gpus N --cpu-stub` runs its multi-rank path (launcher, rank setup,
max-over-ranks timing, parity sample, result gather) on gloo CPU ranks.

The oracle is the checker, never the product: this module lives under tests/
and bench.py loads it only with --cpu-stub, whose line is labelled
"cpu-stub (tests only; not a measurement)".
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from oracle import oracle as O  # noqa: E402


class StubResult:
    def __init__(self, fo, ds, sr):
        lens = np.diff(fo)
        self.sr, self.ds = sr, ds
        self.frame_offsets = fo
        self.doff = np.concatenate([[0], np.cumsum(-(-lens // ds))]).astype(np.int64)
        F = len(fo) - 1
        self.files = [None] * F
        self.n_peaks = torch.zeros(F, dtype=torch.int32)

    def to_host(self):
        return [dict(f) for f in self.files]


class StubDetector:
    device = torch.device("cpu")

    def __init__(self, device: int = 0):
        self.index = device

    def close(self):
        pass

    def synth(self, frame_offsets, fs, channels=1, seed0=0, seeds=None):
        fo = np.asarray(frame_offsets, dtype=np.int64)
        seeds = [seed0 + f for f in range(len(fo) - 1)] if seeds is None else list(seeds)
        return [O.synth(int(s), int(fo[f + 1] - fo[f]), fs, channels) for f, s in enumerate(seeds)]

    def alloc(self, frame_offsets, ds, sr, **_):
        return StubResult(np.asarray(frame_offsets, dtype=np.int64), ds, sr)

    def run(self, pcm, frame_offsets, fs, params, mode="reference", channels=1, out=None, d=None, options=0, **_):
        for f, rec in enumerate(pcm):
            o = O.detect(rec, fs, params, mode=mode)
            out.files[f] = {"sr": o["sr"], "env": o["env"], "floor": o["floor"], "troughs": o["troughs"],
                            "peaks": o["peaks"], "flags": int(o["flags"]), "n_raw_troughs": 0, "y": None}
            out.n_peaks[f] = len(o["peaks"])
        return out

    def tie_check_start(self, out):
        return out

    def tie_check_finish(self, handle, out, params, stages=None, options=0):
        return 0                  # the oracle decides in its stable order; nothing to re-run

    def profile(self, on):
        pass

    def profile_only(self, label=""):
        pass

    def profile_read(self):
        return {}
