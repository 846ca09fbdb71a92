"""Diagnostic: where does a recording's native envelope depend on the batch?
Compares per recording (env, y) of the full batch against sub-batch runs
(aligned clones and misaligned views) and a pipelined run."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from bpm_analysis_amd.engine import Detector
from tests import goldens as G

fs = 44100
lens = [fs * 20, fs * 7 + 13, 146 * 15, fs * 31, fs * 12 + 5, fs * 9, fs * 25, fs * 3 + 77, fs * 16]
seeds = [300 + i for i in range(len(lens))]
fo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
params = dict(G.BASE_PARAMS, trough_rejection_multiplier=1.5)
det = Detector(0)
pcm = det.synth(fo, fs, 1, seeds=seeds)
base = det.run(pcm, fo, fs, params, mode="native", want_y=True, stages=1).to_host()


def cmp(tag, got, idx):
    for r, f in zip(got, idx):
        b = base[f]
        if b["env"] is None or len(b["env"]) == 0:
            continue
        de = np.nanmax(np.abs(r["env"] - b["env"])) if r["env"].size else 0.0
        dy = np.nanmax(np.abs(r["y"] - b["y"])) if r["y"].size else 0.0
        print(tag, f, "env", de, "y", dy, flush=True)


for f0, f1 in [(0, 3), (3, 6), (6, 9), (1, 2), (3, 4)]:
    sub = fo[f0:f1 + 1] - fo[f0]
    view = pcm[int(fo[f0]):int(fo[f1])]
    cmp(f"view[{f0}:{f1}] mis={(int(fo[f0]) * 2) % 16}", det.run(view, sub, fs, params, mode="native", want_y=True,
                                                             stages=1).to_host(), range(f0, f1))
    cmp(f"clone[{f0}:{f1}]", det.run(torch.clone(view), sub, fs, params, mode="native", want_y=True,
                                     stages=1).to_host(), range(f0, f1))
d2 = Detector(0)
d2.set_pipeline(2, 0, 0)
cmp("pipe2", d2.run(pcm, fo, fs, params, mode="native", want_y=True).to_host(), range(len(lens)))
