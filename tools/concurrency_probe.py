"""Probe: the metric batch as one bpmx_run on one stream vs split across
K contexts on K streams (each context owns its scratch; runs overlap on the
GPU).  Prints ms per step for K = 1, 2, 4.  Study tool, not product code."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpm_analysis_amd import DEFAULT_PARAMS  # noqa: E402
from bpm_analysis_amd.design import design  # noqa: E402
from bpm_analysis_amd.engine import Detector  # noqa: E402

F, fs, n, steps = 1024, 44100, 44100 * 60, 10
params = dict(DEFAULT_PARAMS)
params["save_filtered_wav"] = False
d = design(fs, params, log=False)
for K in (1, 2, 4):
    dets = [Detector(0) for _ in range(K)]
    streams = [torch.cuda.Stream() for _ in range(K)]
    per = F // K
    fo = np.arange(per + 1, dtype=np.int64) * n
    pcms, outs = [], []
    for k in range(K):
        with torch.cuda.stream(streams[k]):
            pcms.append(dets[k].synth(fo, fs, 1, seed0=k * per))
            outs.append(dets[k].alloc(fo, d.ds, d.sr))
    torch.cuda.synchronize()

    def step():
        for k in range(K):
            with torch.cuda.stream(streams[k]):
                dets[k].run(pcms[k], fo, fs, params, mode="native", out=outs[k], d=d)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    npk = sum(int(o.n_peaks.sum()) for o in outs)
    print(f"K={K}: {ms:.3f} ms/step, {F * n / ms / 1e6:.1f} G samples/s, peaks {npk}", flush=True)
    for x in dets:
        x.close()
