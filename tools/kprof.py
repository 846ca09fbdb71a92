"""Per-kernel HIP-event profile of one configuration of the metric batch (tools only).

    python tools/kprof.py [--mode native] [--mult 1.0] [--options 8] [--steps 5]

Prints ms per step of the step and of every kernel label (bpmx_profile), and
the path counters (bpmx_stats) of the last step.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="native")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--files", type=int, default=1024)
    ap.add_argument("--options", type=int, default=0)
    ap.add_argument("--mult", type=float, default=0.0)
    a = ap.parse_args()
    import torch
    from bpm_analysis_amd import DEFAULT_PARAMS, _native as N
    from bpm_analysis_amd.design import design
    from bpm_analysis_amd.engine import Detector
    det = Detector(0)
    params = dict(DEFAULT_PARAMS, save_filtered_wav=False)
    if a.mult > 0:
        params["trough_rejection_multiplier"] = a.mult
    fs, F, n = 44100, a.files, 44100 * 60
    d = design(fs, params, log=False)
    fo = np.arange(F + 1, dtype=np.int64) * n
    pcm = det.synth(fo, fs, 1, seed0=0)
    out = det.alloc(fo, d.ds, d.sr)
    for _ in range(2):
        det.run(pcm, fo, fs, params, mode=a.mode, out=out, d=d, options=a.options)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        det.run(pcm, fo, fs, params, mode=a.mode, out=out, d=d, options=a.options)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    det.profile(True)
    for _ in range(a.steps):
        det.run(pcm, fo, fs, params, mode=a.mode, out=out, d=d, options=a.options | N.OPT_STATS)
    torch.cuda.synchronize()
    det.profile(False)
    prof = det.profile_read()
    rows = {k: round(t / a.steps, 4) for k, (c, t) in sorted(prof.items(), key=lambda kv: -kv[1][1])}
    print(json.dumps({"mode": a.mode, "mult": a.mult, "options": a.options, "ms_per_step": round(ms, 4),
                      "kernel_ms_per_step": rows, "stats": det.stats()}))


if __name__ == "__main__":
    main()
