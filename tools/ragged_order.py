"""Ragged batch, device-resident: recordings in ascending length (the longest
dispatched last) against longest first (shard.longest_first).  Prints one JSON
line; DESIGN.md §6 quotes it.

    python tools/ragged_order.py [--files 128] [--steps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=128)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--fs", type=int, default=44100)
    ap.add_argument("--mode", default="native")
    ap.add_argument("--channels", type=int, default=1)
    ap.add_argument("--min-s", type=int, default=60)
    ap.add_argument("--max-s", type=int, default=600)
    args = ap.parse_args()
    import torch
    from bpm_analysis_amd import DEFAULT_PARAMS
    from bpm_analysis_amd.design import design
    from bpm_analysis_amd.engine import Detector
    from bpm_analysis_amd.shard import longest_first
    params = dict(DEFAULT_PARAMS, save_filtered_wav=False)
    fs = args.fs
    rng = np.random.default_rng(3)
    lens = (rng.integers(args.min_s, args.max_s + 1, size=args.files) * fs).astype(np.int64)
    d = design(fs, params, log=False)
    det = Detector(0)
    out = {}
    for name, order in (("ascending", np.argsort(lens, kind="stable")), ("longest_first", longest_first(lens))):
        ln = lens[order]
        fo = np.concatenate([[0], np.cumsum(ln)]).astype(np.int64)
        pcm = det.synth(fo, fs, args.channels, seed0=100)
        res = det.alloc(fo, d.ds, d.sr)
        for _ in range(2):
            det.run(pcm, fo, fs, params, mode=args.mode, out=res, d=d, channels=args.channels)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            det.run(pcm, fo, fs, params, mode=args.mode, out=res, d=d, channels=args.channels)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        det.profile(True)
        det.run(pcm, fo, fs, params, mode=args.mode, out=res, d=d, channels=args.channels)
        torch.cuda.synchronize()
        det.profile(False)
        kern = {k: round(v[1], 3) for k, v in sorted(det.profile_read().items(), key=lambda kv: -kv[1][1])}
        out[name] = {"ms_per_step": dt * 1e3, "audio_samples_per_s": float(lens.sum()) * args.channels / dt,
                     "peaks": int(res.n_peaks.sum()), "kernel_ms": kern}
        del pcm, res
        torch.cuda.empty_cache()
    out.update(files=args.files, total_samples=int(lens.sum()), fs=fs, mode=args.mode,
               speedup=out["ascending"]["ms_per_step"] / out["longest_first"]["ms_per_step"], channels=args.channels)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
