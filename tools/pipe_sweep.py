"""Sweep bpmx_set_pipeline shapes on the bench's metric batch (tools only).

    python tools/pipe_sweep.py [--mode native] [--steps 10] [--shapes 4,192,0 4,192,64 ...]

For each (chunks, env_cus, det_cus) shape: ms per step over `steps` timed
steps (after two warmups) and whether every output array equals the
unpipelined run's, bit for bit.  One JSON line per shape, then a summary.
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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--files", type=int, default=1024)
    ap.add_argument("--options", type=int, default=0)
    ap.add_argument("--mult", type=float, default=0.0, help="trough_rejection_multiplier override (0: default)")
    ap.add_argument("--shapes", nargs="*", default=["0,0,0", "2,0,0", "4,0,0", "4,192,0", "4,160,0", "4,192,64",
                                                    "8,192,0", "8,192,64", "4,128,128", "0,0,0"])
    a = ap.parse_args()
    import torch
    from bpm_analysis_amd import DEFAULT_PARAMS
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
    keys = ("env", "floor", "troughs", "peaks", "n_troughs", "n_peaks", "flags")
    ref = None
    rows = []
    for sh in a.shapes:
        parts = [int(x) for x in sh.split(",")]
        k, ec, dc = parts[:3]
        if len(parts) > 3 and parts[3] > 0:           # persistent grid of the block kernel (BPMX_NM_GRID)
            os.environ["BPMX_NM_GRID"] = str(parts[3])
        else:
            os.environ.pop("BPMX_NM_GRID", None)
        det.set_pipeline(k, ec, dc)
        for _ in range(2):
            det.run(pcm, fo, fs, params, mode=a.mode, out=out, d=d, options=a.options)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            det.run(pcm, fo, fs, params, mode=a.mode, out=out, d=d, options=a.options)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        host = out.to_host()
        cur = {kk: [h[kk] if kk in h else None for h in host] for kk in ("env", "floor", "troughs", "peaks", "flags")}
        if ref is None:
            ref = cur
        same = all(np.array_equal(x, y, equal_nan=True) if isinstance(x, np.ndarray) else x == y
                   for kk in cur for x, y in zip(cur[kk], ref[kk]))
        row = {"chunks": k, "env_cus": ec, "det_cus": dc, "nm_grid": parts[3] if len(parts) > 3 else 0,
               "ms_per_step": round(ms, 4), "identical": bool(same)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    det.set_pipeline(0, 0, 0)
    print(json.dumps({"summary": rows}))


if __name__ == "__main__":
    main()
