"""Probe: engine.BatchPipeline in reference mode under stream configurations
(detection stream's free CUs, envelope stream priority), ms per batch over 10
batches against the unpipelined step.  Study tool, not product code."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpm_analysis_amd import DEFAULT_PARAMS  # noqa: E402
from bpm_analysis_amd.design import design  # noqa: E402
from bpm_analysis_amd.engine import BatchPipeline, Detector  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "reference"
F, fs, n, steps = 1024, 44100, 44100 * 60, 10
params = dict(DEFAULT_PARAMS, save_filtered_wav=False)
d = design(fs, params, log=False)
fo = np.arange(F + 1, dtype=np.int64) * n
det = Detector(0)
pcm = det.synth(fo, fs, 1, seed0=0)
out = det.alloc(fo, d.ds, d.sr)
for _ in range(2):
    det.run(pcm, fo, fs, params, mode=mode, out=out, d=d)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    det.run(pcm, fo, fs, params, mode=mode, out=out, d=d)
torch.cuda.synchronize()
print(f"{mode} unpipelined: {(time.perf_counter() - t0) / steps * 1e3:.3f} ms/batch", flush=True)
ref = out.to_host()
configs = [(16, True, False), (32, True, False), (48, True, False), (64, True, False), (128, True, False)]
for free, prio, emask in configs * 3:
    p = BatchPipeline(0, fo, fs, params, mode=mode, d=d, det_free_cus=free, env_priority=prio, env_masked=emask)
    for _ in range(2):
        p.submit(pcm)
    p.finish()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        last = p.submit(pcm)
    p.finish()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    got = last.to_host()
    same = all(np.array_equal(a[k], b[k], equal_nan=True) for a, b in zip(got, ref)
               for k in ("env", "floor", "troughs", "peaks")) and all(a["flags"] == b["flags"] for a, b in zip(got, ref))
    print(f"{mode} pipelined free_cus={free} env_priority={prio} env_masked={emask}: {ms:.3f} ms/batch, "
          f"identical={same}", flush=True)
    p.close()
