"""Write gpurun_out/env.bin: envelopes of the bench workload (for tools/fpbench).

    python tools/dump_env.py [F] [native|reference|vulpine] [out path]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpm_analysis_amd import DEFAULT_PARAMS, _native as N  # noqa: E402
from bpm_analysis_amd.engine import Detector  # noqa: E402

F, fs, n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024, 44100, 44100 * 60
det = Detector(0)
fo = np.arange(F + 1, dtype=np.int64) * n
pcm = det.synth(fo, fs, 1, seed0=0)
params = dict(DEFAULT_PARAMS)
mode = sys.argv[2] if len(sys.argv) > 2 else "native"
if mode == "vulpine":
    # F windows of the reference's own sample's reference-pipeline envelope
    # (bench.py real_envelope_detection)
    from bpm_analysis_amd.design import design
    g = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                             "vulpine.npz"), allow_pickle=False)
    nd = -(-n // design(fs, params, log=False).ds)
    env0 = g["env"]
    env = np.concatenate([env0[s:s + nd] for s in [(k * 997) % (len(env0) - nd) for k in range(F)]])
else:
    res = det.run(pcm, fo, fs, params, mode=mode, stages=N.STAGE_ENVELOPE)
    env = res.env.cpu().numpy()
nd = len(env) // F
os.makedirs("gpurun_out", exist_ok=True)
path = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/env.bin"
with open(path, "wb") as fh:
    np.array([F, nd], dtype=np.int64).tofile(fh)
    env.astype(np.float64).tofile(fh)
print("wrote", F, nd)
