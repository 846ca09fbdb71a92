"""Write the final-floor inputs of the bench workload for tools/rqbench.hip.

    python tools/dump_floor_inputs.py [F] [native|reference|vulpine] [out path] [mult]

Runs the library (ENVELOPE | FLOOR) on the bench's synthetic batch and writes
F, Nd, then env (f64 [F*Nd]), the sanitised troughs' counts (i32 [F]), the
troughs (i64, Nd slots per recording) and the library's floor (f64 [F*Nd]),
which the harness's kernels must reproduce bit for bit.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpm_analysis_amd import DEFAULT_PARAMS, _native as N  # noqa: E402
from bpm_analysis_amd.engine import Detector  # noqa: E402

F, fs, n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024, 44100, 44100 * 60
mode = sys.argv[2] if len(sys.argv) > 2 else "native"
path = sys.argv[3] if len(sys.argv) > 3 else "/tmp/floor_in.bin"
det = Detector(0)
params = dict(DEFAULT_PARAMS)
if len(sys.argv) > 4:
    params["trough_rejection_multiplier"] = float(sys.argv[4])
if mode == "vulpine":
    # the reference's own sample: F windows of its reference-pipeline envelope
    # (bench.py real_envelope_detection), FLOOR only
    import torch
    from bpm_analysis_amd.design import design, detect_design
    g = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                             "vulpine.npz"), allow_pickle=False)
    sr = int(g["sr"])
    nd = -(-n // design(fs, params, log=False).ds)
    env0 = g["env"]
    starts = [(k * 997) % (len(env0) - nd) for k in range(F)]
    fr = np.arange(F + 1, dtype=np.int64) * nd
    res = det.alloc(fr, 1, sr)
    res.env.copy_(torch.from_numpy(np.concatenate([env0[s:s + nd] for s in starts])).to(det.device))
    det.run(None, fr, sr, params, stages=N.STAGE_FLOOR, out=res, d=detect_design(sr, params))
else:
    fo = np.arange(F + 1, dtype=np.int64) * n
    pcm = det.synth(fo, fs, 1, seed0=0)
    res = det.run(pcm, fo, fs, params, mode=mode, stages=N.STAGE_ENVELOPE | N.STAGE_FLOOR)
env = res.env.cpu().numpy()
floor = res.floor.cpu().numpy()
tr = res.troughs.cpu().numpy()
ntr = res.n_troughs.cpu().numpy().astype(np.int32)
nd = len(env) // F
with open(path, "wb") as fh:
    np.array([F, nd], dtype=np.int64).tofile(fh)
    env.astype(np.float64).tofile(fh)
    ntr.tofile(fh)
    tr.astype(np.int64).tofile(fh)
    floor.astype(np.float64).tofile(fh)
print("wrote", F, nd, "troughs/recording", float(ntr.mean()))
