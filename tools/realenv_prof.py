"""Per-kernel device time of the detection stages (FLOOR | PEAKS) on 60 s
windows of the vulpine sample's envelope (bench.py real_envelope_detection)
and on synthetic envelopes, for library builds given on the command line
(BPMX_LIB per child process).

    python tools/realenv_prof.py [reference|native_style] [lib.so ...]"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, sys
import numpy as np, torch
sys.path.insert(0, ".")
from bpm_analysis_amd import DEFAULT_PARAMS, _native as N
from bpm_analysis_amd.engine import Detector
from bpm_analysis_amd.design import design, detect_design
F, fs, n = 1024, 44100, 44100 * 60
det = Detector(0)
params = dict(DEFAULT_PARAMS)
d = design(fs, params, log=False)
nd = -(-n // d.ds)
import pandas as pd, scipy.signal as ssig
g = np.load("tests/golden/vulpine.npz", allow_pickle=False)
sr = int(g["sr"])
env0 = g["env"] if sys.argv[1] == "reference" else pd.Series(np.abs(ssig.hilbert(g["pcm"].astype(np.float64)))).rolling(
    sr // 10, min_periods=1, center=True).mean().to_numpy()
starts = [(k * 997) % (len(env0) - nd) for k in range(F)]
fr = np.arange(F + 1, dtype=np.int64) * nd
dr = detect_design(sr, params)
o = det.alloc(fr, 1, sr)
o.env.copy_(torch.from_numpy(np.concatenate([env0[s:s + nd] for s in starts])).to(det.device))
fo = np.arange(F + 1, dtype=np.int64) * n
pcm = det.synth(fo, fs, 1, seed0=0)
so = det.alloc(fo, d.ds, d.sr)
det.run(pcm, fo, fs, params, mode="native", out=so, d=d)
s2 = det.alloc(fr, 1, sr)
s2.env.copy_(so.env)
res = {}
for name, oo in (("real", o), ("synthetic", s2)):
    for _ in range(2):
        det.run(None, fr, sr, params, stages=6, out=oo, d=dr)
    torch.cuda.synchronize()
    det.profile(True)
    for _ in range(5):
        det.run(None, fr, sr, params, stages=6, out=oo, d=dr)
    torch.cuda.synchronize()
    p = det.profile_read()
    det.profile(False)
    res[name] = {k: round(v[1] / 5, 4) for k, v in sorted(p.items(), key=lambda kv: -kv[1][1])}
print(json.dumps(res))
'''
src = "native_style"
libs = []
for a in sys.argv[1:]:
    if a in ("reference", "native_style"):
        src = a
    else:
        libs.append(a)
for lib in libs or ["bpm_analysis_amd/libbpmx.so"]:
    r = subprocess.run([sys.executable, "-c", CHILD, src], env=dict(os.environ, BPMX_LIB=lib), capture_output=True,
                       text=True, timeout=600)
    if r.returncode:
        print(lib, "FAILED", r.stderr[-2000:])
        sys.exit(1)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    for k, v in d.items():
        print(lib, k, "total", round(sum(v.values()), 3), v)
