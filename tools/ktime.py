"""A/B kernel timing of library builds on the metric batch (no parity check:
diagnostic builds may produce wrong outputs).

    python tools/ktime.py [--steps K] [--files F] lib1.so lib2.so[,VAR=VALUE...] ...

Each build runs in its own child process (BPMX_LIB), alternating twice:
step time (events around bpmx_run) and per-kernel device time from a fully
profiled pass (bpmx_profile)."""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, sys, time
import numpy as np, torch
sys.path.insert(0, ".")
from bpm_analysis_amd import DEFAULT_PARAMS
from bpm_analysis_amd.engine import Detector
from bpm_analysis_amd.design import design
F, steps, mode = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
fs, n = 44100, 44100 * 60
fo = np.arange(F + 1, dtype=np.int64) * n
det = Detector(0)
params = dict(DEFAULT_PARAMS)
d = design(fs, params, log=False)
pcm = det.synth(fo, fs, 1, seed0=0)
out = det.alloc(fo, d.ds, d.sr)
for _ in range(3):
    det.run(pcm, fo, fs, params, mode=mode, out=out, d=d)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(steps):
    det.run(pcm, fo, fs, params, mode=mode, out=out, d=d)
e1.record()
torch.cuda.synchronize()
step = e0.elapsed_time(e1) / steps
det.profile(True)
for _ in range(steps):
    det.run(pcm, fo, fs, params, mode=mode, out=out, d=d)
torch.cuda.synchronize()
prof = det.profile_read()
det.profile(False)
print(json.dumps({"step_ms": step, "k": {k: v[1] / steps for k, v in prof.items()}}))
'''


def main():
    args = sys.argv[1:]
    steps, files, mode = 10, 1024, "native"
    libs = []
    while args:
        a = args.pop(0)
        if a == "--steps":
            steps = int(args.pop(0))
        elif a == "--files":
            files = int(args.pop(0))
        elif a == "--mode":
            mode = args.pop(0)
        else:
            libs.append(a)
    for rep in range(2):
        for spec in libs:
            lib, *kv = spec.split(",")
            env = dict(os.environ, BPMX_LIB=lib)
            env.update(x.split("=", 1) for x in kv)
            r = subprocess.run([sys.executable, "-c", CHILD, str(files), str(steps), mode], env=env,
                               capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                print(spec, "FAILED", r.stderr[-2000:], flush=True)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            ks = {k: round(v, 4) for k, v in sorted(d["k"].items(), key=lambda kv: -kv[1]) if v > 0.02}
            print(f"{spec} step {d['step_ms']:.4f} ms {ks}", flush=True)


if __name__ == "__main__":
    main()
