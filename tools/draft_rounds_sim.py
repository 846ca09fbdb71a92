"""Host-only study tool: rounds draft_point needs to bring a trough's active set to <= 64
elements with value pivots interpolated between the active extremes vs random element pivots, on
the bench's synthetic recordings (oracle envelopes, raw troughs).  Prints mean / max rounds."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O
from bpm_analysis_amd.config import DEFAULT_PARAMS
p = dict(DEFAULT_PARAMS)
def win(i, n, W):
    off = (W - 1) // 2; e = min(i + 1 + off, n); s = max(e - W, 0); return s, e
rs = {"interp": [], "random": []}
rng = np.random.default_rng(1)
for seed in range(2):
    pcm = O.synth(seed, 2646000, 44100)
    d = O.derive(44100, p)
    env = O.preprocess_native(pcm, d)
    n = env.size; W = d.noise_window; q = 0.2
    thr = O.quantile(env, 0.1)
    tr = O.find_peaks(env, distance=d.distance, prominence=thr, negate=True)
    dense = O.interp_dense(tr, env); t0 = tr[0]
    for t in tr[::3]:
        s, e = win(t, n, W); lo = max(s, t0); w = np.sort(dense[lo:e]); nobs = w.size; k = int(q * (nobs - 1))
        for mode in rs:
            a, b = 0, nobs   # active [a, b) in sorted order
            rounds = 0
            while b - a > 64:
                rounds += 1
                if mode == "random" or rounds > 8:
                    pv = w[rng.integers(a, b)]
                else:
                    amin, amax = w[a], w[b - 1]
                    if amin == amax: break
                    pv = amin + (amax - amin) * ((k - a) + 0.5) / (b - a)
                nl = np.searchsorted(w, pv, 'left'); nr = np.searchsorted(w, pv, 'right')
                if k < nl: b = nl
                elif k < nr: break
                else: a = nr
            rs[mode].append(rounds)
for m, v in rs.items(): v = np.array(v); print(m, "rounds mean %.2f max %d" % (v.mean(), v.max()))
