"""Host-only study tool: find_peaks distance-filter structure on oracle envelopes (reference and
native mode, both signs): synchronous rounds of the local rule, neighbour-count histogram, component
sizes (runs of maxima closer than the distance), and wave-local rounds as k_find_peaks_lds runs them."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O
from bpm_analysis_amd.config import DEFAULT_PARAMS
p = dict(DEFAULT_PARAMS)
def maxima(x):
    n = x.size; out = []
    i = 1
    while i < n - 1:
        if x[i - 1] < x[i]:
            ia = i + 1
            while ia < n - 1 and x[ia] == x[i]: ia += 1
            if x[ia] < x[i]: out.append((i + ia - 1) // 2); i = ia; continue
        i += 1
    return np.array(out)
for mode in ("reference", "native"):
  for sign in (1, -1):
    pcm = O.synth(3, 2646000, 44100)
    d = O.derive(44100, p)
    env = O.preprocess_ref(pcm, d) if mode == "reference" else O.preprocess_native(pcm, d)
    env = env[0] if isinstance(env, tuple) else env
    x = sign * env
    mp = maxima(x); h = x[mp]; M = len(mp); dist = d.distance
    st = np.zeros(M, np.int8)  # 0 undecided 1 kept 2 removed
    rounds = 0
    H = []
    for j in range(M):
        l = []
        k = j - 1
        while k >= 0 and mp[j] - mp[k] < dist:
            if h[k] > h[j]: l.append(k)
            k -= 1
        k = j + 1
        while k < M and mp[k] - mp[j] < dist:
            if h[k] >= h[j]: l.append(k)
            k += 1
        H.append(l)
    while (st == 0).any():
        rounds += 1
        new = st.copy()
        for j in np.nonzero(st == 0)[0]:
            s = [st[k] for k in H[j]]
            if 1 in s: new[j] = 2
            elif 0 not in s: new[j] = 1
        st = new
    # component sizes: gaps < dist
    gaps = np.diff(mp); comps = np.split(np.arange(M), np.nonzero(gaps >= dist)[0] + 1)
    print(mode, sign, "maxima", M, "dist", dist, "synchronous rounds", rounds, "kept", (st == 1).sum(), "max comp", max(len(c) for c in comps), "ncomp", len(comps), "avg |H|", np.mean([len(l) for l in H]))
    Hs = np.array([len(l) for l in H]); print("   |H| hist", np.bincount(Hs)[:12], "frac>4 %.3f" % (Hs > 4).mean())
    # wave-local async simulation: entries j -> wave (j % 1024)//64, rounds local until no progress, then barrier
    st = np.zeros(M, np.int8); gi = 0; lrt = 0
    wave = (np.arange(M) % 1024) // 64
    while (st == 0).any():
        gi += 1
        for w in range(16):
            js = [j for j in np.nonzero(wave == w)[0]]
            while True:
                prog = False
                for j in js:
                    if st[j] != 0: continue
                    s = [st[k] for k in H[j]]
                    if 1 in s: st[j] = 2; prog = True
                    elif 0 not in s: st[j] = 1; prog = True
                lrt += 1
                if not prog: break
    print("   global iters", gi, "local rounds total", lrt)
