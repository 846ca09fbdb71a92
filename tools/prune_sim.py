"""Simulate the value-bin pruning of the final-floor rolling quantile on
synthetic recordings: fraction of the curve's samples that can ever be a
window's k-th or (k+1)-th smallest (exact bound, 64 value bins, 64-output
blocks).  Host-only study tool."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O
from bpm_analysis_amd.config import DEFAULT_PARAMS

NB = int(sys.argv[2]) if len(sys.argv) > 2 else 64


def keep_fraction(dense, t0, W, q, nbins=NB, blk=64):
    n = dense.size
    v = dense[t0:]
    vmin, vmax = v.min(), v.max()
    scale = (nbins - 1e-9) / (vmax - vmin) if vmax > vmin else 0.0
    bins = np.full(n, -1)
    bins[t0:] = np.minimum(((v - vmin) * scale).astype(np.int64), nbins - 1)
    off = (W - 1) // 2
    nbk = (n + blk - 1) // blk
    bstar = np.full(nbk, nbins - 1)
    for B in range(nbk):
        i0, i1 = B * blk, min(n, B * blk + blk) - 1
        e0 = min(i0 + 1 + off, n); s1 = max(min(i1 + 1 + off, n) - W, 0)
        lo, hi = max(s1, t0), e0            # intersection of the block's windows
        kmax = 0
        for i in (i0, i1):
            e = min(i + 1 + off, n); s = max(e - W, 0); nobs = e - max(s, t0)
            kmax = max(kmax, int(q * (nobs - 1)) if nobs > 1 else 0)
        if hi - lo < kmax + 2:
            continue
        c = np.cumsum(np.bincount(bins[lo:hi], minlength=nbins))
        bstar[B] = int(np.searchsorted(c, kmax + 2))
    # threshold per position: max over blocks whose union window contains it
    keep = np.zeros(n, bool)
    thr = np.full(n, -1)
    for B in range(nbk):
        i0, i1 = B * blk, min(n, B * blk + blk) - 1
        s0 = max(min(i0 + 1 + off, n) - W, 0); e1 = min(i1 + 1 + off, n)
        thr[s0:e1] = np.maximum(thr[s0:e1], bstar[B])
    keep[t0:] = bins[t0:] <= thr[t0:]
    return keep[t0:].mean()


p = dict(DEFAULT_PARAMS)
fr = []
for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    pcm = O.synth(seed, 2646000, 44100)
    d = O.derive(44100, p)
    env = O.preprocess_native(pcm, d)
    floor, tr, flags = O.noise_floor(env, d, p)
    dense = O.interp_dense(tr, env)
    fr.append(keep_fraction(dense, int(tr[0]), d.noise_window, p["noise_floor_quantile"]))
    print(seed, len(tr), round(fr[-1], 3))
print("mean keep", np.mean(fr))
