"""Block-state tables for the native-mode sosfiltfilt + decimation kernels.

sosfiltfilt (scipy/signal/_signaltools.py:4718-4829) of the 2-section band-pass
at the native rate is a linear time-invariant recursion, so over one
decimation block of ds samples it collapses to matrix algebra:

  state s = (z00, z01, z10, z11) of the two transposed-direct-form sections,
  one sample:   s' = A s + B u,   y = C s + D u      (sosfilt's per-section ops)

  forward, block j = ext[c_j, c_j+ds), c_j = 15 + j*ds:
      S_{j+1} = M S_j + u_j,     M = A^ds,   u_j = sum_i F_i ext[c_j+i],  F_i = A^(ds-1-i) B
  backward state before processing c_j (the reversed pass walks down):
      Q_j = M Q_{j+1} + P S_j + v_j,
      P = sum_{i=1..ds} A^(i-1) B C A^i,
      v_j = sum_{i'=0..ds} G_i' ext[c_j+i'],
      G_i' = [i'>=1] A^(i'-1) B D + sum_{i=i'+1..ds} A^(i-1) B (C A^(i-1-i') B)
  decimated output (= y[::ds] after trimming the 15-sample pads):
      yd_j = C Q_j + D (C S_j + D ext[c_j])

The per-sample work is the 8 dot products behind u_j and v_j (k_native_blocks);
the recursions over blocks are affine scans (k_native_scan).  Tables are built
in extended precision (np.longdouble) and rounded once to f64.
"""
from __future__ import annotations

import functools

import numpy as np


def state_space(sos: np.ndarray):
    """(A, B, C, D) of the 2-section cascade, probing scipy's _sosfilt step."""
    sos = np.asarray(sos, dtype=np.longdouble).reshape(2, 6)

    def step(s, u):
        s = list(s)
        x1 = sos[0, 0] * u + s[0]
        z00 = sos[0, 1] * u - sos[0, 4] * x1 + s[1]
        z01 = sos[0, 2] * u - sos[0, 5] * x1
        y = sos[1, 0] * x1 + s[2]
        z10 = sos[1, 1] * x1 - sos[1, 4] * y + s[3]
        z11 = sos[1, 2] * x1 - sos[1, 5] * y
        return np.array([z00, z01, z10, z11], dtype=np.longdouble), y

    A = np.zeros((4, 4), dtype=np.longdouble)
    C = np.zeros(4, dtype=np.longdouble)
    for k in range(4):
        e = np.zeros(4, dtype=np.longdouble)
        e[k] = 1
        A[:, k], C[k] = step(e, np.longdouble(0))
    B, D = step(np.zeros(4, dtype=np.longdouble), np.longdouble(1))
    return A, B, C, D


@functools.lru_cache(maxsize=32)
def _tables(sos_key: tuple, ds: int):
    A, B, C, D = state_space(np.array(sos_key))
    L = ds
    pw = [np.eye(4, dtype=np.longdouble)]
    for _ in range(L + 1):
        pw.append(A @ pw[-1])
    F = np.stack([pw[L - 1 - i] @ B for i in range(L)])                    # [L, 4]
    h = np.array([C @ pw[k] @ B for k in range(L + 1)])                     # h[k] = C A^k B
    AB = np.stack([pw[i] @ B for i in range(L + 1)])                        # A^i B
    P = sum(np.outer(AB[i - 1], C @ pw[i]) for i in range(1, L + 1))       # [4, 4]
    G = np.zeros((L + 1, 4), dtype=np.longdouble)
    for ip in range(L + 1):
        g = AB[ip - 1] * D if ip >= 1 else np.zeros(4, dtype=np.longdouble)
        for i in range(ip + 1, L + 1):
            g = g + AB[i - 1] * h[i - 1 - ip]
        G[ip] = g
    M = pw[L]
    f64 = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    return dict(A=f64(A), B=f64(B), C=f64(C), D=float(D), M=f64(M), P=f64(P), F=f64(F), G=f64(G))


def tables(sos: np.ndarray, ds: int) -> dict:
    return _tables(tuple(float(v) for v in np.asarray(sos).ravel()), int(ds))


def pack(sos: np.ndarray, sos_zi: np.ndarray, ds: int) -> np.ndarray:
    """Flat f64 table handed to the kernels (layout mirrored in k_envelope_native.hip):
    [0:16) A row-major | [16:20) B | [20:24) C | [24] D | [25:41) M | [41:57) P |
    [57:61) zi (z00,z01,z10,z11) | [64 : 64+8*ds) F_i | [64+8*ds+4...) interleaved:
    per i in [0, ds]: (F_i[0..3] or 0 for i == ds, G_i[0..3])."""
    t = tables(sos, ds)
    out = np.zeros(64 + 8 * (ds + 1), dtype=np.float64)
    out[0:16] = t["A"].ravel()
    out[16:20] = t["B"]
    out[20:24] = t["C"]
    out[24] = t["D"]
    out[25:41] = t["M"].ravel()
    out[41:57] = t["P"].ravel()
    out[57:61] = np.asarray(sos_zi, dtype=np.float64).ravel()
    coef = out[64:].reshape(ds + 1, 8)
    coef[:ds, 0:4] = t["F"]
    coef[:, 4:8] = t["G"]
    return out


def model_decimated(x_ext: np.ndarray, sos: np.ndarray, sos_zi: np.ndarray, ds: int, n: int) -> np.ndarray:
    """numpy model of the block formulation (test aid): y[::ds] of sosfiltfilt
    given the padded f64 signal x_ext (length n + 30)."""
    t = tables(sos, ds)
    A, B, C, D, M, P, F, G = (t[k] for k in "ABCDMPFG")
    zi = np.asarray(sos_zi, dtype=np.float64).ravel()
    nd = -(-n // ds)
    ne = n + 30

    def stepf(s, u):
        return A @ s + B * u, C @ s + D * u

    s = zi * x_ext[0]
    for m in range(15):
        s, _ = stepf(s, x_ext[m])
    nb = nd - 1
    S = np.zeros((nd, 4))
    S[0] = s
    for j in range(nb):
        c = 15 + j * ds
        S[j + 1] = M @ S[j] + F.T @ x_ext[c:c + ds]
    # tail: exact recursion over [c_{nd-1}, ne)
    c_last = 15 + (nd - 1) * ds
    yf = []
    s = S[nd - 1].copy()
    for m in range(c_last, ne):
        s, y = stepf(s, x_ext[m])
        yf.append(y)
    q = zi * yf[-1]
    for idx in range(len(yf) - 1, 0, -1):
        q = A @ q + B * yf[idx]
    Q = np.zeros((nd, 4))
    Q[nd - 1] = q
    for j in range(nb - 1, -1, -1):
        c = 15 + j * ds
        Q[j] = M @ Q[j + 1] + P @ S[j] + G.T @ x_ext[c:c + ds + 1]
    out = np.empty(nd)
    for j in range(nd):
        c = 15 + j * ds
        out[j] = C @ Q[j] + D * (C @ S[j] + D * x_ext[c])
    return out


TILE = 64   # blocks per k_native_blocks tile (one per lane)


@functools.lru_cache(maxsize=32)
def _tile_tables(sos_key: tuple, ds: int, T: int):
    """Extended-precision tables of the tile formulation (k_native_blocks ->
    k_native_carry -> k_native_yd), see model_tiled."""
    A, B, C, D = state_space(np.array(sos_key))
    L = ds
    pw = [np.eye(4, dtype=np.longdouble)]
    for _ in range(L + 1):
        pw.append(A @ pw[-1])
    M = pw[L]
    AB = np.stack([pw[i] @ B for i in range(L + 1)])
    P = sum(np.outer(AB[i - 1], C @ pw[i]) for i in range(1, L + 1))
    Mp = [np.eye(4, dtype=np.longdouble)]
    for _ in range(T):
        Mp.append(M @ Mp[-1])                                    # Mp[b] = M^b
    G = [None] * (T + 1)
    G[T] = np.zeros((4, 4), dtype=np.longdouble)
    for b in range(T - 1, -1, -1):                                # G_b = P M^b + M G_{b+1}
        G[b] = P @ Mp[b] + M @ G[b + 1]
    alpha = np.stack([C @ Mp[T - b] for b in range(T)])           # C M^(T-b)
    beta = np.stack([C @ G[b] + D * (C @ Mp[b]) for b in range(T)])
    kpow = np.stack([Mp[1 << k] for k in range(int(np.log2(T)))])  # M^1, M^2, ..., M^(T/2)
    f64 = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    return dict(MT=f64(Mp[T]), G0=f64(G[0]), alpha=f64(alpha), beta=f64(beta), kpow=f64(kpow))


def tile_tables(sos: np.ndarray, ds: int, T: int = TILE) -> dict:
    return _tile_tables(tuple(float(v) for v in np.asarray(sos).ravel()), int(ds), int(T))


def model_tiled(x_ext: np.ndarray, sos: np.ndarray, sos_zi: np.ndarray, ds: int, n: int, T: int = TILE):
    """numpy model of the tiled kernels (test aid; must equal model_decimated):

    per full tile t of T blocks (j0 = T t), lane b, with u, v the block sums:
      incl_b = sum_{c<=b} M^(b-c) u_c,   loc_b = incl_(b-1),   w_b = P loc_b + v_b
      R_b = sum_{c>=b} M^(c-b) w_c
      yd_b = alpha_b . Qe_t + beta_b . S0_t + gamma_b,
      gamma_b = C R_b + D C loc_b + D^2 x_b
    carries (per file, sequential over tiles):
      S0_(t+1) = M^T S0_t + incl_(T-1),   Q_start_t = M^T Qe_t + R_0 + G_0 S0_t = Qe_(t-1)
    the partial last tile and the tail run the exact block / sample recursions."""
    t = tables(sos, ds)
    A, B, C, D, M, P, F, G = (t[k] for k in "ABCDMPFG")
    tt = tile_tables(sos, ds, T)
    zi = np.asarray(sos_zi, dtype=np.float64).ravel()
    nd = -(-n // ds)
    nb = nd - 1
    ne = n + 30

    def stepf(s, u):
        return A @ s + B * u, C @ s + D * u

    s = zi * x_ext[0]
    for m in range(15):
        s, _ = stepf(s, x_ext[m])
    c = lambda j: 15 + j * ds
    u = np.array([F.T @ x_ext[c(j):c(j) + ds] for j in range(nb)]).reshape(nb, 4)
    v = np.array([G.T @ x_ext[c(j):c(j) + ds + 1] for j in range(nb)]).reshape(nb, 4)
    xb = np.array([x_ext[c(j)] for j in range(nd)])
    nt = nb // T
    gam = np.zeros(nt * T)
    aggF = np.zeros((nt, 4))
    R0 = np.zeros((nt, 4))
    for ti in range(nt):                                           # k_native_blocks, full tiles
        j0 = ti * T
        incl = np.zeros((T, 4))
        acc = np.zeros(4)
        for b in range(T):
            acc = M @ acc + u[j0 + b]
            incl[b] = acc
        loc = np.vstack([np.zeros(4), incl[:-1]])
        w = (P @ loc.T).T + v[j0:j0 + T]
        R = np.zeros((T, 4))
        acc = np.zeros(4)
        for b in range(T - 1, -1, -1):
            acc = M @ acc + w[b]
            R[b] = acc
        gam[j0:j0 + T] = R @ C + D * (loc @ C) + D * D * xb[j0:j0 + T]
        aggF[ti] = incl[-1]
        R0[ti] = R[0]
    S0 = np.zeros((nt + 1, 4))                                     # k_native_carry
    S0[0] = s
    for ti in range(nt):
        S0[ti + 1] = tt["MT"] @ S0[ti] + aggF[ti]
    Sp = [S0[nt]]
    for j in range(nt * T, nb):
        Sp.append(M @ Sp[-1] + u[j])
    slast = Sp[-1]
    yf = []
    s = slast.copy()
    for m in range(c(nd - 1), ne):
        s, y = stepf(s, x_ext[m])
        yf.append(y)
    q = zi * yf[-1]
    for idx in range(len(yf) - 1, 0, -1):
        q = A @ q + B * yf[idx]
    out = np.empty(nd)
    out[nd - 1] = C @ q + D * yf[0]
    for j in range(nb - 1, nt * T - 1, -1):
        Sj = Sp[j - nt * T]
        q = M @ q + P @ Sj + v[j]
        out[j] = C @ q + D * (C @ Sj + D * xb[j])
    Qe = np.zeros((nt, 4))
    for ti in range(nt - 1, -1, -1):
        Qe[ti] = q
        q = tt["MT"] @ q + R0[ti] + tt["G0"] @ S0[ti]
    for ti in range(nt):                                           # k_native_yd
        j0 = ti * T
        out[j0:j0 + T] = tt["alpha"] @ Qe[ti] + tt["beta"] @ S0[ti] + gam[j0:j0 + T]
    return out
