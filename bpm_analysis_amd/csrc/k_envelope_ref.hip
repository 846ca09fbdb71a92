/*
 * k_envelope_ref.hip — reference-mode envelope, bit-exact.
 *
 * Restates bpm_analysis.py:1031-1054 for a batch of recordings:
 *   x[::ds] (no anti-alias, :1033) -> filtfilt(b, a) at the decimated rate
 *   (:1044-1045; scipy _signaltools.py:4523-4557, odd pad of 15 in the input
 *   dtype, DF-II-transposed recursion of _sigtools._linear_filter) -> |y| ->
 *   pandas centred rolling mean, Kahan add/remove (:1052-1054).
 *
 * Bit-exactness forces a strictly sequential recursion per file, so the
 * parallelism is across files: one lane per recording.  The forward-pass
 * output is parked in an interleaved scratch [step][file] so the 64 lanes of
 * a wave touch one contiguous 512-B row per step (coalesced), the backward
 * pass overwrites it in place with y, and the rolling mean streams it again.
 * The strided PCM gather (one int16 every ds frames) is software-pipelined
 * eight samples ahead so HBM latency overlaps the f64 recursion.
 * Roofline: neither HBM nor VALU — it is the latency of ~3 dependent f64
 * ops per step times 2*(Nd+30) + Nd steps.
 */
#include "bpmx_common.h"
#include "bpmx_kernels.h"

namespace bpmx {

struct Df2t {
    double b0, b1, b2, b3, b4, a1, a2, a3, a4;
    double z0, z1, z2, z3;
    /* scipy DOUBLE filt loop: y = Z0 + b0*x; Z_k = Z_{k+1} + x*b_{k+1} - y*a_{k+1} */
    __device__ __forceinline__ double step(double xn) {
        double yn = z0 + b0 * xn;
        z0 = z1 + xn * b1 - yn * a1;
        z1 = z2 + xn * b2 - yn * a2;
        z2 = z3 + xn * b3 - yn * a3;
        z3 = xn * b4 - yn * a4;
        return yn;
    }
};

/* pandas roll_mean state (aggregations.pyx add_mean/remove_mean/calc_mean) */
struct RollMean {
    double sum = 0, cadd = 0, crem = 0, prev = 0;
    int64_t nobs = 0, neg = 0, same = 0;
    __device__ __forceinline__ void add(double v) {
        if (v == v) {
            nobs++;
            double y = v - cadd, t = sum + y;
            cadd = t - sum - y;
            sum = t;
            if (__signbit(v)) neg++;
            if (v == prev) same++; else same = 1;
            prev = v;
        }
    }
    __device__ __forceinline__ void remove(double v) {
        if (v == v) {
            nobs--;
            double y = -v - crem, t = sum + y;
            crem = t - sum - y;
            sum = t;
            if (__signbit(v)) neg--;
        }
    }
    __device__ __forceinline__ double mean(int64_t minp) const {
        if (nobs >= minp && nobs > 0) {
            double r = sum / (double)nobs;
            if (same >= nobs) r = prev;
            else if (neg == 0 && r < 0) r = 0;
            else if (neg == nobs && r > 0) r = 0;
            return r;
        }
        return __builtin_nan("");
    }
};

/* Kahan rolling mean of |v| where v(j) = src[j*S] (interleaved scratch).
 * Writes env[i] (and y[i] = v(i) when y != nullptr). */
__device__ __forceinline__ void rolling_mean_abs(const double *src, int64_t S, int64_t n, int64_t w,
                                                 double *env, double *y) {
    RollMean R;
    int64_t ps = 0, pe = 0;
    for (int64_t i = 0; i < n; ++i) {
        int64_t s, e;
        win_bounds(i, n, w, s, e);
        if (i == 0 || s >= pe) {
            R = RollMean();
            R.prev = fabs(src[s * S]);
            for (int64_t j = s; j < e; ++j) R.add(fabs(src[j * S]));
        } else {
            for (int64_t j = ps; j < s; ++j) R.remove(fabs(src[j * S]));
            for (int64_t j = pe; j < e; ++j) R.add(fabs(src[j * S]));
        }
        env[i] = R.mean(1);
        if (y) y[i] = src[i * S];
        ps = s;
        pe = e;
    }
}

__global__ __launch_bounds__(64) void k_envelope_ref(EnvRefArgs A) {
    const int f = blockIdx.x * 64 + threadIdx.x;
    if (f >= A.n_files) return;
    const int64_t nd = A.doff[f + 1] - A.doff[f];
    if (nd <= 15 || !A.active[f]) return;
    const int64_t fb = A.foff[f];
    const int wdt = work_dtype(A.dtype, A.channels);
    const int64_t S = A.n_files;
    const int64_t ne = nd + 30;
    const int64_t ds = A.ds;
    double *scr = A.scratch + f;

    Df2t D;
    D.b0 = A.b[0]; D.b1 = A.b[1]; D.b2 = A.b[2]; D.b3 = A.b[3]; D.b4 = A.b[4];
    D.a1 = A.a[1]; D.a2 = A.a[2]; D.a3 = A.a[3]; D.a4 = A.a[4];

    const double x0 = frame_value(A.pcm, A.dtype, A.channels, fb);
    const double xl = frame_value(A.pcm, A.dtype, A.channels, fb + (nd - 1) * ds);
    /* forward pass, left pad: ext[j] = 2*x0 - xd[15-j] in the input dtype */
    double e0 = odd_ext(wdt, x0, frame_value(A.pcm, A.dtype, A.channels, fb + 15 * ds));
    D.z0 = A.zi[0] * e0; D.z1 = A.zi[1] * e0; D.z2 = A.zi[2] * e0; D.z3 = A.zi[3] * e0;
    for (int j = 0; j < 15; ++j) {
        double xn = odd_ext(wdt, x0, frame_value(A.pcm, A.dtype, A.channels, fb + (15 - j) * ds));
        scr[j * S] = D.step(xn);
    }
    /* body: xd[j], gathered 8 ahead */
    {
        double cur[8], nxt[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            int64_t jj = u < nd ? u : nd - 1;
            cur[u] = frame_value(A.pcm, A.dtype, A.channels, fb + jj * ds);
        }
        for (int64_t j = 0; j < nd; j += 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                int64_t jj = j + 8 + u;
                jj = jj < nd ? jj : nd - 1;
                nxt[u] = frame_value(A.pcm, A.dtype, A.channels, fb + jj * ds);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (j + u < nd) scr[(15 + j + u) * S] = D.step(cur[u]);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) cur[u] = nxt[u];
        }
    }
    /* right pad: ext[15+nd+k] = 2*xl - xd[nd-2-k] */
    for (int k = 0; k < 15; ++k) {
        double xn = odd_ext(wdt, xl, frame_value(A.pcm, A.dtype, A.channels, fb + (nd - 2 - k) * ds));
        scr[(15 + nd + k) * S] = D.step(xn);
    }
    /* backward pass over the reversed forward output, in place */
    {
        const double y0 = scr[(ne - 1) * S];
        D.z0 = A.zi[0] * y0; D.z1 = A.zi[1] * y0; D.z2 = A.zi[2] * y0; D.z3 = A.zi[3] * y0;
        int64_t j = ne - 1;
        for (; j >= 7; j -= 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = scr[(j - u) * S];
#pragma unroll
            for (int u = 0; u < 8; ++u) scr[(j - u) * S] = D.step(v[u]);
        }
        for (; j >= 0; --j) scr[j * S] = D.step(scr[j * S]);
    }
    /* |y| centred rolling mean over the trimmed range [15, 15+nd) */
    const int64_t d0 = A.doff[f];
    rolling_mean_abs(scr + 15 * S, S, nd, A.env_window, A.env + d0, A.y ? A.y + d0 : nullptr);
}

}  // namespace bpmx
