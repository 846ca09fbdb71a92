/*
 * bpmx_common.h — device helpers shared by the bpmx kernels (gfx950, wave64).
 *
 * Everything here is compiled with -ffp-contract=off: the bit-exact stages
 * must evaluate a*b+c as a rounded product followed by a rounded sum, as the
 * reference's compiled scipy/pandas/numpy loops do.  Kernels that may fuse
 * call __builtin_fma explicitly.
 */
#ifndef BPMX_COMMON_H
#define BPMX_COMMON_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bpmx.h"

#define BPMX_WAVE 64

namespace bpmx {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

/* ---- PCM access ------------------------------------------------------- */
/* numpy dtype of x after `np.mean(axis=1)` (bpm_analysis.py:1015-1016):
 * mono keeps its dtype, multi-channel ints -> f64, f32 -> f32. */
__host__ __device__ __forceinline__ int work_dtype(int dtype, int channels) {
    if (channels <= 1) return dtype;
    return dtype == BPMX_DT_F32 ? BPMX_DT_F32 : BPMX_DT_F64;
}

__device__ __forceinline__ double load_pcm(const void *pcm, int dtype, int64_t idx) {
    switch (dtype) {
    case BPMX_DT_U8: return (double)((const uint8_t *)pcm)[idx];
    case BPMX_DT_I16: return (double)((const int16_t *)pcm)[idx];
    case BPMX_DT_I32: return (double)((const int32_t *)pcm)[idx];
    case BPMX_DT_F32: return (double)((const float *)pcm)[idx];
    default: return ((const double *)pcm)[idx];
    }
}

/* value of frame `frame` after the channel mean */
__device__ __forceinline__ double frame_value(const void *pcm, int dtype, int channels, int64_t frame) {
    if (channels <= 1) return load_pcm(pcm, dtype, frame);
    if (dtype == BPMX_DT_F32) {
        const float *p = (const float *)pcm + frame * channels;
        float s = p[0];
        for (int c = 1; c < channels; ++c) s = s + p[c];
        return (double)(s / (float)channels);
    }
    double s = load_pcm(pcm, dtype, frame * channels);
    for (int c = 1; c < channels; ++c) s = s + load_pcm(pcm, dtype, frame * channels + c);
    return s / (double)channels;
}

/* scipy odd_ext (_arraytools.py:57-107): 2*end - v evaluated in the working
 * dtype, i.e. with integer wraparound or float32 rounding. */
__device__ __forceinline__ double odd_ext(int wdt, double end, double v) {
    switch (wdt) {
    case BPMX_DT_U8: return (double)(uint8_t)(uint32_t)(2 * (int64_t)end - (int64_t)v);
    case BPMX_DT_I16: return (double)(int16_t)(uint16_t)(uint32_t)(2 * (int64_t)end - (int64_t)v);
    case BPMX_DT_I32: return (double)(int32_t)(uint32_t)(2 * (int64_t)end - (int64_t)v);
    case BPMX_DT_F32: {
        float t = (float)end * 2.0f;
        return (double)(t - (float)v);
    }
    default: return 2.0 * end - v;
    }
}

/* ---- order-preserving f64 key ----------------------------------------- */
__device__ __forceinline__ uint64_t f64_key(double v) {
    uint64_t b = (uint64_t)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double key_f64(uint64_t k) {
    uint64_t b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
    return __longlong_as_double((long long)b);
}

/* numpy _lerp (numpy/lib/_function_base_impl.py:4639-4660) */
__host__ __device__ __forceinline__ double np_lerp(double a, double b, double t) {
    double d = b - a;
    if (t >= 0.5) return b - d * (1.0 - t);
    return a + d * t;
}

/* np.interp(x, t, v) with NaN left of t[0] — bpm_analysis.py:1082 /
 * numpy/_core/src/multiarray/compiled_base.c arr_interp: slope*(x-x0)+y0,
 * falling back to the right-anchored form (and y0 when y0 == y1) on NaN.
 * t: m ascending positions, v(j): the value at t[j]. */
template <typename TP, typename VF>
__device__ __forceinline__ double interp_at(int64_t x, const TP *t, VF v, int m) {
    if (m == 0 || x < (int64_t)t[0]) return __builtin_nan("");
    int lo = 0, hi = m;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)t[mid] <= x) lo = mid + 1; else hi = mid;
    }
    const int j = lo - 1;
    if (j == m - 1 || (int64_t)t[j] == x) return v(j);
    const double y0 = v(j), y1 = v(j + 1);
    const double slope = (y1 - y0) / ((double)t[j + 1] - (double)t[j]);
    double r = slope * ((double)x - (double)t[j]) + y0;
    if (r != r) {
        r = slope * ((double)x - (double)t[j + 1]) + y1;
        if (r != r && y0 == y1) r = y0;
    }
    return r;
}

/* pandas centered fixed window (pandas/core/indexers/objects.py:93-120) */
__host__ __device__ __forceinline__ void win_bounds(int64_t i, int64_t n, int64_t w, int64_t &s, int64_t &e) {
    int64_t off = (w - 1) / 2;
    int64_t ee = i + 1 + off, ss = ee - w;
    e = ee < 0 ? 0 : (ee > n ? n : ee);
    s = ss < 0 ? 0 : (ss > n ? n : ss);
}

/* ---- wave / block primitives (64-lane) -------------------------------- */
__device__ __forceinline__ double wave_min(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

/* position of the nth (0-based) set bit of x (nth < popcount(x)) */
__device__ __forceinline__ int select64(uint64_t x, int nth) {
    int pos = 0;
#pragma unroll
    for (int w = 32; w > 0; w >>= 1) {
        const int c = __popcll(x & ((1ull << w) - 1ull));
        if (nth >= c) {
            nth -= c;
            x >>= w;
            pos += w;
        }
    }
    return pos;
}

/* 64 x 64 bit-matrix transpose across a wave: on entry lane e holds row e
 * (bit j = column j), on exit lane j holds column j (bit e = row e).  Six
 * butterfly stages, partner lane ^ s, exchanging s-bit groups.  Every lane
 * of the wave must be active. */
__device__ __forceinline__ uint64_t transpose64(uint64_t x) {
    const int lane = threadIdx.x & 63;
    uint64_t msk = 0x00000000FFFFFFFFull;
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
        const uint64_t p = (uint64_t)__shfl_xor((long long)x, s);
        if (!(lane & s)) x ^= (((x >> s) ^ p) & msk) << s;
        else x ^= ((p >> s) ^ x) & msk;
        msk ^= msk << (s >> 1);
    }
    return x;
}

/* wave64 inclusive scan (sum, or running max) in registers with DPP: row
 * shifts 1/2/4/8 scan each 16-lane row, row_bcast:15 / row_bcast:31 carry the
 * row totals forward (GFX9 DPP; no LDS round trip, unlike __shfl_up).  Every
 * lane of the wave must be active. */
template <bool MAX>
__device__ __forceinline__ int wave_iscan_dpp(int x) {
    const int id = MAX ? INT_MIN : 0;
#define BPMX_DPP_STEP(ctrl, rmask)                                              \
    {                                                                           \
        const int t = __builtin_amdgcn_update_dpp(id, x, ctrl, rmask, 0xf, false); \
        x = MAX ? (t > x ? t : x) : x + t;                                      \
    }
    BPMX_DPP_STEP(0x111, 0xf)   /* row_shr:1 */
    BPMX_DPP_STEP(0x112, 0xf)   /* row_shr:2 */
    BPMX_DPP_STEP(0x114, 0xf)   /* row_shr:4 */
    BPMX_DPP_STEP(0x118, 0xf)   /* row_shr:8 */
    BPMX_DPP_STEP(0x142, 0xa)   /* row_bcast:15 -> rows 1, 3 */
    BPMX_DPP_STEP(0x143, 0xc)   /* row_bcast:31 -> rows 2, 3 */
#undef BPMX_DPP_STEP
    return x;
}
/* wave-wide maximum (every lane active) */
__device__ __forceinline__ int wave_max_dpp(int x) {
    return __builtin_amdgcn_readlane(wave_iscan_dpp<true>(x), 63);
}
/* value of the lane below (lane 0 gets `edge`) */
__device__ __forceinline__ int wave_shr1_dpp(int x, int edge) {
    return __builtin_amdgcn_update_dpp(edge, x, 0x138, 0xf, 0xf, false);   /* wave_shr:1 */
}

/* f64 one-lane wave shifts (DPP wave_shr:1 / wave_shl:1 on both halves): the
 * lane below / above, `edge` at lane 0 / 63.  Every lane must be active. */
__device__ __forceinline__ double dpp_shr1_d(double x, double edge) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(edge), __double2loint(x), 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(edge), __double2hiint(x), 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_shl1_d(double x, double edge) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(edge), __double2loint(x), 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(edge), __double2hiint(x), 0x130, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

/* exclusive block scan of 0/1 flags; `sh` holds NT/64+1 ints.  Returns the
 * exclusive prefix, writes the block total to *total.  Ends with a barrier. */
template <int NT>
__device__ __forceinline__ int block_scan_flag(bool flag, int *sh, int *total) {
    const int lane = lane_id(), wid = wave_id();
    unsigned long long m = __ballot(flag);
    int pre = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) sh[wid] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int w = 0; w < NT / 64; ++w) { int t = sh[w]; sh[w] = acc; acc += t; }
        sh[NT / 64] = acc;
    }
    __syncthreads();
    int r = pre + sh[wid];
    *total = sh[NT / 64];
    __syncthreads();
    return r;
}

/* exclusive block scan of small non-negative ints */
template <int NT>
__device__ __forceinline__ int block_scan_int(int v, int *sh, int *total) {
    const int lane = lane_id(), wid = wave_id();
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int w = 0; w < NT / 64; ++w) { int t = sh[w]; sh[w] = acc; acc += t; }
        sh[NT / 64] = acc;
    }
    __syncthreads();
    int r = x - v + sh[wid];
    *total = sh[NT / 64];
    __syncthreads();
    return r;
}

}  // namespace bpmx

#endif
