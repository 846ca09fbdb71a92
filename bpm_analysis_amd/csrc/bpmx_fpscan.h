/*
 * bpmx_fpscan.h — the extrema scan of find_peaks (scipy's _local_maxima_1d,
 * plateau midpoints, scipy/signal/_peak_finding_utils.pyx) as k_find_peaks_lds
 * runs it: over positions 1 .. n-2 of x (x = sign * env), wave w of a
 * 1024-thread workgroup scans its own contiguous run [w0, w1) 64 positions at
 * a time and compacts, in order, the local maxima (plateau midpoints) into
 * mp[w0 - 1 ..] and the valleys (strict local minima / flat bottoms, also at
 * their plateau midpoints; only their values are used) into vp[w0 - 1 ..],
 * with their values x (equal along a plateau) in mv / vv at the same indices:
 * the consumers read the extrema's values from these lists instead of
 * gathering them from the envelope (a recording's envelope does not stay in
 * L2 between the scan and the gathers: ~2000 scattered cache lines each).
 *
 * The maxima of -env are the valleys of env and its valleys env's maxima, at
 * the same positions in the same per-wave runs, so one scan serves both
 * find_peaks calls of a run (bpm_analysis.py:1066-1070 and :223-229): the
 * record (PeakArgs scan_ok) says which sign the lists were made for, and a consumer of
 * the other sign swaps them: the trough launch of k_find_peaks_lds writes it
 * and the peak launch reads it.  (Scanning in k_hilbert_env from the staged
 * envelope instead was measured: the trough launch 0.150 -> 0.115 ms, the
 * Hilbert kernel 0.39 -> 0.44 ms, no gain.)
 */
#ifndef BPMX_FPSCAN_H
#define BPMX_FPSCAN_H

#include "bpmx_common.h"

namespace bpmx {

constexpr int FPS_NW = 16;                       /* waves of the scanning workgroup (1024 threads) */

/* wave wid's run of positions */
__device__ __forceinline__ void fp_scan_run(int64_t n, int wid, int64_t &w0, int64_t &w1) {
    const int64_t span = n > 2 ? n - 2 : 0;      /* positions 1 .. n-2 */
    const int64_t chunk = ((span + FPS_NW - 1) / FPS_NW + 63) & ~(int64_t)63;
    w0 = 1 + (int64_t)wid * chunk;
    w1 = w0 + chunk < n - 1 ? w0 + chunk : n - 1;
}

/* one wave: x(i) = the signed value at position i (0 <= i < n) */
template <class X>
__device__ __forceinline__ void fp_scan_wave(X x, int64_t n, int64_t w0, int64_t w1, int32_t *mp, int32_t *vp,
                                             double *mv, double *vv, int &cm, int &cv) {
    const int lane = lane_id();
    const unsigned long long lt = (1ull << lane) - 1ull;
    cm = cv = 0;
    /* one coalesced load per 64 positions, issued a block ahead; the left and
     * right neighbours come from the adjacent lanes (DPP wave shifts), the
     * block edges from the previous / next block's end lanes */
    double xc = w0 < w1 && w0 + lane < n ? x(w0 + lane) : 0.0;
    double xedge = w0 < w1 ? x(w0 - 1) : 0.0;    /* position b - 1 */
    for (int64_t b = w0; b < w1; b += 64) {
        const int64_t i = b + lane;
        const double xn = b + 64 + lane < n ? x(b + 64 + lane) : 0.0;
        const double xl = dpp_shr1_d(xc, xedge);
        const double xr1 = dpp_shl1_d(xc, __shfl(xn, 0));
        bool ism = false, isv = false;
        int32_t pk = 0;
        if (i < w1) {
            const double xi = xc;
            if (xl != xi) {
                int64_t ia = i + 1;
                double xr = xr1;
                if (xr == xi && ia < n - 1) {    /* plateau: walk it */
                    ia = i + 2;
                    while (ia < n - 1 && x(ia) == xi) ia++;
                    xr = x(ia);
                }
                if (xl < xi && xr < xi) { ism = true; pk = (int32_t)((i + ia - 1) >> 1); }
                else if (xl > xi && xr > xi) { isv = true; pk = (int32_t)((i + ia - 1) >> 1); }
            }
        }
        const unsigned long long bm = __ballot(ism), bv = __ballot(isv);
        if (ism) {
            const int64_t k = w0 - 1 + cm + __popcll(bm & lt);
            mp[k] = pk;
            mv[k] = xc;
        }
        if (isv) {
            const int64_t k = w0 - 1 + cv + __popcll(bv & lt);
            vp[k] = pk;
            vv[k] = xc;
        }
        cm += __popcll(bm);
        cv += __popcll(bv);
        xedge = __shfl(xc, 63);
        xc = xn;
    }
}

/* the record (PeakArgs scan_ok / scan_cnt): per recording ok[f] = +1 / -1
 * (lists made for x = +env / -env) or 0 (none: scan), zeroed at the start of
 * every run (k_init_out); per wave the two counts (maxima, valleys) */

}  // namespace bpmx

#endif
