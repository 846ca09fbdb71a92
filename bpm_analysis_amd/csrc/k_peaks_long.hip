/*
 * k_peaks_long.hip — find_peaks (bpm_analysis.py:1066-1070 troughs, :223-229
 * raw peaks: scipy.signal.find_peaks with height, distance, prominence) for
 * long recordings, spread over many workgroups per recording.
 *
 * Same formulation as k_find_peaks_lds (k_detect.hip): the local maxima
 * (scipy _local_maxima_1d, plateau midpoints) and the one valley between each
 * pair of consecutive maxima determine every prominence:
 *     left_min(j)  = min(vv[k* + 1 .. j])   k* = nearest maximum left of j higher than j (or -1)
 *     right_min(j) = min(vv[j + 1 .. k'])   k' = nearest maximum right of j higher than j (or M)
 * with vv[g] the valley of gap g (between maxima g-1 and g; vv[0] and vv[M]
 * include x[0] and x[n-1]).  Here the extrema live in global scratch:
 *   k_fpl_scan      one wave per 1024 positions: maxima and valley starts,
 *                   compacted per unit (coalesced env reads)
 *   k_fpl_place     per recording: unit offsets of the maxima, M, edge gaps
 *   k_fpl_fill      one wave per unit: dense maxima (position, value, state
 *                   after the height filter) and gap valleys
 *   k_fpl_distance  per recording: 32- and 1024-maxima block summaries, then
 *                   the distance rounds (k_find_peaks' rule: a candidate is
 *                   decided once every higher-priority neighbour within the
 *                   distance is)
 *   k_fpl_prom      one thread per kept maximum: walk the maxima outwards to
 *                   the nearest higher one, whole blocks of no-higher maxima
 *                   skipped through their summaries
 *   k_fpl_compact   per recording: ordered output, counts
 * Selected recordings: A.only[f] != 0 (k_find_peaks_lds hands over those
 * longer than A.lds_nmax or with more than FL_MC maxima).
 */
#include "bpmx_common.h"
#include "bpmx_kernels.h"

namespace bpmx {

namespace {
__device__ __forceinline__ bool fpl_selected(const PeakArgs &A, int f) {
    return f < A.n_files && A.active[f] && (!A.only || A.only[f]);
}
__device__ __forceinline__ int fpl_units(int64_t n) {
    return n > 2 ? (int)((n - 2 + FPL_U - 1) / FPL_U) : 0;
}
}  // namespace

constexpr int FPL_T = 256;   /* threads of the per-unit kernels: 4 units per workgroup */
constexpr int FPD_MMAX = 30720;   /* k_fpl_distance: candidates with LDS states and neighbour lists (150 KB) */

__global__ __launch_bounds__(FPL_T) void k_fpl_scan(PeakArgs A, FplArgs L) {
    const int f = blockIdx.y;
    if (!fpl_selected(A, f)) return;
    const int u = blockIdx.x * (FPL_T / 64) + wave_id(), lane = lane_id();
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    if (u >= fpl_units(n)) return;
    const double *e = A.env + d0;
    const double sg = A.sign;
    const int64_t w0 = 1 + (int64_t)u * FPL_U, w1 = min<int64_t>(n - 1, w0 + FPL_U);
    int32_t *mp_g = A.cand + d0 + (int64_t)u * FPL_U, *vp_g = A.vcand + d0 + (int64_t)u * FPL_U;
    int cm = 0, cv = 0;
    const unsigned long long lt = (1ull << lane) - 1ull;
    double xc = w0 + lane < n ? sg * e[w0 + lane] : 0.0;     /* as k_find_peaks_lds: one load a block ahead */
    double xedge = sg * e[w0 - 1];
    for (int64_t b = w0; b < w1; b += 64) {
        const int64_t i = b + lane;
        const double xn = b + 64 + lane < n ? sg * e[b + 64 + lane] : 0.0;
        const double xl = dpp_shr1_d(xc, xedge);
        const double xr1 = dpp_shl1_d(xc, __shfl(xn, 0));
        bool ism = false, isv = false;
        int32_t pk = 0;
        if (i < w1) {
            const double xi = xc;
            if (xl != xi) {
                int64_t ia = i + 1;
                double xr = xr1;
                if (xr == xi && ia < n - 1) {
                    ia = i + 2;
                    while (ia < n - 1 && sg * e[ia] == xi) ia++;
                    xr = sg * e[ia];
                }
                if (xl < xi && xr < xi) { ism = true; pk = (int32_t)((i + ia - 1) >> 1); }
                else if (xl > xi && xr > xi) { isv = true; pk = (int32_t)i; }
            }
        }
        const unsigned long long bm = __ballot(ism), bv = __ballot(isv);
        if (ism) mp_g[cm + __popcll(bm & lt)] = pk;
        if (isv) vp_g[cv + __popcll(bv & lt)] = pk;
        cm += __popcll(bm);
        cv += __popcll(bv);
        xedge = __shfl(xc, 63);
        xc = xn;
    }
    if (lane == 0) {
        int32_t *c = L.cnt + ((int64_t)f * L.nu + u) * 2;
        c[0] = cm;
        c[1] = cv;
    }
}

/* per recording: exclusive scan of the units' maxima counts (in place), M,
 * and the edge gaps' sample terms */
__global__ __launch_bounds__(FPL_T) void k_fpl_place(PeakArgs A, FplArgs L) {
    const int f = blockIdx.x;
    if (!fpl_selected(A, f)) return;
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    const int nu = fpl_units(n), tid = threadIdx.x;
    __shared__ int sh[FPL_T / 64 + 1];
    int32_t *c = L.cnt + (int64_t)f * L.nu * 2;
    int run = 0;
    for (int u0 = 0; u0 < nu; u0 += FPL_T) {
        const int u = u0 + tid;
        const int v = u < nu ? c[2 * u] : 0;
        int tot;
        const int off = block_scan_int<FPL_T>(v, sh, &tot);
        if (u < nu) c[2 * u] = run + off;
        run += tot;
    }
    if (tid == 0) {
        L.mtot[f] = run;
        if (L.dfail) L.dfail[f] = 0;
        double *vv = L.vv + d0 + f;
        if (n > 0) {
            vv[0] = A.sign * A.env[d0];
            if (run > 0) vv[run] = A.sign * A.env[d0 + n - 1];
        }
    }
}

__global__ __launch_bounds__(FPL_T) void k_fpl_fill(PeakArgs A, FplArgs L) {
    const int f = blockIdx.y;
    if (!fpl_selected(A, f)) return;
    const int u = blockIdx.x * (FPL_T / 64) + wave_id(), lane = lane_id();
    const int64_t d0 = A.doff[f], n = A.doff[f + 1] - d0;
    const int nu = fpl_units(n);
    if (u >= nu) return;
    const double *e = A.env + d0;
    const double *h = A.height ? A.height + d0 : nullptr;
    const double sg = A.sign;
    const int32_t *c = L.cnt + (int64_t)f * L.nu * 2;
    const int M = L.mtot[f];
    const int off = c[2 * u], cm = (u + 1 < nu ? c[2 * u + 2] : M) - off, cv = c[2 * u + 1];
    const int32_t *mp_u = A.cand + d0 + (int64_t)u * FPL_U, *vp_u = A.vcand + d0 + (int64_t)u * FPL_U;
    int32_t *mp = L.mp + d0;
    double *mh = L.mh + d0, *vv = L.vv + d0 + f;
    uint8_t *st = A.state + d0;
    const uint8_t open = A.distance > 1 ? ST_UNDECIDED : ST_KEPT;
    for (int t = lane; t < cm; t += 64) {
        const int32_t p = mp_u[t];
        const double xv = sg * e[p];
        mp[off + t] = p;
        mh[off + t] = xv;
        st[off + t] = (!h || h[p] <= xv) ? open : ST_HEIGHT;    /* height filter */
    }
    /* maxima and valleys alternate (k_find_peaks_lds): the unit's valley t
     * has t of its maxima before it, plus one when its first extremum is one */
    const int vfirst = (cm > 0 && (cv == 0 || mp_u[0] < vp_u[0])) ? 1 : 0;
    for (int t = lane; t < cv; t += 64) {
        const int32_t pv = vp_u[t];
        const int g = off + t + vfirst;
        const double val = sg * e[pv];
        if (g == 0 || g == M) vv[g] = fmin(vv[g], val);      /* edge gaps: at most one valley each */
        else vv[g] = val;
    }
}

__global__ __launch_bounds__(1024) void k_fpl_distance(PeakArgs A, FplArgs L) {
    const int f = blockIdx.x;
    if (!fpl_selected(A, f)) return;
    const int tid = threadIdx.x;
    const int64_t d0 = A.doff[f];
    const int M = L.mtot[f];
    const int32_t *mp = L.mp + d0;
    const double *mh = L.mh + d0, *vv = L.vv + d0 + f;
    uint8_t *st = A.state + d0;
    const double INF = __builtin_inf();
    __shared__ int s_flag;
    /* block summaries for the prominence walks */
    double *b32h = L.b32h + fpl_b32_off(d0, f), *b32l = L.b32l + fpl_b32_off(d0, f), *b32r = L.b32r + fpl_b32_off(d0, f);
    const int NB32 = (M + 31) >> 5, NB1K = (M + 1023) >> 10;
    for (int b = tid; b < NB32; b += 1024) {
        double hx = -INF, vl = INF, vr = INF;
        const int k1 = min(M, b * 32 + 32);
        for (int k = b * 32; k < k1; ++k) {
            hx = fmax(hx, mh[k]);
            vl = fmin(vl, vv[k + 1]);
            vr = fmin(vr, vv[k]);
        }
        b32h[b] = hx;
        b32l[b] = vl;
        b32r[b] = vr;
    }
    __syncthreads();
    {
        double *bh = L.b1kh + fpl_b1k_off(d0, f), *bl = L.b1kl + fpl_b1k_off(d0, f), *br = L.b1kr + fpl_b1k_off(d0, f);
        for (int B = tid; B < NB1K; B += 1024) {
            double hx = -INF, vl = INF, vr = INF;
            const int b1 = min(NB32, B * 32 + 32);
            for (int b = B * 32; b < b1; ++b) {
                hx = fmax(hx, b32h[b]);
                vl = fmin(vl, b32l[b]);
                vr = fmin(vr, b32r[b]);
            }
            bh[B] = hx;
            bl[B] = vl;
            br[B] = vr;
        }
    }
    const int64_t dist = A.distance;
    if (dist <= 1) return;
    if (L.dchunk && !L.dfail[f]) return;                     /* k_fpl_dist_ch decided every chunk */
    if (M <= FPD_MMAX) {
        /* States in LDS and each candidate's higher-priority neighbours listed
         * once (up to four, as signed index offsets packed in a register; more
         * or farther: a full scan of mp / mh each round).  Rounds run
         * wave-locally (a candidate's neighbours are mostly the adjacent lanes)
         * until the wave makes no progress; one workgroup barrier then lets
         * decisions cross wave boundaries.  A decision needs a KEPT neighbour
         * (final) or no UNDECIDED one, so unsynchronised reads only delay it. */
        __shared__ uint8_t s_st[FPD_MMAX];
        __shared__ uint32_t s_nb[FPD_MMAX];
        for (int j = tid; j < M; j += 1024) {
            s_st[j] = st[j];
            const int64_t pj = mp[j];
            const double vj = mh[j];
            uint32_t w = 0u;
            int c = 0;
            bool over = false;
            auto add = [&](int k) {
                const int o = k - j;
                if (c < 4 && o >= -63 && o <= 63) w |= (uint32_t)(o & 127) << (7 * c);
                else over = true;
                ++c;
            };
            for (int k = j - 1; k >= 0 && pj - mp[k] < dist; --k)
                if (mh[k] > vj) add(k);
            for (int k = j + 1; k < M && mp[k] - pj < dist; ++k)
                if (mh[k] >= vj) add(k);
            s_nb[j] = w | (uint32_t)(over ? 7 : c) << 28;
        }
        __syncthreads();
        for (int gi = 0; gi <= M; ++gi) {
            bool pending = false;
            for (int lr = 0; lr <= M; ++lr) {
                bool progress = false;
                pending = false;
                for (int j = tid; j < M; j += 1024) {
                    if (ld_state(&s_st[j]) != ST_UNDECIDED) continue;
                    bool killed = false, blocked = false;
                    const uint32_t w = s_nb[j];
                    const int c = (int)(w >> 28);
                    if (c != 7) {
                        for (int q = 0; q < c; ++q) {
                            const int o = (int)((w >> (7 * q)) & 127u);
                            const int k = j + (o >= 64 ? o - 128 : o);
                            const uint8_t sk = ld_state(&s_st[k]);
                            killed |= sk == ST_KEPT;
                            blocked |= sk == ST_UNDECIDED;
                        }
                    } else {
                        const int64_t pj = mp[j];
                        const double vj = mh[j];
                        for (int k = j - 1; k >= 0 && pj - mp[k] < dist && !killed; --k)
                            if (mh[k] > vj) {
                                const uint8_t sk = ld_state(&s_st[k]);
                                killed = sk == ST_KEPT;
                                blocked |= sk == ST_UNDECIDED;
                            }
                        for (int k = j + 1; k < M && mp[k] - pj < dist && !killed; ++k)
                            if (mh[k] >= vj) {
                                const uint8_t sk = ld_state(&s_st[k]);
                                killed = sk == ST_KEPT;
                                blocked |= sk == ST_UNDECIDED;
                            }
                    }
                    if (killed) { st_state(&s_st[j], ST_REMOVED); progress = true; }
                    else if (!blocked) { st_state(&s_st[j], ST_KEPT); progress = true; }
                    else pending = true;
                }
                if (!__ballot(progress)) break;                  /* wave-uniform */
            }
            if (!__syncthreads_or(pending)) break;
        }
        for (int j = tid; j < M; j += 1024) st[j] = s_st[j];
        return;
    }
    /* every round decides at least the highest-priority undecided candidate */
    for (int round = 0; round <= M; ++round) {
        if (tid == 0) s_flag = 0;
        __syncthreads();
        bool pending = false;
        for (int j = tid; j < M; j += 1024) {
            if (ld_state(&st[j]) != ST_UNDECIDED) continue;
            const int64_t pj = mp[j];
            const double vj = mh[j];
            bool killed = false, blocked = false;
            for (int k = j - 1; k >= 0 && pj - mp[k] < dist; --k) {
                if (mh[k] > vj) {                            /* earlier index wins only when strictly higher */
                    const uint8_t s = ld_state(&st[k]);
                    if (s == ST_KEPT) { killed = true; break; }
                    if (s == ST_UNDECIDED) blocked = true;
                }
            }
            if (!killed) {
                for (int k = j + 1; k < M && mp[k] - pj < dist; ++k) {
                    if (mh[k] >= vj) {                       /* later index wins ties (stable argsort order) */
                        const uint8_t s = ld_state(&st[k]);
                        if (s == ST_KEPT) { killed = true; break; }
                        if (s == ST_UNDECIDED) blocked = true;
                    }
                }
            }
            if (killed) st_state(&st[j], ST_REMOVED);
            else if (!blocked) st_state(&st[j], ST_KEPT);
            else pending = true;
        }
        if (pending) s_flag = 1;
        __syncthreads();
        const int again = s_flag;
        __syncthreads();
        if (!again) break;
    }
}


/* One workgroup per chunk of a long recording's maxima: nominal [c S, c S + S),
 * taken from its first component start (a maximum >= distance after the
 * previous one, or the first) to the first component start at or after the
 * nominal end.  Components never straddle such a cut, so every chunk decides
 * its own exactly as the whole-recording rounds would; a component reaching
 * more than FPC_H maxima past the nominal end sets dfail and k_fpl_distance
 * runs the recording's rounds (from whatever other chunks have decided: their
 * decisions are final).  Rounds as k_find_peaks_lds: neighbour lists of up to
 * eight 8-bit offsets, every listed state read before the decisions, rounds
 * wave-locally, one barrier to cross waves. */
__global__ __launch_bounds__(FPC_T) void k_fpl_dist_ch(PeakArgs A, FplArgs L) {
    const int f = blockIdx.y;
    if (!fpl_selected(A, f)) return;
    const int64_t dist = A.distance;
    if (dist <= 1) return;
    const int M = L.mtot[f];
    const int n0 = blockIdx.x * FPC_S;
    if (n0 >= M) return;
    const int tid = threadIdx.x;
    const int64_t d0 = A.doff[f];
    const int32_t *mp = L.mp + d0;
    const double *mh = L.mh + d0;
    uint8_t *st = A.state + d0;
    __shared__ int s_js, s_je;
    __shared__ int32_t s_mp[FPC_S + FPC_H];
    __shared__ double s_mh[FPC_S + FPC_H];
    __shared__ uint8_t s_st[FPC_S + FPC_H];
    const int n1 = min(M, n0 + FPC_S), n2 = min(M, n1 + FPC_H);
    if (tid == 0) { s_js = n1; s_je = n1 < M ? INT_MAX : M; }
    __syncthreads();
    auto is_start = [&](int j) { return j == 0 || (int64_t)mp[j] - (int64_t)mp[j - 1] >= dist; };
    for (int j = n0 + tid; j < n1; j += FPC_T)
        if (is_start(j)) atomicMin(&s_js, j);
    if (n1 < M)
        for (int j = n1 + tid; j < n2; j += FPC_T)
            if (is_start(j)) atomicMin(&s_je, j);
    __syncthreads();
    const int js = s_js, je = s_je;
    if (js >= n1) return;                                    /* no component starts here */
    if (je == INT_MAX) {                                     /* a component runs past the halo */
        if (tid == 0) __hip_atomic_store(&L.dfail[f], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const int m = je - js;
    for (int t = tid; t < m; t += FPC_T) {
        s_mp[t] = mp[js + t];
        s_mh[t] = mh[js + t];
        s_st[t] = st[js + t];
    }
    __syncthreads();
    constexpr int NBX = 8;
    uint32_t nb[FPC_R][2];
    int nbc[FPC_R];
    uint32_t und = 0u;
#pragma unroll
    for (int r = 0; r < FPC_R; ++r) {
        const int j = tid + r * FPC_T;
        nb[r][0] = nb[r][1] = 0u;
        nbc[r] = 0;
        if (j >= m || s_st[j] != ST_UNDECIDED) continue;
        und |= 1u << r;
        const int64_t pj = s_mp[j];
        const double vj = s_mh[j];
        int c = 0;
        auto add = [&](int k) {
            const int o = k - j;
            if (o < -128 || o > 127) c = NBX;
            if (c < NBX) nb[r][c >> 2] |= ((uint32_t)o & 0xFFu) << (8 * (c & 3));
            ++c;
        };
        for (int k = j - 1; k >= 0 && pj - s_mp[k] < dist; --k)
            if (s_mh[k] > vj && s_st[k] == ST_UNDECIDED) add(k);       /* earlier index: strictly higher */
        for (int k = j + 1; k < m && s_mp[k] - pj < dist; ++k)
            if (s_mh[k] >= vj && s_st[k] == ST_UNDECIDED) add(k);      /* later index wins ties */
        nbc[r] = c <= NBX ? c : -1;
    }
    for (int gi = 0; gi <= m; ++gi) {
        for (int lr = 0; lr <= m; ++lr) {
            bool progress = false;
            uint32_t kill = 0u, block = 0u;
            int nbv[FPC_R];                                  /* opaque per round: no hoisted (r, q) masks (k_find_peaks_lds) */
#pragma unroll
            for (int r = 0; r < FPC_R; ++r) {
                nbv[r] = nbc[r];
                asm volatile("" : "+v"(nbv[r]));
            }
#pragma unroll
            for (int r = 0; r < FPC_R; ++r) {
                if (!((und >> r) & 1u) || nbv[r] < 0) continue;
                const int j = tid + r * FPC_T;
#pragma unroll
                for (int q = 0; q < NBX; ++q) {
                    if (q < nbv[r]) {
                        const int k = j + (int)(int8_t)((nb[r][q >> 2] >> (8 * (q & 3))) & 0xFFu);
                        const uint8_t sk = ld_state(&s_st[k]);
                        kill |= (sk == ST_KEPT ? 1u : 0u) << r;
                        block |= (sk == ST_UNDECIDED ? 1u : 0u) << r;
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < FPC_R; ++r) {
                if (!((und >> r) & 1u)) continue;
                const int j = tid + r * FPC_T;
                bool killed = (kill >> r) & 1u, blocked = (block >> r) & 1u;
                if (nbc[r] < 0) {
                    const int64_t pj = s_mp[j];
                    const double vj = s_mh[j];
                    for (int k = j - 1; k >= 0 && pj - s_mp[k] < dist; --k)
                        if (s_mh[k] > vj) {
                            const uint8_t sk = ld_state(&s_st[k]);
                            if (sk == ST_KEPT) { killed = true; break; }
                            if (sk == ST_UNDECIDED) blocked = true;
                        }
                    if (!killed)
                        for (int k = j + 1; k < m && s_mp[k] - pj < dist; ++k)
                            if (s_mh[k] >= vj) {
                                const uint8_t sk = ld_state(&s_st[k]);
                                if (sk == ST_KEPT) { killed = true; break; }
                                if (sk == ST_UNDECIDED) blocked = true;
                            }
                }
                if (killed || !blocked) {
                    st_state(&s_st[j], killed ? ST_REMOVED : ST_KEPT);
                    und &= ~(1u << r);
                    progress = true;
                }
            }
            if (!__ballot(progress)) break;
        }
        if (!__syncthreads_or(und != 0u)) break;
    }
    for (int t = tid; t < m; t += FPC_T) st[js + t] = s_st[t];
}

__global__ __launch_bounds__(FPL_T) void k_fpl_prom(PeakArgs A, FplArgs L) {
    const int f = blockIdx.y;
    if (!fpl_selected(A, f)) return;
    const int j = blockIdx.x * FPL_T + threadIdx.x;
    const int M = L.mtot[f];
    if (j >= M) return;
    const int64_t d0 = A.doff[f];
    uint8_t *st = A.state + d0;
    const uint8_t sj = st[j];
    if (sj == ST_REMOVED && A.distance > 1) {
        /* removed by the distance filter: a decisive tie (include/bpmx.h
         * BPMX_F_*_TIE) unless a strictly higher candidate the filter kept lies
         * within distance (kept states are odd whatever the prominence did) */
        const int32_t *mp = L.mp + d0;
        const double *mh = L.mh + d0;
        const int64_t pj = mp[j], dist = A.distance;
        const double vj = mh[j];
        bool dom = false;
        for (int k = j - 1; !dom && k >= 0 && pj - mp[k] < dist; --k)
            dom = mh[k] > vj && st_kept_by_distance(__hip_atomic_load(&st[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        for (int k = j + 1; !dom && k < M && mp[k] - pj < dist; ++k)
            dom = mh[k] > vj && st_kept_by_distance(__hip_atomic_load(&st[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (!dom && A.flags) atomicOr(&A.flags[f], A.tie_bit);
        return;
    }
    if (sj != ST_KEPT) return;
    const double *mh = L.mh + d0, *vv = L.vv + d0 + f;
    const int64_t o32 = fpl_b32_off(d0, f), o1k = fpl_b1k_off(d0, f);
    const double *b32h = L.b32h + o32, *b32l = L.b32l + o32, *b32r = L.b32r + o32;
    const double *bkh = L.b1kh + o1k, *bkl = L.b1kl + o1k, *bkr = L.b1kr + o1k;
    const double INF = __builtin_inf();
    const double hj = mh[j];
    double lmin = INF, rmin = INF;
    /* both walks step together and a step reads every candidate (the 1024-
     * and 32-maximum block summaries, the gap valley, the maximum) before
     * choosing: one memory round trip per step of both sides */
    int kl = j - 1, kr = j + 1;
    bool dl = false, dr = false;
    while (!(dl && dr)) {
        if (!dl) {
            if (kl < 0) {
                lmin = fmin(lmin, vv[0]);
                dl = true;
            } else {
                const double h2 = bkh[kl >> 10], v2 = bkl[kl >> 10], h1 = b32h[kl >> 5], v1 = b32l[kl >> 5];
                const double v0 = vv[kl + 1], m0 = mh[kl];
                const bool c2 = (kl & 1023) == 1023 && h2 <= hj;
                const bool c1 = !c2 && (kl & 31) == 31 && h1 <= hj;
                lmin = fmin(lmin, c2 ? v2 : (c1 ? v1 : v0));
                if (!(c2 || c1) && m0 > hj) dl = true;
                else kl -= c2 ? 1024 : (c1 ? 32 : 1);
            }
        }
        if (!dr) {
            if (kr >= M) {
                rmin = fmin(rmin, vv[M]);
                dr = true;
            } else {
                const double h2 = bkh[kr >> 10], v2 = bkr[kr >> 10], h1 = b32h[kr >> 5], v1 = b32r[kr >> 5];
                const double v0 = vv[kr], m0 = mh[kr];
                const bool c2 = (kr & 1023) == 0 && kr + 1023 < M && h2 <= hj;
                const bool c1 = !c2 && (kr & 31) == 0 && kr + 31 < M && h1 <= hj;
                rmin = fmin(rmin, c2 ? v2 : (c1 ? v1 : v0));
                if (!(c2 || c1) && m0 > hj) dr = true;
                else kr += c2 ? 1024 : (c1 ? 32 : 1);
            }
        }
    }
    const double prom = hj - fmax(lmin, rmin);
    const double thr = A.qv[(int64_t)f * Q_SLOTS + A.qslot];
    __hip_atomic_store(&st[j], (uint8_t)(thr <= prom ? ST_FINAL : ST_PREMOVED), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(1024) void k_fpl_compact(PeakArgs A, FplArgs L) {
    const int f = blockIdx.x;
    if (!fpl_selected(A, f)) return;
    const int tid = threadIdx.x;
    const int64_t d0 = A.doff[f];
    const int M = L.mtot[f];
    const int32_t *mp = L.mp + d0;
    const uint8_t *st = A.state + d0;
    __shared__ int sh[1024 / 64 + 1];
    int64_t *out = A.out + d0;
    int w = 0;
    for (int q0 = 0; q0 < M; q0 += 1024) {
        const int j = q0 + tid;
        const bool keep = j < M && st[j] == ST_FINAL;
        int tot;
        const int off = block_scan_flag<1024>(keep, sh, &tot);
        if (keep) {
            out[w + off] = mp[j];
            if (A.outv) A.outv[d0 + w + off] = A.sign * L.mh[d0 + j];
        }
        w += tot;
    }
    if (tid == 0) {
        A.nout[f] = w;
        if (A.run_out) A.run_out[f] = w >= A.run_min ? 1 : 0;
    }
}

}  // namespace bpmx
