/*
 * bpmx_api.hip — host side of the C ABI (include/bpmx.h): context, scratch,
 * stage sequencing, synthetic input, per-kernel event timing.
 *
 * Stage order follows analyze_wav_file (bpm_analysis.py:1731-1732) and the
 * classifier's raw-peak call (:89 -> :223-229):
 *   ENVELOPE  k_envelope_ref | native kernels (k_envelope_native.hip)
 *   FLOOR     k_block_stats, k_quantile, k_find_peaks(-env), k_interp,
 *             k_rolling_quantile (draft), k_sanitize, k_interp,
 *             k_rolling_quantile (final), k_floor_final
 *   PEAKS     k_find_peaks(env, height=floor)
 * Everything is enqueued on one stream; no host synchronisation inside a run
 * except the (cached) upload of the batch geometry.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "bpmx_common.h"
#include "bpmx_kernels.h"
#include "bpmx_ctx.h"
#include "bpmx_native.h"
#include "bpmx_fpscan.h"
#include "bpmx_synth.h"

#include <rocprofiler-sdk-roctx/roctx.h>

using namespace bpmx;

namespace bpmx {
thread_local std::string g_err;
int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
}  // namespace bpmx

namespace {

/* Per-stage roctx ranges (SURVEY.md §5 tracing): a run's ENVELOPE, FLOOR and
 * PEAKS launches are enqueued inside "bpmx:<stage>" ranges, so a profile taken
 * with rocprofv3 --marker-trace --kernel-trace groups each kernel under its
 * stage (the reference itself only logs a total time, bpm_analysis.py:1727,
 * :1767-1768).  The ranges cover host-side enqueueing; the kernels they
 * correlate with run asynchronously after. */
struct StageRange {
    explicit StageRange(const char *name) { roctxRangePushA(name); }
    ~StageRange() { roctxRangePop(); }
    StageRange(const StageRange &) = delete;
    StageRange &operator=(const StageRange &) = delete;
};

/* per-run output init from the cached device geometry (no pageable H2D copy
 * on the run path): flags = TOO_SHORT for inactive recordings, counts 0 */
__global__ __launch_bounds__(256) void k_init_out(InitOutArgs I) {
    const int f = blockIdx.x * 256 + threadIdx.x;
    if (f < I.n_files) init_out_one(I, f);
}

/* recordings with >= 5 raw troughs reach the rolling quantile: with a noise
 * window below min_periods pandas raises there (bpm_analysis.py:1085) */
__global__ __launch_bounds__(256) void k_flag_window(int n_files, const int32_t *run, int32_t *flags) {
    const int f = blockIdx.x * 256 + threadIdx.x;
    if (f < n_files && run[f]) flags[f] |= BPMX_F_BAD_WINDOW;
}

__global__ __launch_bounds__(64) void k_synth_beats(uint64_t seed0, int n_files, const int64_t *foff,
                                                    const int64_t *boff, int32_t fs, int64_t *s1, int64_t *s2,
                                                    int32_t *nb) {
    const int f = blockIdx.x * 64 + threadIdx.x;
    if (f >= n_files) return;
    const int cap = (int)(boff[f + 1] - boff[f]);
    nb[f] = bpmx_synth_beats(seed0 + (uint64_t)f, foff[f + 1] - foff[f], fs, s1 + boff[f], s2 + boff[f], cap);
}

__global__ __launch_bounds__(256) void k_synth_pcm(uint64_t seed0, int n_files, const int64_t *foff,
                                                   const int64_t *boff, int32_t fs, int channels,
                                                   const int64_t *s1, const int64_t *s2, const int32_t *nb,
                                                   int16_t *pcm) {
    const int f = blockIdx.y;
    const int64_t n = foff[f + 1] - foff[f];
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        for (int c = 0; c < channels; ++c)
            pcm[(foff[f] + i) * channels + c] =
                bpmx_synth_sample(seed0 + (uint64_t)f, c, i, fs, s1 + boff[f], s2 + boff[f], nb[f]);
}

int beats_cap(int64_t n_frames, int32_t fs) {
    int64_t q = fs / 4 > 0 ? fs / 4 : 1;
    return (int)(n_frames / q) + 16;
}

}  // namespace

extern "C" {

int bpmx_abi_version(void) { return BPMX_ABI_VERSION; }

const char *bpmx_last_error(void) { return g_err.c_str(); }

int bpmx_create(int device, bpmx_ctx **out) {
    if (!out) return fail(BPMX_E_ARG, "out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(BPMX_E_NODEV, "no HIP device visible");
    if (device < 0 || device >= n) return fail(BPMX_E_ARG, "device index out of range");
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(BPMX_E_NODEV, std::string("libbpmx is built for gfx950, device is ") + prop.gcnArchName);
    bpmx_ctx *c = new bpmx_ctx();
    c->device = device;
    *out = c;
    return BPMX_OK;
}

void bpmx_destroy(bpmx_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    for (auto &kv : ctx->bufs)
        if (kv.second.first) (void)hipFree(kv.second.first);
    for (auto &r : ctx->recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
    for (auto e : ctx->pool) (void)hipEventDestroy(e);
    for (int i = 0; i < bpmx_ctx::NSIDE && !ctx->root; ++i) {   /* a pipeline sub-context borrows its root's */
        if (ctx->side[i]) (void)hipStreamDestroy(ctx->side[i]);
        if (ctx->side_join[i]) (void)hipEventDestroy(ctx->side_join[i]);
    }
    if (ctx->side_fork && !ctx->root) (void)hipEventDestroy(ctx->side_fork);
    if (ctx->stats_ev) (void)hipEventDestroy(ctx->stats_ev);
    for (bpmx_ctx *c : ctx->pipe_sub) bpmx_destroy(c);
    bpmx::longfft_free(ctx);
    if (ctx->pipe_env) (void)hipStreamDestroy(ctx->pipe_env);
    if (ctx->pipe_det) (void)hipStreamDestroy(ctx->pipe_det);
    for (auto e : ctx->pipe_ev) (void)hipEventDestroy(e);
    delete ctx;
}

int64_t bpmx_decimated_length(int64_t n_frames, int32_t ds) {
    if (ds < 1) ds = 1;
    return n_frames <= 0 ? 0 : (n_frames + ds - 1) / ds;
}

void bpmx_synth_host(uint64_t seed, int64_t n_frames, int32_t fs, int32_t channels, int16_t *out) {
    const int cap = beats_cap(n_frames, fs);
    std::vector<int64_t> s1(cap), s2(cap);
    const int nb = bpmx_synth_beats(seed, n_frames, fs, s1.data(), s2.data(), cap);
    for (int64_t i = 0; i < n_frames; ++i)
        for (int c = 0; c < channels; ++c)
            out[i * channels + c] = bpmx_synth_sample(seed, c, i, fs, s1.data(), s2.data(), nb);
}

int bpmx_synth(bpmx_ctx *ctx, uint64_t seed0, int32_t n_files, const int64_t *frame_offsets, int32_t fs,
               int32_t channels, int16_t *pcm, void *stream) {
    if (!ctx || !frame_offsets || !pcm || n_files < 1 || fs < 4 || channels < 1)
        return fail(BPMX_E_ARG, "bpmx_synth: bad argument");
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    std::vector<int64_t> geo(2 * (n_files + 1));
    int64_t acc = 0, maxn = 0;
    for (int f = 0; f <= n_files; ++f) {
        geo[f] = frame_offsets[f] - frame_offsets[0];
        if (f < n_files) {
            int64_t n = frame_offsets[f + 1] - frame_offsets[f];
            if (n < 0) return fail(BPMX_E_ARG, "bpmx_synth: frame offsets must be non-decreasing");
            geo[n_files + 1 + f] = acc;
            acc += beats_cap(n, fs);
            maxn = std::max(maxn, n);
        }
    }
    geo[n_files + 1 + n_files] = acc;
    int rc = BPMX_OK;
    int64_t *dgeo = (int64_t *)ctx->buf("synth_geo", geo.size() * 8, &rc);
    int64_t *s1 = (int64_t *)ctx->buf("synth_s1", (size_t)acc * 8, &rc);
    int64_t *s2 = (int64_t *)ctx->buf("synth_s2", (size_t)acc * 8, &rc);
    int32_t *nb = (int32_t *)ctx->buf("synth_nb", (size_t)n_files * 4, &rc);
    if (rc != BPMX_OK) return rc;
    HIP_TRY(hipMemcpyAsync(dgeo, geo.data(), geo.size() * 8, hipMemcpyHostToDevice, s));
    const int64_t *foff = dgeo, *boff = dgeo + n_files + 1;
    int16_t *base = pcm + frame_offsets[0] * channels;
    LAUNCH(ctx, s, "k_synth_beats", k_synth_beats, dim3((n_files + 63) / 64), dim3(64), 0, s, seed0, n_files, foff,
           boff, fs, s1, s2, nb);
    int gx = (int)std::min<int64_t>((maxn + 255) / 256, 512);
    LAUNCH(ctx, s, "k_synth_pcm", k_synth_pcm, dim3(std::max(gx, 1), n_files), dim3(256), 0, s, seed0, n_files,
           foff, boff, fs, channels, s1, s2, nb, base);
    return BPMX_OK;
}

int bpmx_profile(bpmx_ctx *ctx, int on) {
    if (!ctx) return fail(BPMX_E_ARG, "ctx is NULL");
    ctx->prof = on != 0;
    if (on) {
        ctx->totals.clear();
        /* events created now, not inside the profiled launches (hipEventCreate
         * on the launch path leaves the GPU waiting on the host) */
        HIP_TRY(hipSetDevice(ctx->device));
        while (ctx->pool.size() < 4096) {
            hipEvent_t e;
            HIP_TRY(hipEventCreate(&e));
            ctx->pool.push_back(e);
        }
    }
    return BPMX_OK;
}

int bpmx_profile_only(bpmx_ctx *ctx, const char *label) {
    if (!ctx) return fail(BPMX_E_ARG, "ctx is NULL");
    ctx->prof_only = label ? label : "";
    return BPMX_OK;
}

int bpmx_profile_read(bpmx_ctx *ctx, char *buf, int len) {
    if (!ctx) return fail(BPMX_E_ARG, "ctx is NULL");
    HIP_TRY(hipSetDevice(ctx->device));
    for (auto &r : ctx->recs) {
        HIP_TRY(hipEventSynchronize(r.b));
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, r.a, r.b));
        auto &t = ctx->totals[r.name];
        t.first += 1;
        t.second += ms;
        ctx->pool.push_back(r.a);
        ctx->pool.push_back(r.b);
    }
    ctx->recs.clear();
    std::string s;
    char line[256];
    for (auto &kv : ctx->totals) {
        std::snprintf(line, sizeof line, "%s %ld %.6f\n", kv.first.c_str(), kv.second.first, kv.second.second);
        s += line;
    }
    if (buf && len > 0) {
        std::strncpy(buf, s.c_str(), (size_t)len - 1);
        buf[len - 1] = 0;
    }
    return (int)s.size();
}

int bpmx_stats(bpmx_ctx *ctx, int64_t *out, int n) {
    if (!ctx || !out || n < 0) return fail(BPMX_E_ARG, "NULL argument");
    HIP_TRY(hipSetDevice(ctx->device));
    int64_t h[BPMX_NSTATS] = {};
    auto it = ctx->bufs.find("stats");
    if (it != ctx->bufs.end()) {
        if (ctx->stats_ev) HIP_TRY(hipEventSynchronize(ctx->stats_ev));
        HIP_TRY(hipMemcpy(h, it->second.first, sizeof h, hipMemcpyDeviceToHost));
    }
    for (int i = 0; i < n; ++i) out[i] = i < BPMX_NSTATS ? h[i] : 0;
    return BPMX_NSTATS;
}

/* the rolling-quantile kernels' dynamic-LDS limit, raised once per device
 * (the attribute applies to the current device) to the largest layout they
 * take, not per launch on the run path */
static void wm_lds_attr(int device) {
    static std::mutex mu;
    static std::vector<char> done;
    std::lock_guard<std::mutex> lk(mu);
    if (device < 0) return;
    if ((int)done.size() <= device) done.resize((size_t)device + 1, 0);
    if (done[(size_t)device]) return;
    const int mx = (int)wm_layout(WM_MMAX, false).total;
    (void)hipFuncSetAttribute((const void *)k_rollq_wm_t<true>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    (void)hipFuncSetAttribute((const void *)k_rollq_wm_t<false>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    (void)hipFuncSetAttribute((const void *)k_floor_wm, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    done[(size_t)device] = 1;
}

static int run_impl(bpmx_ctx *ctx, const bpmx_params *P, const bpmx_batch *B, const bpmx_out *O, void *stream,
                    bool env_active, const bpmx_peak_order *ord = nullptr) {
    if (!ctx || !P || !B || !O) return fail(BPMX_E_ARG, "NULL argument");
    const int F = B->n_files;
    if (F < 1 || !B->frame_offsets) return fail(BPMX_E_ARG, "empty batch");
    if (P->mode != BPMX_MODE_REFERENCE && P->mode != BPMX_MODE_NATIVE) return fail(BPMX_E_ARG, "bad mode");
    if (P->dtype < BPMX_DT_U8 || P->dtype > BPMX_DT_F64) return fail(BPMX_E_ARG, "bad dtype");
    if (P->channels < 1 || P->ds < 1 || P->sr < 1) return fail(BPMX_E_ARG, "bad channels/ds/sr");
    const int st = P->stages;
    if (st <= 0 || st > BPMX_STAGE_ALL) return fail(BPMX_E_ARG, "bad stage mask");
    const bool do_env = st & BPMX_STAGE_ENVELOPE, do_floor = st & BPMX_STAGE_FLOOR, do_peaks = st & BPMX_STAGE_PEAKS;
    if (do_env && !B->pcm) return fail(BPMX_E_ARG, "ENVELOPE stage needs pcm");
    if (!O->env || !O->n_troughs || !O->n_peaks || !O->flags) return fail(BPMX_E_ARG, "missing output arrays");
    if ((do_floor || do_peaks) && !O->floor) return fail(BPMX_E_ARG, "floor array required");
    if (do_floor && !O->troughs) return fail(BPMX_E_ARG, "troughs array required");
    if (do_peaks && !O->peaks) return fail(BPMX_E_ARG, "peaks array required");
    if ((do_floor || do_peaks) && P->distance < 1) return fail(BPMX_E_ARG, "`distance` must be greater or equal to 1");
    if (do_floor && P->min_periods < 1) return fail(BPMX_E_ARG, "min_periods must be >= 1");
    /* noise window < min_periods: pandas' rolling() raises ValueError, but only
     * for recordings that reach it (>= 5 troughs, :1073-1085); those get
     * BPMX_F_BAD_WINDOW and the rest of the batch runs normally */
    const bool bad_window = do_floor && P->noise_window < P->min_periods;
    if (do_env && P->env_window < 1) return fail(BPMX_E_ARG, "envelope window must be >= 1");
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    int64_t *d_stats = nullptr;
    if (P->options & BPMX_OPT_STATS) {
        int src = BPMX_OK;
        d_stats = (int64_t *)ctx->pr()->buf("stats", BPMX_NSTATS * 8, &src);
        if (src != BPMX_OK) return src;
        if (!ctx->root)                                /* a pipelined run zeroes them once */
            HIP_TRY(hipMemsetAsync(d_stats, 0, BPMX_NSTATS * 8, s));
    }

    /* ---- geometry ---- */
    std::vector<int64_t> foff(F + 1), doff(F + 1), boff(F + 1);
    std::vector<int32_t> active(F);
    int64_t maxnd = 0;
    foff[0] = 0; doff[0] = 0; boff[0] = 0;
    for (int f = 0; f < F; ++f) {
        const int64_t n = B->frame_offsets[f + 1] - B->frame_offsets[f];
        if (n < 0) return fail(BPMX_E_ARG, "frame offsets must be non-decreasing");
        const int64_t nd = bpmx_decimated_length(n, P->ds);
        foff[f + 1] = foff[f] + n;
        doff[f + 1] = doff[f] + nd;
        boff[f + 1] = boff[f] + (nd + 63) / 64;
        maxnd = std::max(maxnd, nd);
        const bool ok = (do_env || env_active) ? nd > 15 : nd >= 1;
        active[f] = ok ? 1 : 0;
        if (nd >= (int64_t)INT_MAX / 2) return fail(BPMX_E_LIMIT, "recording too long");
    }
    const int64_t sumnd = doff[F], sumb = boff[F];
    if (sumnd == 0) return fail(BPMX_E_ARG, "empty recordings");
    /* int16 PCM whose base is not 16-byte aligned but sits a whole number of
     * frames past a 16-byte boundary (e.g. a pipelined chunk or any sub-range
     * of an aligned buffer): the kernels read from that boundary and every
     * recording's frame offset moves up by the difference, so the matrix-core
     * block kernel (16-byte aligned base) serves it.  Its projections are exact
     * integer sums and its tiles start at each recording's own first block, so
     * a recording's envelope does not depend on where it lies in the buffer
     * (include/bpmx.h, bpmx_set_pipeline).  The boundary is in the same page as
     * the base, and the kernels drop what lies before a recording's start. */
    bpmx_batch b_shift;
    if (do_env && P->dtype == BPMX_DT_I16 && B->pcm) {
        const uintptr_t mis = (uintptr_t)B->pcm & 15;
        const uintptr_t fb = (uintptr_t)2 * (uintptr_t)P->channels;
        if (mis != 0 && mis % fb == 0) {
            const int64_t sh = (int64_t)(mis / fb);
            for (int f = 0; f <= F; ++f) foff[f] += sh;
            b_shift = *B;
            b_shift.pcm = (const void *)((const char *)B->pcm - mis);
            B = &b_shift;
        }
    }

    int rc = BPMX_OK;
    std::vector<int64_t> geo;
    geo.reserve(3 * (F + 1));
    geo.insert(geo.end(), foff.begin(), foff.end());
    geo.insert(geo.end(), doff.begin(), doff.end());
    geo.insert(geo.end(), boff.begin(), boff.end());
    bool g1 = false, g2 = false;
    int64_t *dgeo = (int64_t *)ctx->buf("geo", geo.size() * 8, &rc, &g1);
    int32_t *di = (int32_t *)ctx->buf("geo_i", (size_t)F * 4 * 8, &rc, &g2);
    if (rc != BPMX_OK) return rc;
    if (g1 || g2) ctx->g_key.clear();
    std::vector<int64_t> key = geo;
    key.push_back(F);
    key.push_back(do_env);
    if (key != ctx->g_key) {
        HIP_TRY(hipMemcpyAsync(dgeo, geo.data(), geo.size() * 8, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(di, active.data(), (size_t)F * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(hipStreamSynchronize(s));
        ctx->g_key = key;
    }
    const int64_t *d_foff = dgeo, *d_doff = dgeo + F + 1, *d_boff = dgeo + 2 * (F + 1);
    const int32_t *d_active = di;
    int32_t *d_run1 = di + F, *d_run2 = di + 2 * F, *d_an1 = di + 3 * F, *d_an2 = di + 4 * F;
    /* raw-trough counts go straight into the caller's array when it asks for them */
    int32_t *d_nraw = (do_floor && O->n_raw_troughs) ? (int32_t *)O->n_raw_troughs : di + 5 * F;

    /* the draft bracket's per-recording masks and counters (FLOOR below) are
     * zeroed here, with the outputs, instead of by two memset launches */
    const bool bounds = do_floor && !(P->options & BPMX_OPT_DRAFT_FULL);
    int32_t *draft_masks = nullptr, *draft_vfl = nullptr;
    if (bounds) {
        draft_masks = (int32_t *)ctx->buf("draft_masks", (size_t)F * 8, &rc);
        draft_vfl = (int32_t *)ctx->buf("draft_vfl", (size_t)F * 16, &rc);
        if (rc != BPMX_OK) return rc;
    }
    /* find_peaks' candidate lists and the run's scan record (bpmx_fpscan.h:
     * the trough launch's scan, reused by the peak launch) */
    int32_t *cand = nullptr, *vcand = nullptr, *fp_scan = nullptr;
    double *cval = nullptr, *vval = nullptr;
    if (do_floor || do_peaks) {
        cand = (int32_t *)ctx->buf("cand", (size_t)sumnd * 4, &rc);
        vcand = (int32_t *)ctx->buf("vcand", (size_t)sumnd * 4, &rc);
        cval = (double *)ctx->buf("cval", (size_t)sumnd * 8, &rc);
        vval = (double *)ctx->buf("vval", (size_t)sumnd * 8, &rc);
        fp_scan = (int32_t *)ctx->buf("fp_scan", (size_t)F * 4 * (1 + 2 * FPS_NW), &rc);
        if (rc != BPMX_OK) return rc;
    }
    InitOutArgs io;
    io.active = d_active; io.flags = (int32_t *)O->flags; io.n_files = F;
    io.ntr = do_floor ? (int32_t *)O->n_troughs : nullptr;
    io.npk = do_peaks ? (int32_t *)O->n_peaks : nullptr;
    io.runs = d_run1;
    io.nraw = d_nraw != di + 5 * F ? d_nraw : nullptr;       /* the caller's raw-trough counts */
    io.z1 = draft_masks; io.z2 = bounds ? draft_vfl + 2 * F : nullptr; io.z3 = fp_scan;
    /* a native envelope stage resets them in k_native_carry (one launch fewer) */
    const bool init_in_carry = do_env && P->mode != BPMX_MODE_REFERENCE;
    if (!init_in_carry) LAUNCH(ctx, s, "k_init_out", k_init_out, dim3((F + 255) / 256), dim3(256), 0, s, io);

    /* ---- ENVELOPE ---- */
    /* the detection stage's quantile levels, built here so that the fused
     * native Hilbert kernel can compute them from the envelope it writes */
    QuantArgs qa{};
    bool noise_lazy = false;
    double *qv = nullptr;
    if (do_floor || do_peaks) {
        qv = (double *)ctx->buf("qv", (size_t)F * Q_SLOTS * 8, &rc);
        if (rc != BPMX_OK) return rc;
        qa.env = O->env; qa.doff = d_doff; qa.active = d_active; qa.n_files = F; qa.qv = qv; qa.skip_le = QR_MAX;
        int L = 0;
        auto add = [&](double q, int slot) {      /* one radix select per distinct level */
            for (int l = 0; l < L; ++l)
                if (qa.q[l] == q) { qa.slot[l] |= 1 << slot; return; }
            qa.q[L] = q; qa.slot[L] = 1 << slot; ++L;
        };
        /* the noise-floor level (static fallback, < 5 troughs) is computed
         * lazily after the trough search unless it coincides with a level
         * needed anyway */
        if (do_floor) { add(P->trough_prom_q, Q_TROUGH); add(P->fallback_q, Q_FALLBACK); }
        if (do_peaks) add(P->peak_prom_q, Q_PEAK);
        if (do_floor) {
            noise_lazy = true;
            for (int l = 0; l < L; ++l)
                if (qa.q[l] == P->noise_floor_q) { qa.slot[l] |= 1 << Q_NOISE; noise_lazy = false; }
        }
        qa.n_levels = L;
        qa.skip = nullptr;
        qa.stats = 0;                     /* k_find_peaks builds its own block tables when it runs */
    }
    bool q_in_env = false;                /* every active recording's quantiles came with its envelope */
    if (do_env) {
        StageRange range("bpmx:envelope");
        if (P->mode == BPMX_MODE_REFERENCE) {
            double *scr = (double *)ctx->buf("ref_scratch", (size_t)((maxnd + 30 + 63) / 64 * 64) * F * 8, &rc);
            if (rc != BPMX_OK) return rc;
            EnvRefArgs a;
            a.pcm = B->pcm; a.foff = d_foff; a.doff = d_doff; a.active = d_active;
            a.n_files = F; a.dtype = P->dtype; a.channels = P->channels; a.ds = P->ds; a.env_window = P->env_window;
            std::memcpy(a.b, P->ba_b, sizeof a.b);
            std::memcpy(a.a, P->ba_a, sizeof a.a);
            std::memcpy(a.zi, P->ba_zi, sizeof a.zi);
            a.scratch = scr; a.env = O->env; a.y = O->y;
            /* chain mode (the rolling mean's outputs formed in parallel afterwards) */
            const bool chain = !(P->options & BPMX_OPT_REF_SERIAL_MEAN) && P->env_window > 1;
            a.sums = chain ? (double *)ctx->buf("ref_sums", (size_t)(std::max<int64_t>(maxnd, 1) + 1) * F * 8, &rc) : nullptr;
            a.chain = (int32_t *)ctx->buf("ref_chain", (size_t)F * 4, &rc);
            if (rc != BPMX_OK) return rc;
            const bool multi = P->channels > 1;
            const dim3 g((F + 63) / 64), b(64);
            const dim3 gp((unsigned)((maxnd + 30 + 63) / 64), (unsigned)((F + 63) / 64));
            /* b = b0 (1, 0, -2, 0, 1) exactly with integer PCM (always finite):
             * the filter step's short form (k_envelope_ref.hip, Df2t::step) */
            const bool zb = P->ba_b[1] == 0.0 && P->ba_b[3] == 0.0 && P->ba_b[4] == P->ba_b[0] &&
                            P->ba_b[2] == -2.0 * P->ba_b[0] &&
                            (P->dtype == BPMX_DT_U8 || P->dtype == BPMX_DT_I16 || P->dtype == BPMX_DT_I32);
            /* the forward pass in row chunks while k_ref_pick gathers the next
             * chunks on a side stream (BPMX_OPT_REF_NOSPLIT: one gather, then
             * the whole pass in k_envelope_ref_t) */
            const int64_t rows = maxnd + 30;
            /* chunk k: rows [R (2^k - 1), R (2^(k+1) - 1)): the first gather is
             * short (it is not overlapped), the later ones grow while the
             * gather (faster per row than the sequential pass) stays ahead */
            auto fwd_row = [&](int64_t k) -> int64_t { return std::min(rows, REF_FWD_ROWS * ((int64_t(1) << k) - 1)); };
            int64_t nfc = 1;
            while (fwd_row(nfc) < rows) ++nfc;
            const bool split = nfc >= 2 && !(P->options & BPMX_OPT_REF_NOSPLIT) && ctx->side_ready() &&
                               ctx->ref_events((size_t)nfc);
            a.pick_r0 = 0; a.fwd_rb = 0; a.fwd_re = 0; a.fwd_z = nullptr;
            a.kahan_z = nullptr; a.kahan_ib = 0; a.kahan_ie = 0; a.mean_r0 = 0;
            if (split) {
                a.fwd_z = (double *)ctx->buf("ref_fwd_z", (size_t)F * 4 * 8, &rc);
                if (rc != BPMX_OK) return rc;
            }
            /* chain mode: the Kahan pass in row chunks ending at 1/2, 3/4, 7/8
             * and all of the rows, each finished chunk's means formed by
             * k_ref_env_mean on the side stream while the next chunk runs */
            int64_t kend[4] = {0, 0, 0, 0};
            int nkc = 0;
            if (chain && split && maxnd >= 4096 && ctx->ref_events((size_t)nfc + 8)) {
                for (int k = 1; k <= 3; ++k) kend[nkc++] = (maxnd - (maxnd >> k)) & ~(int64_t)63;
                kend[nkc++] = maxnd;
                a.kahan_z = (double *)ctx->buf("ref_kahan_z", (size_t)F * 6 * 8, &rc);
                if (rc != BPMX_OK) return rc;
                a.kahan_ie = kend[0];
            }
            auto env_ref = [&](void (*pick)(EnvRefArgs), void (*body)(EnvRefArgs), void (*fwd)(EnvRefArgs)) -> int {
                if (!split) {
                    LAUNCH(ctx, s, "k_ref_pick", pick, gp, dim3(256), 0, s, a);
                    LAUNCH(ctx, s, "k_envelope_ref", body, g, b, 0, s, a);
                    return BPMX_OK;
                }
                EnvRefArgs c = a;
                hipStream_t s2 = ctx->side[0];
                HIP_TRY(hipEventRecord(ctx->side_fork, s));
                HIP_TRY(hipStreamWaitEvent(s2, ctx->side_fork, 0));
                for (int64_t k = 0; k < nfc; ++k) {
                    const int64_t r0 = fwd_row(k), r1 = fwd_row(k + 1);
                    c.pick_r0 = r0;
                    const dim3 gk((unsigned)((r1 - r0 + 63) / 64), (unsigned)((F + 63) / 64));
                    hipStream_t sk = k == 0 ? s : s2;
                    LAUNCH(ctx, sk, "k_ref_pick", pick, gk, dim3(256), 0, sk, c);
                    if (k > 0) HIP_TRY(hipEventRecord(ctx->ref_ev[k], s2));
                }
                for (int64_t k = 0; k < nfc; ++k) {
                    if (k > 0) HIP_TRY(hipStreamWaitEvent(s, ctx->ref_ev[k], 0));
                    c.fwd_rb = fwd_row(k);
                    c.fwd_re = fwd_row(k + 1);
                    LAUNCH(ctx, s, "k_ref_fwd", fwd, g, b, 0, s, c);
                }
                LAUNCH(ctx, s, "k_envelope_ref", body, g, b, 0, s, c);
                return BPMX_OK;
            };
#define ENV_REF_K(DT, M, Z) rc = env_ref(k_ref_pick<DT, M>, k_envelope_ref_t<DT, M, Z>, k_ref_fwd<Z>)
#define ENV_REF(DT)                                                                                  \
    if (multi) {                                                                                     \
        if (zb && DT <= BPMX_DT_I32) ENV_REF_K(DT, true, DT <= BPMX_DT_I32); else ENV_REF_K(DT, true, false); \
    } else {                                                                                         \
        if (zb && DT <= BPMX_DT_I32) ENV_REF_K(DT, false, DT <= BPMX_DT_I32); else ENV_REF_K(DT, false, false); \
    }
            switch (P->dtype) {
            case BPMX_DT_U8: ENV_REF(BPMX_DT_U8) break;
            case BPMX_DT_I16: ENV_REF(BPMX_DT_I16) break;
            case BPMX_DT_I32: ENV_REF(BPMX_DT_I32) break;
            case BPMX_DT_F32: ENV_REF(BPMX_DT_F32) break;
            default: ENV_REF(BPMX_DT_F64) break;
            }
            if (rc != BPMX_OK) return rc;
#undef ENV_REF
#undef ENV_REF_K
            if (chain && !a.kahan_z) {
                const dim3 gm((unsigned)((maxnd + 63) / 64), (unsigned)((F + 63) / 64));
                if (a.y) LAUNCH(ctx, s, "k_ref_env_mean", k_ref_env_mean<true>, gm, dim3(256), 0, s, a);
                else LAUNCH(ctx, s, "k_ref_env_mean", k_ref_env_mean<false>, gm, dim3(256), 0, s, a);
            } else if (chain) {
                hipStream_t s2 = ctx->side[0];
                EnvRefArgs c = a;
                for (int k = 0; k < nkc; ++k) {
                    if (k > 0) {                             /* steps [kend[k-1], kend[k]) */
                        c.kahan_ib = kend[k - 1];
                        c.kahan_ie = kend[k];
                        LAUNCH(ctx, s, "k_ref_kahan", k_ref_kahan, g, b, 0, s, c);
                    }
                    hipEvent_t ek = ctx->ref_ev[nfc + k];
                    HIP_TRY(hipEventRecord(ek, s));
                    HIP_TRY(hipStreamWaitEvent(s2, ek, 0));
                    const int64_t r0 = k > 0 ? kend[k - 1] : 0;
                    EnvRefArgs mk = a;
                    mk.mean_r0 = r0;
                    const dim3 gm((unsigned)((kend[k] - r0 + 63) / 64), (unsigned)((F + 63) / 64));
                    if (a.y) LAUNCH(ctx, s2, "k_ref_env_mean", k_ref_env_mean<true>, gm, dim3(256), 0, s2, mk);
                    else LAUNCH(ctx, s2, "k_ref_env_mean", k_ref_env_mean<false>, gm, dim3(256), 0, s2, mk);
                }
                hipEvent_t ej = ctx->ref_ev[nfc + 4];
                HIP_TRY(hipEventRecord(ej, s2));
                HIP_TRY(hipStreamWaitEvent(s, ej, 0));
            }
        } else {
            int r = native_envelope(ctx, P, B, O, s, F, foff, doff, maxnd, d_foff, d_doff, d_active,
                                    (do_floor || do_peaks) ? &qa : nullptr, &io);
            if (r != BPMX_OK) return r;
            if (do_floor || do_peaks) {
                q_in_env = true;
                for (int f = 0; f < F && q_in_env; ++f) q_in_env = !active[f] || ctx->nat_fused[f];
            }
        }
    }
    if (!do_floor && !do_peaks) return BPMX_OK;

    /* ---- shared detection inputs: block tables, quantiles ---- */
    StageRange range_in("bpmx:detection-inputs");
    double *bmax = (double *)ctx->buf("bmax", (size_t)sumb * 8, &rc);
    double *bmin = (double *)ctx->buf("bmin", (size_t)sumb * 8, &rc);
    int32_t *fp_fb = (int32_t *)ctx->buf("fp_fallback", (size_t)F * 4, &rc);
    uint8_t *state = (uint8_t *)ctx->buf("state", (size_t)sumnd, &rc);
    if (rc != BPMX_OK) return rc;
    BlockStatArgs bs;
    bs.env = O->env; bs.doff = d_doff; bs.boff = d_boff; bs.active = d_active; bs.n_files = F;
    bs.bmax = bmax; bs.bmin = bmin; bs.skip_le = QR_MAX;     /* k_quantile_reg writes those tables */
    const bool long_files = maxnd > QR_MAX;
    /* an ordered run (bpmx_run_ordered: candidate export, the caller's visiting
     * ranks) takes k_find_peaks, the kernel that implements them */
    const bool fp_global = (P->options & BPMX_OPT_PEAKS_GLOBAL) != 0 || ord != nullptr;
    auto set_order = [&](PeakArgs &a, int search) {
        if (!ord) return;
        a.cand_out = ord->cand[search];
        a.ncand_out = ord->n_cand[search];
        a.rank = ord->rank[search];
        a.use_rank = ord->use_rank[search];
        a.ordered_bit = search == 0 ? BPMX_F_TROUGH_ORDERED : BPMX_F_PEAK_ORDERED;
    };
    /* find_peaks: k_find_peaks_lds for every recording it holds; the others
     * (longer than FPL_NMIN, or more than FL_MC maxima) take the multi-
     * workgroup k_fpl_* path when the batch has long recordings, else the
     * one-workgroup k_find_peaks (BPMX_OPT_PEAKS_GLOBAL: k_find_peaks for all) */
    const bool fp_long = !fp_global && maxnd > FPL_NMIN;
    FplArgs fl{};
    if (fp_long) {
        fl.nu = (int32_t)((maxnd - 2 + FPL_U - 1) / FPL_U);
        fl.cnt = (int32_t *)ctx->buf("fpl_cnt", (size_t)F * fl.nu * 8, &rc);
        fl.mtot = (int32_t *)ctx->buf("fpl_mtot", (size_t)F * 4, &rc);
        fl.mp = (int32_t *)ctx->buf("fpl_mp", (size_t)sumnd * 4, &rc);
        fl.mh = (double *)ctx->buf("fpl_mh", (size_t)sumnd * 8, &rc);
        fl.vv = (double *)ctx->buf("fpl_vv", (size_t)(sumnd + F) * 8, &rc);
        const size_t n32 = (size_t)(sumnd >> 5) + 4 * (size_t)F + 4, n1k = (size_t)(sumnd >> 10) + 4 * (size_t)F + 4;
        double *b32 = (double *)ctx->buf("fpl_b32", n32 * 3 * 8, &rc);
        double *b1k = (double *)ctx->buf("fpl_b1k", n1k * 3 * 8, &rc);
        if (rc != BPMX_OK) return rc;
        fl.b32h = b32; fl.b32l = b32 + n32; fl.b32r = b32 + 2 * n32;
        fl.b1kh = b1k; fl.b1kl = b1k + n1k; fl.b1kr = b1k + 2 * n1k;
        fl.dfail = (int32_t *)ctx->buf("fpl_dfail", (size_t)F * 4, &rc);
        if (rc != BPMX_OK) return rc;
        fl.dchunk = 1;
    }
    const dim3 g_unit((unsigned)((((maxnd - 2 + FPL_U - 1) / FPL_U) + 3) / 4), (unsigned)F);
    const dim3 g_prom((unsigned)((maxnd / 2 + 1 + 255) / 256), (unsigned)F);
    const dim3 g_dch((unsigned)((maxnd / 2 + 1 + FPC_S - 1) / FPC_S), (unsigned)F);
#define FIND_PEAKS(A, TAG)                                                                                  \
    do {                                                                                                   \
        (A).vcand = vcand; (A).cval = cval; (A).vval = vval; (A).fallback = fp_fb; (A).only = nullptr; (A).flags = (int32_t *)O->flags;     \
        (A).lds_nmax = fp_long ? FPL_NMIN : INT64_MAX;                                                     \
        if (!fp_global) {                                                                                  \
            LAUNCH(ctx, s, "k_find_peaks[" TAG "]", k_find_peaks_lds, dim3(F), dim3(1024), 0, s, (A));    \
            (A).only = fp_fb;             /* recordings the LDS kernel hands over */                       \
        }                                                                                                  \
        if (fp_long) {                                                                                     \
            LAUNCH(ctx, s, "k_fpl_scan[" TAG "]", k_fpl_scan, g_unit, dim3(256), 0, s, (A), fl);          \
            LAUNCH(ctx, s, "k_fpl_place[" TAG "]", k_fpl_place, dim3(F), dim3(256), 0, s, (A), fl);       \
            LAUNCH(ctx, s, "k_fpl_fill[" TAG "]", k_fpl_fill, g_unit, dim3(256), 0, s, (A), fl);          \
            LAUNCH(ctx, s, "k_fpl_dist_ch[" TAG "]", k_fpl_dist_ch, g_dch, dim3(FPC_T), 0, s, (A), fl);   \
            LAUNCH(ctx, s, "k_fpl_distance[" TAG "]", k_fpl_distance, dim3(F), dim3(1024), 0, s, (A), fl);\
            LAUNCH(ctx, s, "k_fpl_prom[" TAG "]", k_fpl_prom, g_prom, dim3(256), 0, s, (A), fl);          \
            LAUNCH(ctx, s, "k_fpl_compact[" TAG "]", k_fpl_compact, dim3(F), dim3(1024), 0, s, (A), fl);  \
        } else {                                                                                           \
            LAUNCH(ctx, s, "k_find_peaks[" TAG ",gm]", k_find_peaks, dim3(F), dim3(1024), 0, s, (A));     \
        }                                                                                                  \
    } while (0)
    if (long_files) {
        /* a few workgroups per long recording when the batch is small */
        const int64_t gy = std::min<int64_t>((((maxnd + 63) >> 6) + 3) / 4, std::max<int64_t>(1, 2048 / F));
        LAUNCH(ctx, s, "k_block_stats", k_block_stats, dim3(F, (unsigned)gy), dim3(256), 0, s, bs);
    }
    /* long recordings' quantiles: radix select over many workgroups (k_ql_*) */
    auto quantile_long = [&](const QuantArgs &q) -> int {
        int qrc = BPMX_OK;
#ifndef BPMX_QL_RADIX
        /* five launches, two passes over env (k_qv_*, r06) */
        QvArgs V;
        V.Q = q;
        V.boff = d_boff; V.bmax = bmax; V.bmin = bmin;
        V.rg = (QvRange *)ctx->buf("qv_range", (size_t)F * sizeof(QvRange), &qrc);
        V.st = (QvState *)ctx->buf("qv_state", (size_t)F * Q_SLOTS * sizeof(QvState), &qrc);
        V.hist = (unsigned int *)ctx->buf("qv_hist", (size_t)F * QV_BINS * 4, &qrc);
        V.cand = (unsigned long long *)ctx->buf("qv_cand", (size_t)sumnd * Q_SLOTS * 8, &qrc);
        if (qrc != BPMX_OK) return qrc;
        HIP_TRY(hipMemsetAsync(V.hist, 0, (size_t)F * QV_BINS * 4, s));
        const dim3 gv((unsigned)((maxnd + QV_CHUNK - 1) / QV_CHUNK), (unsigned)F);
        LAUNCH(ctx, s, "k_quantile", k_qv_range, dim3(F), dim3(64), 0, s, V);
        LAUNCH(ctx, s, "k_quantile", k_qv_hist, gv, dim3(256), 0, s, V);
        LAUNCH(ctx, s, "k_quantile", k_qv_select, dim3(F, q.n_levels), dim3(256), 0, s, V);
        LAUNCH(ctx, s, "k_quantile", k_qv_collect, gv, dim3(256), 0, s, V);
        LAUNCH(ctx, s, "k_quantile", k_qv_final, dim3(F, q.n_levels), dim3(256), 0, s, V);
        return BPMX_OK;
#endif
        QlArgs A;
        A.Q = q;
        A.st = (QlState *)ctx->buf("ql_state", (size_t)F * Q_SLOTS * sizeof(QlState), &qrc);
        const size_t hb = (size_t)QL_PASSES * F * Q_SLOTS * QL_BINS * 4;
        A.hist = (unsigned int *)ctx->buf("ql_hist", hb, &qrc);
        if (qrc != BPMX_OK) return qrc;
        HIP_TRY(hipMemsetAsync(A.hist, 0, hb, s));
        const dim3 gc((unsigned)((maxnd + QL_CHUNK - 1) / QL_CHUNK), (unsigned)F);
        A.pass = 0;
        LAUNCH(ctx, s, "k_quantile", k_ql_init, dim3(F), dim3(64), 0, s, A);
        for (int p = 0; p < QL_PASSES; ++p) {
            A.pass = p;
            LAUNCH(ctx, s, "k_quantile", k_ql_hist, gc, dim3(256), 0, s, A);
            LAUNCH(ctx, s, "k_quantile", k_ql_select, dim3(F, q.n_levels), dim3(256), 0, s, A);
        }
        LAUNCH(ctx, s, "k_quantile", k_ql_next, gc, dim3(256), 0, s, A);
        LAUNCH(ctx, s, "k_quantile", k_ql_final, dim3(F), dim3(64), 0, s, A);
        return BPMX_OK;
    };
    {
        QuantArgs a = qa;
        if (!q_in_env) LAUNCH(ctx, s, "k_quantile_reg", k_quantile_reg, dim3(F), dim3(QR_T), 0, s, a, bs);
        if (long_files) {
            /* long recordings take the noise-floor level in the same passes (one
             * more compare per key) instead of a second 15-launch round later */
            QuantArgs al = a;
            if (noise_lazy) {
                al.q[al.n_levels] = P->noise_floor_q;
                al.slot[al.n_levels] = 1 << Q_NOISE;
                al.n_levels++;
            }
            if ((rc = quantile_long(al)) != BPMX_OK) return rc;
        }
    }

    /* ---- FLOOR ---- */
    if (do_floor) {
        StageRange range("bpmx:floor");
        int64_t *rawt = (int64_t *)ctx->buf("raw_troughs", (size_t)sumnd * 8, &rc);
        /* env at the raw and at the sanitised troughs, beside the indices (the
         * trough search and k_sanitize write them; the floor kernels read them
         * instead of gathering a cache line of env per trough) */
        double *rawv = (double *)ctx->buf("raw_trough_vals", (size_t)sumnd * 8, &rc);
        double *trv = (double *)ctx->buf("trough_vals", (size_t)sumnd * 8, &rc);
        double *dense = (double *)ctx->buf("dense", (size_t)sumnd * 8, &rc);
        double *draft = (double *)ctx->buf("draft", (size_t)sumnd * 8, &rc);
        if (rc != BPMX_OK) return rc;
        {
            PeakArgs a;
            a.env = O->env; a.height = nullptr; a.doff = d_doff; a.boff = d_boff; a.active = d_active;
            a.bmax = bmax; a.bmin = bmin; a.qv = qv; a.qslot = Q_TROUGH; a.n_files = F; a.distance = P->distance;
            a.sign = -1.0; a.cand = cand; a.state = state; a.out = rawt; a.outv = rawv; a.nout = d_nraw;
            a.run_out = d_run1; a.run_min = 5; a.tie_bit = BPMX_F_TROUGH_TIE;
            a.scan_ok = fp_scan; a.scan_cnt = fp_scan + F;
            set_order(a, 0);
            FIND_PEAKS(a, "troughs");
        }
        if (bad_window)
            LAUNCH(ctx, s, "k_flag_window", k_flag_window, dim3((F + 255) / 256), dim3(256), 0, s, F, d_run1,
                   (int32_t *)O->flags);
        /* recordings of <= WM_MMAX samples: everything after the draft bracket
         * in one launch (k_floor_wm), the static floor's quantile included */
        const bool floor_wm = !(P->options & (BPMX_OPT_ROLLQ_MERGE | BPMX_OPT_ROLLQ_GLOBAL | BPMX_OPT_ROLLQ_NOPRUNE)) &&
                              maxnd <= WM_MMAX;
        if (noise_lazy && !floor_wm) {    /* the static-floor quantile, for recordings with < 5 troughs */
            QuantArgs a;
            a.env = O->env; a.doff = d_doff; a.active = d_active; a.n_files = F; a.qv = qv; a.skip_le = QR_MAX;
            a.n_levels = 1; a.q[0] = P->noise_floor_q; a.slot[0] = 1 << Q_NOISE;
            a.skip = d_run1; a.stats = 0;
            LAUNCH(ctx, s, "k_quantile_reg", k_quantile_reg, dim3(F), dim3(QR_T), 0, s, a, bs);
            /* long recordings computed this level with the others (at most three
             * distinct levels before it, so it always fits in Q_SLOTS) */
        }
        /* rolling-quantile geometry: T outputs per step, sorted union in LDS */
        const int64_t W = bad_window ? P->min_periods : P->noise_window;
        const int cap = (int)((W + RQ_T - 1 + 63) / 64 * 64);
        const size_t lds = rollq_lds_bytes(RQ_T, cap);
        /* wavelet-matrix kernel for recordings that fit its LDS budget; the
         * sorted-union kernel for longer ones (or when forced) */
        const bool use_wm = !(P->options & (BPMX_OPT_ROLLQ_MERGE | BPMX_OPT_ROLLQ_GLOBAL));
        const bool need_merge = !use_wm || maxnd > WM_MMAX;
        /* windows beyond the LDS sorted-union kernel: the same algorithm with
         * the union in global scratch (any window, any length) */
        const bool merge_g = need_merge && (cap > 32 * RQ_T || W + RQ_T >= 65000 || (P->options & BPMX_OPT_ROLLQ_GLOBAL));
        const int64_t gcap = (std::min<int64_t>(W + RQ_T, maxnd + 64) + 63) / 64 * 64;
        const size_t lds_g = rollq_g_lds_bytes(RQ_T, gcap);
        if (merge_g && lds_g > 160 * 1024)
            return fail(BPMX_E_LIMIT, "noise window and recording both longer than " +
                                          std::to_string((160 * 1024 - 16384) / 4 * 64) + " samples");
        uint16_t *wm_pos = use_wm ? (uint16_t *)ctx->buf("wm_pos", (size_t)sumnd * 2, &rc) : nullptr;   /* rank -> index */
        int32_t *wm_full = use_wm ? (int32_t *)ctx->buf("wm_full", (size_t)F * 4, &rc) : nullptr;
        if (rc != BPMX_OK) return rc;
        const int64_t wm_n = std::min<int64_t>(maxnd, WM_MMAX);
        const size_t wm_lds_p = wm_layout(wm_n, true).total, wm_lds = wm_layout(wm_n, false).total;
        /* long recordings: the pruned wavelet matrix over chunks of wm_c outputs
         * (a chunk's windows reach wm_c + W - 1 samples); a recording with a
         * chunk it cannot take falls to the sorted-union kernel */
        const int64_t wm_c = (WM_MMAX - W + 1) / 64 * 64;
        const bool wm_chunks = use_wm && maxnd > WM_MMAX && !(P->options & BPMX_OPT_ROLLQ_NOPRUNE) && wm_c >= 2048;
        const int64_t wm_nch = wm_chunks ? (maxnd + wm_c - 1) / wm_c : 1;
        int32_t *wm_fail = wm_chunks ? (int32_t *)ctx->buf("wm_fail", (size_t)F * 4, &rc) : nullptr;
        uint16_t *wm_pos_ch = wm_chunks ? (uint16_t *)ctx->buf("wm_pos_ch", (size_t)F * wm_nch * WM_PMAX * 2, &rc) : nullptr;
        if (rc != BPMX_OK) return rc;
        if (wm_nch > 65535) return fail(BPMX_E_LIMIT, "recording too long for the chunked rolling quantile");
        /* k_interp / k_floor_final stride over a recording with gx workgroups:
         * 8, or more when the batch has few recordings */
        const dim3 g2((unsigned)std::min<int64_t>((maxnd + 255) / 256, std::max<int64_t>(8, 2048 / F)), F);
        /* dense = np.interp of the troughs, for the recordings the rolling-quantile
         * kernels do not interpolate themselves (the wavelet matrix stages up to
         * WM_TRMAX troughs, or a long recording's chunk) */
        auto interp = [&](const int32_t *run, const int64_t *tr, const int32_t *ntr, int64_t skip_gt) -> int {
            InterpArgs a;
            a.env = O->env; a.doff = d_doff; a.troughs = tr; a.ntr = ntr; a.run = run; a.n_files = F;
            a.dense = dense; a.skip_n = use_wm ? WM_MMAX : -1; a.skip_gt = skip_gt;
            /* with no long recording only those with > WM_TRMAX troughs (rare): two workgroups each */
            const dim3 gi = maxnd <= WM_MMAX && use_wm ? dim3(2, (unsigned)F) : g2;
            LAUNCH(ctx, s, "k_interp", k_interp, gi, dim3(256), 0, s, a);
            return BPMX_OK;
        };
        auto rollq = [&](const int32_t *run, const int64_t *tr, const int32_t *ntr, double *outp,
                         int32_t *allnan, const double *tv) -> int {
            RollqArgs a;
            a.dense = dense; a.doff = d_doff; a.troughs = tr; a.tv = tv; a.run = run; a.n_files = F;
            a.env = O->env; a.ntr = ntr;
            a.window = (int32_t)W; a.min_periods = P->min_periods; a.cap = cap; a.q = P->noise_floor_q;
            a.out = outp; a.allnan = allnan; a.wm_max = use_wm ? WM_MMAX : 0;
            a.wm_chunk = 0; a.wm_fail = wm_fail; a.wm_pos_ch = wm_pos_ch;
            int rq_rc = BPMX_OK;
            int32_t *vfl = need_merge ? (int32_t *)ctx->buf("rollq_valid", (size_t)F * 8, &rq_rc) : nullptr;
            if (rq_rc != BPMX_OK) return rq_rc;
            a.vfirst = vfl;
            a.vlast = vfl ? vfl + F : nullptr;
            if (need_merge) {
                HIP_TRY(hipMemsetAsync(a.vfirst, 0x7F, (size_t)F * 4, s));      /* 0x7F7F7F7F: above any index */
                HIP_TRY(hipMemsetAsync(a.vlast, 0xFF, (size_t)F * 4, s));       /* -1 */
            }
            if (wm_chunks) {
                HIP_TRY(hipMemsetAsync(wm_fail, 0, (size_t)F * 4, s));
                a.wm_chunk = (int32_t)wm_c;
            }
            /* the wavelet-matrix kernels interpolate every recording <= WM_MMAX
             * themselves (from the troughs in LDS, or over global memory past
             * WM_TRMAX troughs): dense only for the sorted-union kernels */
            if (need_merge && (rq_rc = interp(run, tr, ntr, wm_chunks ? WM_MMAX : INT64_MAX)) != BPMX_OK) return rq_rc;
            if (use_wm) {
                /* the pruned structure; a recording it cannot take (too many
                 * kept samples, > WM_TRMAX troughs, a compact-key collision)
                 * runs unpruned in the same workgroup, so its LDS is the
                 * larger layout (BPMX_OPT_ROLLQ_NOPRUNE: unpruned for all) */
                wm_lds_attr(ctx->device);
                if (!(P->options & BPMX_OPT_ROLLQ_NOPRUNE))
                    LAUNCH(ctx, s, "k_rollq_wm", k_rollq_wm_t<true>, dim3(F, (unsigned)wm_nch), dim3(WM_T),
                           std::max(wm_lds_p, wm_lds), s, a, wm_pos, wm_full);
                else
                    LAUNCH(ctx, s, "k_rollq_wm[full]", k_rollq_wm_t<false>, dim3(F), dim3(WM_T), wm_lds, s, a, wm_pos,
                           wm_full);
            }
            if (!need_merge) return BPMX_OK;
            /* long recordings: a workgroup per chunk of outputs (each chunk pays
             * one extra window fill: ~13 merge rounds against 32 or 16 tiles);
             * after the chunked wavelet matrix only the recordings it gave up */
            RollqArgs fill = a;
            if (wm_chunks) {
                a.run = wm_fail;
                if ((rq_rc = interp(wm_fail, tr, ntr, INT64_MAX)) != BPMX_OK) return rq_rc;
            }
            /* 8192 outputs per chunk, halved (down to 1024) while the batch
             * gives fewer than 1024 workgroups: a chunk's first-window fill is
             * fixed overhead, worth paying only when CUs would sit idle */
            a.chunk = 8192;
            while (a.chunk > 1024 && (int64_t)F * ((maxnd + a.chunk - 1) / a.chunk) < 1024) a.chunk >>= 1;
            /* the global-union kernel pays a window-sized fill per chunk: chunks of at least W */
            if (merge_g) a.chunk = std::max<int64_t>(a.chunk, (W + RQ_T - 1) / RQ_T * RQ_T);
            const int64_t nch = (maxnd + a.chunk - 1) / a.chunk;
            if (nch > 65535) return fail(BPMX_E_LIMIT, "recording too long for the chunked rolling quantile");
            const dim3 gq((unsigned)F, (unsigned)nch);
            if (merge_g) {
                a.gcap = gcap;
                a.gv = (double *)ctx->buf("rollq_gv", (size_t)F * nch * 2 * gcap * 8, &rq_rc);
                a.gp = (int32_t *)ctx->buf("rollq_gp", (size_t)F * nch * 2 * gcap * 4, &rq_rc);
                if (rq_rc != BPMX_OK) return rq_rc;
                (void)hipFuncSetAttribute((const void *)k_rolling_quantile_g<RQ_T>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_g);
                LAUNCH(ctx, s, "k_rolling_quantile", (k_rolling_quantile_g<RQ_T>), gq, dim3(RQ_T), lds_g, s, a);
            } else if (cap <= 16 * RQ_T) {
                (void)hipFuncSetAttribute((const void *)k_rolling_quantile<RQ_T, 16>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                LAUNCH(ctx, s, "k_rolling_quantile", (k_rolling_quantile<RQ_T, 16>), gq, dim3(RQ_T), lds, s, a);
            } else {
                (void)hipFuncSetAttribute((const void *)k_rolling_quantile<RQ_T, 32>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                LAUNCH(ctx, s, "k_rolling_quantile", (k_rolling_quantile<RQ_T, 32>), gq, dim3(RQ_T), lds, s, a);
            }
            LAUNCH(ctx, s, "k_rollq_fill", k_rollq_fill, dim3(4, (unsigned)F), dim3(256), 0, s, fill);
            return BPMX_OK;
        };
        /* Draft floor: sanitize reads it at the raw troughs only, so the
         * recordings whose every keep decision follows from k_draft_bounds'
         * bracket skip the full rolling quantile; the others (and, after
         * sanitize, bounded ones left with <= 2 troughs, whose floor IS the
         * draft) get it exactly.  BPMX_OPT_DRAFT_FULL forces it for all. */
        uint8_t *tdec = nullptr;
        int32_t *d_exact = d_run1, *d_runfb = nullptr;
        if (bounds) {
            tdec = (uint8_t *)ctx->buf("trough_dec", (size_t)sumnd, &rc);
            if (rc != BPMX_OK) return rc;
            d_exact = draft_masks;                             /* zeroed by k_init_out */
            d_runfb = draft_masks + F;
            DraftBoundArgs a;
            a.env = O->env; a.doff = d_doff; a.raw = rawt; a.rawv = rawv; a.nraw = d_nraw; a.run = d_run1;
            a.n_files = F;
            a.window = (int32_t)W; a.min_periods = P->min_periods; a.q = P->noise_floor_q; a.mult = P->reject_mult;
            a.dec = tdec; a.exact = d_exact;
            a.local_m = (P->options & BPMX_OPT_DRAFT_GLOBAL_RANK) ? INT_MAX : DB_LOCAL_M;
            a.stats = d_stats;
            if (rc != BPMX_OK) return rc;
            /* find_peaks' distance spaces the troughs, so a recording has at most Nd / distance + 1 */
            const int64_t trmax = maxnd / std::max<int64_t>(1, P->distance) + 1;
            const unsigned gy = (unsigned)std::max<int64_t>(1, (trmax + DB_T - 1) / DB_T);
            a.vfl = draft_vfl;
            a.nund = draft_vfl + 2 * F;                        /* zeroed by k_init_out */
            LAUNCH(ctx, s, "k_draft_bounds", k_draft_bounds, dim3(F, gy), dim3(DB_T), 0, s, a);
            /* at most BPMX_DP_GY workgroups per recording, each taking every
             * gridDim.y-th chunk of 32 troughs */
#ifndef BPMX_DP_GY
#define BPMX_DP_GY 4
#endif
            const unsigned gp = (unsigned)std::max<int64_t>(1, std::min<int64_t>(BPMX_DP_GY, (trmax + DP_CHUNK - 1) / DP_CHUNK));
            LAUNCH(ctx, s, "k_draft_points", k_draft_points<1>, dim3(F, gp), dim3(DB_T), 0, s, a);
            LAUNCH(ctx, s, "k_draft_points[wide]", k_draft_points<4>, dim3(F, gp), dim3(DB_T), 0, s, a);
        }
        SanitizeArgs sa;
        sa.env = O->env; sa.draft = draft; sa.doff = d_doff; sa.active = d_active; sa.raw = rawt; sa.nraw = d_nraw;
        sa.rawv = rawv; sa.outv = trv;
        sa.n_files = F; sa.mult = P->reject_mult; sa.out = O->troughs; sa.nout = O->n_troughs; sa.flags = O->flags;
        sa.run2 = d_run2; sa.dec = tdec; sa.exact = d_exact; sa.run_fb = d_runfb;
        if (floor_wm) {
            FloorWmArgs a;
            a.rq.dense = dense; a.rq.doff = d_doff; a.rq.n_files = F; a.rq.env = O->env;
            a.rq.window = (int32_t)W; a.rq.min_periods = P->min_periods; a.rq.cap = cap; a.rq.q = P->noise_floor_q;
            a.rq.wm_max = WM_MMAX; a.rq.wm_chunk = 0; a.rq.wm_fail = nullptr; a.rq.wm_pos_ch = nullptr;
            a.rq.vfirst = a.rq.vlast = nullptr; a.rq.chunk = 0; a.rq.gv = nullptr; a.rq.gp = nullptr; a.rq.gcap = 0;
            a.rq.troughs = nullptr; a.rq.tv = nullptr; a.rq.ntr = nullptr; a.rq.run = nullptr; a.rq.out = nullptr;
            a.rq.allnan = nullptr;
#ifdef BPMX_STAMPS
            a.rq.stamps = nullptr;
#endif
            sa.run2 = nullptr; sa.run_fb = nullptr;
            a.sa = sa;
            a.exact = d_exact;
            a.qv = qv;
            a.qn = QuantArgs{};
            if (noise_lazy) {
                a.qn.env = O->env; a.qn.doff = d_doff; a.qn.active = d_active; a.qn.n_files = F; a.qn.qv = qv;
                a.qn.skip_le = QR_MAX; a.qn.n_levels = 1; a.qn.q[0] = P->noise_floor_q; a.qn.slot[0] = 1 << Q_NOISE;
                a.qn.skip = nullptr; a.qn.stats = 0;
            }
            a.floor = O->floor; a.draft = draft; a.an_draft = d_an1; a.an_final = d_an2; a.full = wm_full;
            if ((rc = rollq(d_exact, rawt, d_nraw, draft, d_an1, rawv)) != BPMX_OK) return rc;   /* the full draft */
            wm_lds_attr(ctx->device);
            LAUNCH(ctx, s, "k_floor_wm", k_floor_wm, dim3(F), dim3(WM_T), std::max(wm_lds_p, wm_lds), s, a);
        }
        if (!floor_wm && (rc = rollq(d_exact, rawt, d_nraw, draft, d_an1, rawv)) != BPMX_OK) return rc;
        if (!floor_wm) {
            SanitizeArgs a;
            a.env = O->env; a.draft = draft; a.doff = d_doff; a.active = d_active; a.raw = rawt; a.nraw = d_nraw;
            a.rawv = rawv; a.outv = trv;
            a.n_files = F; a.mult = P->reject_mult; a.out = O->troughs; a.nout = O->n_troughs; a.flags = O->flags;
            a.run2 = d_run2; a.dec = tdec; a.exact = d_exact; a.run_fb = d_runfb;
            LAUNCH(ctx, s, "k_sanitize", k_sanitize, dim3(F), dim3(256), 0, s, a);
        }
        if (!floor_wm && bounds && (rc = rollq(d_runfb, rawt, d_nraw, draft, d_an1, rawv)) != BPMX_OK) return rc;
        if (!floor_wm && (rc = rollq(d_run2, O->troughs, O->n_troughs, O->floor, d_an2, trv)) != BPMX_OK) return rc;
        if (!floor_wm) {
            FinalArgs a;
            a.draft = draft; a.doff = d_doff; a.active = d_active; a.qv = qv; a.allnan_draft = d_an1;
            a.allnan_final = d_an2; a.n_files = F; a.floor = O->floor; a.flags = O->flags;
            /* one workgroup per recording unless they are long: most recordings
             * exit at once, and a static or draft floor is a short fill */
#ifndef BPMX_FF_WIDE
            const dim3 gf(maxnd > 65536 ? g2.x : 1u, (unsigned)F);
#else
            const dim3 gf = g2;
#endif
            LAUNCH(ctx, s, "k_floor_final", k_floor_final, gf, dim3(256), 0, s, a);
        }
    }

    /* ---- PEAKS ---- */
    if (do_peaks) {
        StageRange range("bpmx:peaks");
        PeakArgs a;
        a.env = O->env; a.height = O->floor; a.doff = d_doff; a.boff = d_boff; a.active = d_active;
        a.bmax = bmax; a.bmin = bmin; a.qv = qv; a.qslot = Q_PEAK; a.n_files = F; a.distance = P->distance;
        a.sign = 1.0; a.cand = cand; a.state = state; a.out = O->peaks; a.nout = O->n_peaks;
        a.run_out = nullptr; a.run_min = 0; a.tie_bit = BPMX_F_PEAK_TIE;
        a.scan_ok = fp_scan; a.scan_cnt = fp_scan + F;   /* the run's scan record: the trough launch's */
        set_order(a, 1);
        FIND_PEAKS(a, "peaks");
    }
#undef FIND_PEAKS
    return BPMX_OK;
}

/* ---------------------------------------------------------------------------
 * Pipelined run (bpmx_set_pipeline): the batch in `chunks` runs of whole
 * recordings.  Chunk k's envelope stage (native mode: the HBM-bound block
 * kernel and the per-recording transforms) runs on an internal stream that may
 * be restricted to `env_cus` CUs; its detection stages (quantiles, troughs,
 * noise floor, peaks: latency-bound per-recording kernels) run on the caller's
 * stream (or an internal one restricted to the other CUs) once its envelope is
 * done, while chunk k+1's envelope streams its PCM.  Each chunk slot has its
 * own contexts (scratch, geometry) for the two stages, so the only data the
 * streams share are the output arrays, ordered by events.  Outputs are those
 * of one run over the whole batch.
 * ------------------------------------------------------------------------- */
static int pipe_ready(bpmx_ctx *ctx, int K) {
    if ((int)ctx->pipe_sub.size() < 2 * K) {
        while ((int)ctx->pipe_sub.size() < 2 * K) {
            bpmx_ctx *c = new bpmx_ctx();
            c->device = ctx->device;
            c->root = ctx;
            ctx->pipe_sub.push_back(c);
        }
    }
    while ((int)ctx->pipe_ev.size() < K + 1) {
        hipEvent_t e;
        HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->pipe_ev.push_back(e);
    }
    auto mk = [&](hipStream_t *st, int lo, int ncu) -> int {
        if (*st) return BPMX_OK;
        int total = 0;
        HIP_TRY(hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, ctx->device));
        if (ncu <= 0 || ncu >= total) {
            HIP_TRY(hipStreamCreateWithFlags(st, hipStreamNonBlocking));
            return BPMX_OK;
        }
        /* mask bits [lo, lo + ncu): the driver deals the bits of a stream's CU
         * mask round-robin over the XCDs (bit c -> XCD c % 8, the (c / 8)-th CU
         * there), so a contiguous run of a multiple of 8 bits keeps the same
         * share of CUs on every XCD, as the workgroups are dealt too */
        std::vector<uint32_t> mask((total + 31) / 32, 0u);
        if (std::getenv("BPMX_CUMASK_PER_WORD")) {
            /* diagnostic: the other reading, one 32-bit word per XCD */
            const int X = (total + 31) / 32;
            for (int x = 0; x < X; ++x)
                for (int c = lo / X; c < (lo + ncu) / X && c < 32; ++c) mask[x] |= 1u << c;
        } else {
            for (int c = lo; c < lo + ncu && c < total; ++c) mask[c / 32] |= 1u << (c % 32);
        }
        HIP_TRY(hipExtStreamCreateWithCUMask(st, (uint32_t)mask.size(), mask.data()));
        return BPMX_OK;
    };
    int rc = mk(&ctx->pipe_env, 0, ctx->pipe_env_cus);
    if (rc != BPMX_OK) return rc;
    if (ctx->pipe_det_cus > 0 && (rc = mk(&ctx->pipe_det, ctx->pipe_env_cus, ctx->pipe_det_cus)) != BPMX_OK) return rc;
    return BPMX_OK;
}

static size_t dtype_bytes(int dt) {
    switch (dt) {
    case BPMX_DT_U8: return 1;
    case BPMX_DT_I16: return 2;
    case BPMX_DT_F64: return 8;
    default: return 4;
    }
}

static int run_pipelined(bpmx_ctx *ctx, const bpmx_params *P, const bpmx_batch *B, const bpmx_out *O,
                         hipStream_t s) {
    const int F = B->n_files;
    const int K = std::min(ctx->pipe_chunks, F);
    HIP_TRY(hipSetDevice(ctx->device));
    int rc = pipe_ready(ctx, K);
    if (rc != BPMX_OK) return rc;
    if (P->options & BPMX_OPT_STATS) {
        int64_t *d_stats = (int64_t *)ctx->buf("stats", BPMX_NSTATS * 8, &rc);
        if (rc != BPMX_OK) return rc;
        HIP_TRY(hipMemsetAsync(d_stats, 0, BPMX_NSTATS * 8, s));
    }
    /* chunk boundaries by frames (recordings are whole), decimated offsets */
    const int64_t *fo = B->frame_offsets;
    const int64_t total = fo[F] - fo[0];
    std::vector<int> fb(K + 1, F);
    fb[0] = 0;
    for (int k = 1, f = 0; k < K; ++k) {
        const int64_t want = fo[0] + total * k / K;
        while (f < F && fo[f] < want) ++f;
        fb[k] = std::max(fb[k - 1] + 1, std::min(f, F - (K - k)));
    }
    std::vector<int64_t> doff(F + 1, 0);
    for (int f = 0; f < F; ++f) doff[f + 1] = doff[f] + bpmx_decimated_length(fo[f + 1] - fo[f], P->ds);
    /* the envelope stream starts after everything already queued on the caller's stream */
    hipEvent_t start = ctx->pipe_ev[K];
    HIP_TRY(hipEventRecord(start, s));
    HIP_TRY(hipStreamWaitEvent(ctx->pipe_env, start, 0));
    if (ctx->pipe_det) HIP_TRY(hipStreamWaitEvent(ctx->pipe_det, start, 0));
    const size_t fbytes = dtype_bytes(P->dtype) * (size_t)P->channels;
    bpmx_params pe = *P, pd = *P;
    pe.stages = BPMX_STAGE_ENVELOPE;
    pd.stages = P->stages & ~BPMX_STAGE_ENVELOPE;
    for (int k = 0; k < K; ++k) {
        const int f0 = fb[k], f1 = fb[k + 1];
        bpmx_batch b;
        b.n_files = f1 - f0;
        b.reserved = 0;
        b.pcm = (const char *)B->pcm + (size_t)(fo[f0] - fo[0]) * fbytes;
        b.frame_offsets = fo + f0;
        const int64_t d0 = doff[f0];
        bpmx_out o;
        o.env = O->env + d0;
        o.floor = O->floor ? O->floor + d0 : nullptr;
        o.y = O->y ? O->y + d0 : nullptr;
        o.troughs = O->troughs ? O->troughs + d0 : nullptr;
        o.peaks = O->peaks ? O->peaks + d0 : nullptr;
        o.n_troughs = O->n_troughs + f0;
        o.n_peaks = O->n_peaks + f0;
        o.flags = O->flags + f0;
        o.n_raw_troughs = O->n_raw_troughs ? O->n_raw_troughs + f0 : nullptr;
        if ((rc = run_impl(ctx->pipe_sub[2 * k], &pe, &b, &o, ctx->pipe_env, true)) != BPMX_OK) return rc;
        HIP_TRY(hipEventRecord(ctx->pipe_ev[k], ctx->pipe_env));
        /* detection: the restricted stream while later envelopes run, the
         * caller's stream for the last chunk (every CU free by then) */
        hipStream_t sd = (ctx->pipe_det && k + 1 < K) ? ctx->pipe_det : s;
        HIP_TRY(hipStreamWaitEvent(sd, ctx->pipe_ev[k], 0));
        if (pd.stages && (rc = run_impl(ctx->pipe_sub[2 * k + 1], &pd, &b, &o, sd, true)) != BPMX_OK) return rc;
    }
    if (ctx->pipe_det) {
        /* the caller's stream completes after every chunk's detection */
        hipEvent_t done = ctx->pipe_ev[K];
        HIP_TRY(hipEventRecord(done, ctx->pipe_det));
        HIP_TRY(hipStreamWaitEvent(s, done, 0));
    }
    return BPMX_OK;
}

int bpmx_set_pipeline(bpmx_ctx *ctx, int chunks, int env_cus, int det_cus) {
    if (!ctx || ctx->root) return fail(BPMX_E_ARG, "bad context");
    if (chunks < 0 || chunks > 64 || env_cus < 0 || det_cus < 0) return fail(BPMX_E_ARG, "bad pipeline shape");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipDeviceSynchronize());
    if (env_cus != ctx->pipe_env_cus || det_cus != ctx->pipe_det_cus) {
        if (ctx->pipe_env) (void)hipStreamDestroy(ctx->pipe_env);
        if (ctx->pipe_det) (void)hipStreamDestroy(ctx->pipe_det);
        ctx->pipe_env = ctx->pipe_det = nullptr;
    }
    ctx->pipe_chunks = chunks;
    ctx->pipe_env_cus = env_cus;
    ctx->pipe_det_cus = det_cus;
    return BPMX_OK;
}

int bpmx_run_ordered(bpmx_ctx *ctx, const bpmx_params *P, const bpmx_batch *B, const bpmx_out *O,
                     const bpmx_peak_order *order, void *stream) {
    if (!order) return bpmx_run(ctx, P, B, O, stream);
    for (int s = 0; s < 2; ++s) {
        if ((order->cand[s] != nullptr) != (order->n_cand[s] != nullptr))
            return fail(BPMX_E_ARG, "bpmx_peak_order: cand and n_cand go together");
        if ((order->rank[s] != nullptr) != (order->use_rank[s] != nullptr))
            return fail(BPMX_E_ARG, "bpmx_peak_order: rank and use_rank go together");
    }
    if (P && (P->options & BPMX_OPT_STATS)) return fail(BPMX_E_ARG, "bpmx_run_ordered: no BPMX_OPT_STATS");
    return run_impl(ctx, P, B, O, stream, false, order);
}

int bpmx_run(bpmx_ctx *ctx, const bpmx_params *P, const bpmx_batch *B, const bpmx_out *O, void *stream) {
    int rc;
    if (ctx && P && B && O && !ctx->root && ctx->pipe_chunks >= 2 && B->n_files >= 2 * ctx->pipe_chunks &&
        (P->stages & BPMX_STAGE_ENVELOPE) && (P->stages & (BPMX_STAGE_FLOOR | BPMX_STAGE_PEAKS)) &&
        B->frame_offsets && B->pcm && O->env && O->n_troughs && O->n_peaks && O->flags)
        rc = run_pipelined(ctx, P, B, O, (hipStream_t)stream);
    else
        rc = run_impl(ctx, P, B, O, stream, false);
    if (rc == BPMX_OK && (P->options & BPMX_OPT_STATS)) {
        /* bpmx_stats waits for this context-owned event, not for the caller's
         * stream, which the caller may destroy in between */
        if (!ctx->stats_ev) HIP_TRY(hipEventCreateWithFlags(&ctx->stats_ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(ctx->stats_ev, (hipStream_t)stream));
    }
    return rc;
}

}  // extern "C"
