/*
 * bpmx_ctx.h — host-side context shared by the bpmx translation units.
 */
#ifndef BPMX_CTX_H
#define BPMX_CTX_H

#include <hip/hip_runtime.h>

#include <map>
#include <string>
#include <vector>

#include "../../include/bpmx.h"

namespace bpmx {
int fail(int code, const std::string &msg);
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess)                                                                \
            return bpmx::fail(BPMX_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

struct bpmx_ctx {
    int device = 0;
    /* pipelined runs (bpmx_set_pipeline): per chunk slot one context for the
     * envelope stage and one for detection, each with its own scratch and
     * geometry; they profile into the root context */
    bpmx_ctx *root = nullptr;
    int pipe_chunks = 0, pipe_env_cus = 0, pipe_det_cus = 0;
    std::vector<bpmx_ctx *> pipe_sub;              /* [2 * chunks]: env, det per slot */
    hipStream_t pipe_env = nullptr, pipe_det = nullptr;
    std::vector<hipEvent_t> pipe_ev;               /* [chunks + 1]: envelope k done, start fork */
    bpmx_ctx *pr() { return root ? root : this; }
    void *lf = nullptr;                            /* k_longfft.hip's plan state (LfHost) */
    std::map<std::string, std::pair<void *, size_t>> bufs;
    std::vector<int64_t> g_key;   /* geometry of the last upload */
    /* native-mode block-state tables (host copies back the async uploads) */
    std::vector<int64_t> nat_key;
    std::vector<double> nat_tab;
    std::vector<int64_t> blu_key;     /* Bluestein group geometry of the FFT(b) tables in "blu_b" */
    std::vector<int32_t> blu_files;   /* host copy of the Bluestein groups' file lists */
    std::vector<int32_t> nat_fused;   /* per-file: envelope done by the fused Hilbert kernel (host copy outlives async uploads) */
    std::vector<int32_t> nat_fyrec;   /* per-file: yd made inside k_hilbert_env (k_native_yd skips its tiles) */
    std::vector<int64_t> nat_boff;              /* block offsets | per-file tile offsets */
    std::vector<int64_t> nat_tkey;              /* tile-list geometry key */
    std::vector<char> nat_tiles;                /* host copy of the tile list */
    bool nat_tiles_dirty = false;
    bool nat_tab_dirty = false;
    std::vector<double> nat_ttab;               /* tail tables of k_native_carry (host copy) */
    std::vector<double> nat_tkey2;              /* their key: the sos coefficients and zi */
    bool nat_ttab_dirty = false;
    bool prof = false;
    hipEvent_t stats_ev = nullptr;               /* recorded after the last run with BPMX_OPT_STATS */
    struct Rec { std::string name; hipEvent_t a, b; };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    std::string prof_only;              /* bpmx_profile_only: record this label only (empty: all) */
    std::map<std::string, std::pair<long, double>> totals;
    /* side streams for the native-mode rocFFT runs (one plan per distinct Nd:
     * small, latency-bound executions that overlap when spread out) */
    static constexpr int NSIDE = 4;
    hipStream_t side[NSIDE] = {};
    hipEvent_t side_fork = nullptr, side_join[NSIDE] = {};
    std::vector<hipEvent_t> ref_ev;   /* reference mode: row chunk k gathered (side stream) */
    bool ref_events(size_t n) {
        while (ref_ev.size() < n) {
            hipEvent_t e;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return false;
            ref_ev.push_back(e);
        }
        return true;
    }
    bool side_ready() {
        if (side[0]) return true;
        if (root) {                     /* pipeline sub-contexts share the root context's side streams */
            if (!root->side_ready()) return false;
            for (int i = 0; i < NSIDE; ++i) { side[i] = root->side[i]; side_join[i] = root->side_join[i]; }
            side_fork = root->side_fork;
            return true;
        }
        for (int i = 0; i < NSIDE; ++i) {
            if (hipStreamCreateWithFlags(&side[i], hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&side_join[i], hipEventDisableTiming) != hipSuccess)
                return false;
        }
        return hipEventCreateWithFlags(&side_fork, hipEventDisableTiming) == hipSuccess;
    }

    /* grow-only device scratch; *grew (optional) reports a fresh allocation,
     * whose contents the caller must re-upload */
    void *buf(const std::string &name, size_t bytes, int *rc, bool *grew = nullptr) {
        auto &e = bufs[name];
        if (grew) *grew = false;
        if (e.second < bytes) {
            if (grew) *grew = true;
            if (e.first) (void)hipFree(e.first);
            e.first = nullptr;
            e.second = 0;
            size_t want = bytes + bytes / 8 + 256;
            if (hipMalloc(&e.first, want) != hipSuccess) {
                e.first = nullptr;
                *rc = bpmx::fail(BPMX_E_HIP, "hipMalloc failed for scratch '" + name + "' (" + std::to_string(want) + " B)");
                return nullptr;
            }
            e.second = want;
        }
        return e.first;
    }
    hipEvent_t ev() {
        if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
        hipEvent_t e;
        (void)hipEventCreate(&e);
        return e;
    }
};

namespace bpmx {

/* one kernel launch, optionally bracketed by events for bpmx_profile */
struct Launch {
    bpmx_ctx *ctx;
    hipStream_t s;
    const char *name;
    hipEvent_t a = nullptr, b = nullptr;
    bool on() const { return ctx->prof && (ctx->prof_only.empty() || ctx->prof_only == name); }
    Launch(bpmx_ctx *c, hipStream_t st, const char *n) : ctx(c->pr()), s(st), name(n) {
        if (on()) { a = ctx->ev(); (void)hipEventRecord(a, s); }
    }
    int done() {
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return fail(BPMX_E_HIP, std::string("launch of ") + name + ": " + hipGetErrorString(e));
        if (on()) {
            b = ctx->ev();
            (void)hipEventRecord(b, s);
            ctx->recs.push_back({name, a, b});
        }
        return BPMX_OK;
    }
};

}  // namespace bpmx

#define LAUNCH(ctx, stream, name, ...)                \
    do {                                              \
        bpmx::Launch _l(ctx, stream, name);           \
        hipLaunchKernelGGL(__VA_ARGS__);              \
        int _rc = _l.done();                          \
        if (_rc != BPMX_OK) return _rc;               \
    } while (0)

#endif
