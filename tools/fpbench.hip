/*
 * fpbench.hip — phase timing for k_find_peaks on real envelopes.
 * Reads gpurun_out/env.bin (written by tools/dump_env.py: int64 F, int64 n,
 * then F*n f64 envelopes), times k_find_peaks for both signs.
 *   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/fpbench.hip -o tools/fpbench
 */
#define BPMX_STAMPS 1
#include "../bpm_analysis_amd/csrc/k_detect.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace bpmx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char **argv) {
    FILE *fp = fopen(argc > 1 ? argv[1] : "gpurun_out/env.bin", "rb");
    if (!fp) { printf("no env.bin\n"); return 1; }
    int64_t F, n;
    if (fread(&F, 8, 1, fp) != 1 || fread(&n, 8, 1, fp) != 1) return 1;
    std::vector<double> env((size_t)F * n);
    if (fread(env.data(), 8, env.size(), fp) != env.size()) return 1;
    fclose(fp);
    std::vector<int64_t> doff(F + 1), boff(F + 1);
    for (int64_t f = 0; f <= F; ++f) { doff[f] = f * n; boff[f] = f * ((n + 63) / 64); }
    std::vector<int32_t> active(F, 1);
    std::vector<double> qv((size_t)F * Q_SLOTS);
    for (int64_t f = 0; f < F; ++f) {
        std::vector<double> s(env.begin() + f * n, env.begin() + (f + 1) * n);
        std::sort(s.begin(), s.end());
        qv[f * Q_SLOTS + Q_TROUGH] = qv[f * Q_SLOTS + Q_PEAK] = s[(size_t)(0.1 * (n - 1))];
    }
    double *d_env, *d_bmx, *d_bmn, *d_qv;
    int64_t *d_doff, *d_boff, *d_out;
    int32_t *d_act, *d_cand, *d_nout;
    uint8_t *d_state;
    unsigned long long *d_st;
    CK(hipMalloc(&d_env, env.size() * 8));
    CK(hipMalloc(&d_bmx, (size_t)boff[F] * 8));
    CK(hipMalloc(&d_bmn, (size_t)boff[F] * 8));
    CK(hipMalloc(&d_qv, qv.size() * 8));
    CK(hipMalloc(&d_doff, (F + 1) * 8));
    CK(hipMalloc(&d_boff, (F + 1) * 8));
    CK(hipMalloc(&d_out, env.size() * 8));
    CK(hipMalloc(&d_act, F * 4));
    CK(hipMalloc(&d_cand, env.size() * 4));
    CK(hipMalloc(&d_nout, F * 4));
    CK(hipMalloc(&d_state, env.size()));
    CK(hipMalloc(&d_st, (size_t)F * 16 * 8));
    int32_t *d_vc, *d_fb, *d_sok, *d_scnt;
    double *d_cval, *d_vval, *d_outv;
    CK(hipMalloc(&d_vc, env.size() * 4));
    CK(hipMalloc(&d_fb, F * 4));
    CK(hipMalloc(&d_sok, F * 4));
    CK(hipMalloc(&d_scnt, (size_t)F * FPS_NW * 2 * 4));
    CK(hipMalloc(&d_cval, env.size() * 8));
    CK(hipMalloc(&d_vval, env.size() * 8));
    CK(hipMalloc(&d_outv, env.size() * 8));
    CK(hipMemcpy(d_env, env.data(), env.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_qv, qv.data(), qv.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_doff, doff.data(), (F + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_boff, boff.data(), (F + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_act, active.data(), F * 4, hipMemcpyHostToDevice));
    BlockStatArgs b;
    b.env = d_env; b.doff = d_doff; b.boff = d_boff; b.active = d_act; b.n_files = (int)F; b.bmax = d_bmx; b.bmin = d_bmn;
    hipLaunchKernelGGL(k_block_stats, dim3(F), dim3(256), 0, 0, b);
    for (double sg : {-1.0, 1.0}) {
        PeakArgs a;
        a.env = d_env; a.height = nullptr; a.doff = d_doff; a.boff = d_boff; a.active = d_act; a.bmax = d_bmx;
        a.bmin = d_bmn; a.qv = d_qv; a.qslot = sg < 0 ? Q_TROUGH : Q_PEAK; a.n_files = (int)F; a.distance = 15;
        a.sign = sg; a.cand = d_cand; a.state = d_state; a.out = d_out; a.nout = d_nout; a.run_out = nullptr;
        a.run_min = 0; a.stamps = d_st; a.vcand = d_vc; a.fallback = d_fb; a.only = nullptr; a.lds_nmax = INT64_MAX;
        a.flags = nullptr; a.tie_bit = 0;
        /* as in the pipeline: the trough launch scans and records, the peak
         * launch takes its lists; values beside the trough indices */
        a.cval = d_cval; a.vval = d_vval; a.scan_ok = d_sok; a.scan_cnt = d_scnt;
        a.outv = sg < 0 ? d_outv : nullptr;
        const bool lds = argc > 2 && argv[2][0] == 'l';
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(e0, 0));
            CK(hipMemset(d_st, 0, (size_t)F * 16 * 8));
            if (sg < 0) CK(hipMemset(d_sok, 0, F * 4));
            if (lds) hipLaunchKernelGGL(k_find_peaks_lds, dim3(F), dim3(FP_T), 0, 0, a);
            else hipLaunchKernelGGL(k_find_peaks, dim3(F), dim3(FP_T), 0, 0, a);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
        }
        std::vector<unsigned long long> st((size_t)F * 16);
        CK(hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost));
        std::vector<int32_t> no(F);
        CK(hipMemcpy(no.data(), d_nout, F * 4, hipMemcpyDeviceToHost));
        double sum[8] = {0}, tot = 0;
        for (int64_t f = 0; f < F; ++f)
            for (int k = 0; k < 8; ++k) sum[k] += (double)st[f * 16 + k];
        for (int k = 0; k < 8; ++k) tot += sum[k];
        long long np = 0;
        for (auto v : no) np += v;
        const char *names0[8] = {"tables", "maxima", "distance", "prominence", "compact", "(prom max wave)", "(prom mean wave)", "-"};
        const char *names1[8] = {"-", "extrema", "to LDS", "dist:rounds", "prom:walks", "compact", "dist:lists", "prom:prep"};
        const char **names = lds ? names1 : names0;
        printf("sign %+.0f: %.3f ms, %lld peaks; per-WG cycles %.0f\n", sg, best, np, tot / F);
        for (int k = 0; k < 8; ++k)
            if (sum[k] > 0) printf("   %-11s %10.0f  %5.1f%%\n", names[k], sum[k] / F, 100 * sum[k] / tot);
    }
    return 0;
}
