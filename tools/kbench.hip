/*
 * kbench.hip — standalone phase-timing harness for k_rolling_quantile.
 * Builds the kernel with -DBPMX_STAMPS (s_memtime deltas per phase, thread 0
 * of each workgroup) and prints the mean cycles per phase per workgroup.
 *   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/kbench.hip -o tools/kbench
 *   ./tools/kbench [files] [nd] [window]
 */
#define BPMX_STAMPS 1
#include "../bpm_analysis_amd/csrc/k_floor.hip"
#include "../bpm_analysis_amd/csrc/k_rollq_wm.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace bpmx;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main(int argc, char **argv) {
    int F = argc > 1 ? atoi(argv[1]) : 1024;
    int nd = argc > 2 ? atoi(argv[2]) : 18124;
    int W = argc > 3 ? atoi(argv[3]) : 3020;
    std::vector<double> dense((size_t)F * nd);
    std::vector<int64_t> doff(F + 1), tr((size_t)F * nd, 0);
    std::vector<int32_t> run(F, 1), allnan(F, 0);
    const bool verify = true;
    unsigned long long s = 12345;
    auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return (double)(s >> 11) / 9007199254740992.0; };
    for (int f = 0; f < F; ++f) {
        doff[f] = (int64_t)f * nd;
        int t = 20 + (int)(rnd() * 40);
        tr[(size_t)f * nd] = t;
        double *d = dense.data() + (size_t)f * nd;
        for (int i = 0; i < t; ++i) d[i] = __builtin_nan("");
        double v0 = 100 + 1900 * rnd();
        while (t < nd) {
            int len = 40 + (int)(rnd() * 80);
            double v1 = 100 + 1900 * rnd();
            for (int k = 0; k < len && t + k < nd; ++k) d[t + k] = v0 + (v1 - v0) / len * k;
            t += len;
            v0 = v1;
        }
    }
    doff[F] = (int64_t)F * nd;
    double *d_dense, *d_out;
    int64_t *d_doff, *d_tr;
    int32_t *d_run, *d_an;
    unsigned long long *d_st;
    CK(hipMalloc(&d_dense, dense.size() * 8));
    CK(hipMalloc(&d_out, dense.size() * 8));
    CK(hipMalloc(&d_doff, doff.size() * 8));
    CK(hipMalloc(&d_tr, tr.size() * 8));
    CK(hipMalloc(&d_run, F * 4));
    CK(hipMalloc(&d_an, F * 4));
    CK(hipMalloc(&d_st, (size_t)F * 16 * 8));
    CK(hipMemcpy(d_dense, dense.data(), dense.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_doff, doff.data(), doff.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_tr, tr.data(), tr.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_run, run.data(), F * 4, hipMemcpyHostToDevice));
    for (int T : {256}) {
        int cap = (W + T - 1 + 63) / 64 * 64;
        size_t lds = rollq_lds_bytes(T, cap);
        RollqArgs a;
        a.dense = d_dense; a.doff = d_doff; a.troughs = d_tr; a.run = d_run; a.n_files = F; a.window = W;
        a.min_periods = 3; a.cap = cap; a.q = 0.2; a.out = d_out; a.allnan = d_an; a.stamps = d_st;
        a.wm_max = 0; a.env = nullptr; a.ntr = nullptr;
        a.chunk = (int64_t)1 << 40;                    /* one chunk per recording (the fill pass is not timed) */
        CK(hipMalloc(&a.vfirst, F * 8));
        a.vlast = a.vfirst + F;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        float best = 1e9;
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipMemset(a.vfirst, 0x7F, F * 4));
            CK(hipMemset(a.vlast, 0xFF, F * 4));
            CK(hipEventRecord(e0, 0));
            if (cap <= 16 * 256) {
                CK(hipFuncSetAttribute((const void *)k_rolling_quantile<256, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                hipLaunchKernelGGL((k_rolling_quantile<256, 16>), dim3(F), dim3(256), lds, 0, a);
            } else {
                CK(hipFuncSetAttribute((const void *)k_rolling_quantile<256, 32>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                hipLaunchKernelGGL((k_rolling_quantile<256, 32>), dim3(F), dim3(256), lds, 0, a);
            }
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        std::vector<unsigned long long> st((size_t)F * 16);
        CK(hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost));
        double sum[16] = {0};
        for (int f = 0; f < F; ++f)
            for (int k = 0; k < 16; ++k) sum[k] += (double)st[(size_t)f * 16 + k];
        const char *names[16] = {"rank+scan", "ub", "scatter", "edges", "walk", "out", "-", "tile-head", "", "", "", "", "", "", "", ""};
        double tot = 0;
        for (int k = 0; k < 16; ++k) tot += sum[k];
        printf("T=%d cap=%d lds=%zu: %.3f ms; per-WG cycles (memtime) total %.0f\n", T, cap, lds, best, tot / F);
        for (int k = 0; k < 16; ++k)
            if (sum[k] > 0) printf("   %-10s %12.0f  %5.1f%%\n", names[k], sum[k] / F, 100.0 * sum[k] / tot);
    }
    {   /* wavelet-matrix kernel, fused interpolation from troughs (the library's final-floor launch):
         * pruned variant, then the unpruned one on the same input; outputs must agree bit for bit */
        std::vector<double> env((size_t)F * nd, 0.0);
        std::vector<int64_t> trs((size_t)F * nd, 0);
        std::vector<int32_t> ntr(F, 0);
        for (int f = 0; f < F; ++f) {
            int t = 20 + (int)(rnd() * 40), j = 0;
            while (t < nd && j < WM_TRMAX) {
                trs[(size_t)f * nd + j] = t;
                env[(size_t)f * nd + t] = 100 + 1900 * rnd();
                ++j;
                t += 40 + (int)(rnd() * 80);
            }
            ntr[f] = j;
        }
        double *d_env, *d_sorted, *d_out2;
        int64_t *d_trs;
        int32_t *d_ntr, *d_full;
        uint16_t *d_pos;
        CK(hipMalloc(&d_env, env.size() * 8));
        CK(hipMalloc(&d_trs, trs.size() * 8));
        CK(hipMalloc(&d_ntr, F * 4));
        CK(hipMalloc(&d_full, F * 4));
        CK(hipMalloc(&d_sorted, dense.size() * 8));
        CK(hipMalloc(&d_out2, dense.size() * 8));
        CK(hipMalloc(&d_pos, dense.size() * 2));
        CK(hipMemcpy(d_env, env.data(), env.size() * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_trs, trs.data(), trs.size() * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_ntr, ntr.data(), F * 4, hipMemcpyHostToDevice));
        for (int prune = 1; prune >= 0; --prune) {
            RollqArgs a;
            a.dense = d_dense; a.doff = d_doff; a.troughs = d_trs; a.run = d_run; a.n_files = F; a.window = W;
            a.min_periods = 3; a.cap = 0; a.q = 0.2; a.out = prune ? d_out : d_out2; a.allnan = d_an; a.stamps = d_st;
            a.wm_max = WM_MMAX; a.env = d_env; a.ntr = d_ntr;
            CK(hipMemset(d_st, 0, (size_t)F * 16 * 8));
            const size_t lds = wm_layout(nd, prune).total;
            const void *fn = prune ? (const void *)k_rollq_wm_t<true> : (const void *)k_rollq_wm_t<false>;
            CK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            float best = 1e9;
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipEventRecord(e0, 0));
                if (prune) hipLaunchKernelGGL(k_rollq_wm_t<true>, dim3(F), dim3(WM_T), lds, 0, a, d_pos, d_full);
                else hipLaunchKernelGGL(k_rollq_wm_t<false>, dim3(F), dim3(WM_T), lds, 0, a, d_pos, d_full);
                CK(hipGetLastError());
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
            }
            std::vector<unsigned long long> st((size_t)F * 16);
            CK(hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost));
            double sum[16] = {0};
            for (int f = 0; f < F; ++f)
                for (int k = 0; k < 16; ++k) sum[k] += (double)st[(size_t)f * 16 + k];
            const char *names[16] = {"load", "count", "scan", "exchange", "sorted-out", "build", "query", "compact", "p:tables", "p:hist", "p:prefix", "p:bstar", "p:thr", "p:keep", "-", "-"};
            double tot = 0;
            for (int k = 0; k < 16; ++k) tot += sum[k];
            std::vector<int32_t> fl(F);
            CK(hipMemcpy(fl.data(), d_full, F * 4, hipMemcpyDeviceToHost));
            int nfull = 0;
            for (int f = 0; f < F; ++f) nfull += fl[f];
            printf("k_rollq_wm_t<%d> lds=%zu: %.3f ms (4 reps best); per-WG cycles total %.0f; flagged full %d\n",
                   prune, lds, best, tot / F, prune ? nfull : -1);
            for (int k = 0; k < 16; ++k)
                if (sum[k] > 0) printf("   %-10s %12.0f  %5.1f%%\n", names[k], sum[k] / F, 100.0 * sum[k] / tot);
        }
        std::vector<double> o1(dense.size()), o2(dense.size());
        std::vector<int32_t> fl(F);
        CK(hipMemcpy(o1.data(), d_out, o1.size() * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(o2.data(), d_out2, o2.size() * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(fl.data(), d_full, F * 4, hipMemcpyDeviceToHost));
        long bad = 0, checked = 0;
        for (int f = 0; f < F; ++f) {
            if (fl[f]) continue;   /* the pruned launch left it to the unpruned variant */
            for (int i = 0; i < nd; ++i) {
                const double x = o1[(size_t)f * nd + i], y = o2[(size_t)f * nd + i];
                ++checked;
                if (!(x == y || (x != x && y != y))) ++bad;
            }
        }
        printf("pruned vs unpruned: %ld of %ld outputs differ\n", bad, checked);
    }
    return 0;
}
