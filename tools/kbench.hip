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
    CK(hipMalloc(&d_st, (size_t)F * 8 * 8));
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
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        float best = 1e9;
        for (int rep = 0; rep < 4; ++rep) {
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
        std::vector<unsigned long long> st((size_t)F * 8);
        CK(hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost));
        double sum[8] = {0};
        for (int f = 0; f < F; ++f)
            for (int k = 0; k < 8; ++k) sum[k] += (double)st[(size_t)f * 8 + k];
        const char *names[8] = {"rank+scan", "ub", "scatter", "edges", "walk", "out", "-", "tile-head"};
        double tot = 0;
        for (int k = 0; k < 8; ++k) tot += sum[k];
        printf("T=%d cap=%d lds=%zu: %.3f ms; per-WG cycles (memtime) total %.0f\n", T, cap, lds, best, tot / F);
        for (int k = 0; k < 8; ++k)
            if (sum[k] > 0) printf("   %-10s %12.0f  %5.1f%%\n", names[k], sum[k] / F, 100.0 * sum[k] / tot);
    }
    {   /* wavelet-matrix kernel */
        RollqArgs a;
        a.dense = d_dense; a.doff = d_doff; a.troughs = d_tr; a.run = d_run; a.n_files = F; a.window = W;
        a.min_periods = 3; a.cap = 0; a.q = 0.2; a.out = d_out; a.allnan = d_an; a.stamps = d_st; a.wm_max = WM_MMAX;
        a.env = nullptr; a.ntr = nullptr;
        double *d_sorted;
        CK(hipMalloc(&d_sorted, dense.size() * 8));

        CK(hipMemset(d_st, 0, (size_t)F * 8 * 8));
        const size_t lds = wm_lds_bytes(nd);
        CK(hipFuncSetAttribute((const void *)k_rollq_wm, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        float best = 1e9;
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k_rollq_wm, dim3(F), dim3(WM_T), lds, 0, a, d_sorted);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        std::vector<unsigned long long> st((size_t)F * 8);
        CK(hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost));
        double sum[8] = {0};
        for (int f = 0; f < F; ++f)
            for (int k = 0; k < 8; ++k) sum[k] += (double)st[(size_t)f * 8 + k];
        const char *names[8] = {"load", "count", "scan", "exchange", "sorted-out", "build", "query", "-"};
        double tot = 0;
        for (int k = 0; k < 8; ++k) tot += sum[k];
        printf("k_rollq_wm lds=%zu: %.3f ms (4 reps best); per-WG cycles total %.0f\n", lds, best, tot / F);
        for (int k = 0; k < 8; ++k)
            if (sum[k] > 0) printf("   %-10s %12.0f  %5.1f%%\n", names[k], sum[k] / F, 100.0 * sum[k] / tot);
    }
    return 0;
}
