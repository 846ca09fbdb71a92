/*
 * hbench.hip — standalone phase timing of k_hilbert_env (s_memtime stamps,
 * thread 0 of each workgroup): load | fwd stage 0 | 1 | 2 | pointwise | inverse | |z| | rolling mean.
 *   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/hbench.hip -o tools/hbench
 *   ./tools/hbench [files] [nd]
 * Runs the plan with the direct, matrix-core and Rader odd-prime stages and
 * prints the largest envelope differences (relative to max |env|).
 */
#define BPMX_STAMPS 1
#define BPMX_QS_STAMPS 1
#include "../bpm_analysis_amd/csrc/k_hilbert.hip"

#include <cstdio>
#include <cstdlib>

using namespace bpmx;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

static double run(int F, int64_t nd, bool mfma, bool rader, std::vector<double> &y, std::vector<double> &env_out,
                  bool cprime = true) {
    HilbPlan P;
    std::vector<double2> tabs;
    size_t lds = 0;
    if (!hilbert_plan(nd, 30, &P, &tabs, &lds, mfma, rader, cprime)) { printf("no plan\n"); exit(1); }
    printf("nd %lld M %d stages", (long long)nd, P.M);
    for (int i = 0; i < P.ns; ++i) printf(" %d%s", P.rad[i], P.mf[i] ? "(mfma)" : P.rd[i] ? "(rader)" : P.cp[i] ? "(const)" : "");
    printf(" lds %zu\n", lds);
    std::vector<int64_t> doff(F + 1);
    for (int f = 0; f <= F; ++f) doff[f] = (int64_t)f * nd;
    std::vector<int32_t> act(F, 1);
    double *dy, *denv; int64_t *dd; int32_t *da; double2 *dt; unsigned long long *dst;
    CK(hipMalloc(&dy, y.size() * 8)); CK(hipMalloc(&denv, y.size() * 8)); CK(hipMalloc(&dd, (F + 1) * 8));
    CK(hipMalloc(&da, F * 4)); CK(hipMalloc(&dt, tabs.size() * 16)); CK(hipMalloc(&dst, (size_t)F * 16 * 8));
    CK(hipMemcpy(dy, y.data(), y.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dd, doff.data(), (F + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(da, act.data(), F * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dt, tabs.data(), tabs.size() * 16, hipMemcpyHostToDevice));
    HilbArgs a{dy, dd, da, 0, F, dt, denv, dst};
    double *dqv = nullptr;
    if (getenv("HB_Q")) {                       /* the library's one native-mode level (q = 0.1) */
        CK(hipMalloc(&dqv, (size_t)F * Q_SLOTS * 8));
        a.q.env = denv; a.q.doff = dd; a.q.active = da; a.q.n_files = F; a.q.qv = dqv;
        a.q.n_levels = 1; a.q.q[0] = 0.1; a.q.slot[0] = 1; a.q.skip_le = QR_MAX;
    }
    CK(hipFuncSetAttribute((const void *)k_hilbert_env, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(k_hilbert_env, dim3(F), dim3(HB_T), lds, 0, a, P);
    CK(hipDeviceSynchronize());
    const int R = 10;
    CK(hipMemset(dst, 0, (size_t)F * 16 * 8));
    CK(hipEventRecord(e0));
    for (int it = 0; it < R; ++it) hipLaunchKernelGGL(k_hilbert_env, dim3(F), dim3(HB_T), lds, 0, a, P);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> st((size_t)F * 16);
    CK(hipMemcpy(st.data(), dst, st.size() * 8, hipMemcpyDeviceToHost));
    env_out.resize(y.size());
    CK(hipMemcpy(env_out.data(), denv, y.size() * 8, hipMemcpyDeviceToHost));
    if (dqv) {
        std::vector<unsigned long long> qs((size_t)8 * 4096);
        CK(hipMemcpyFromSymbol(qs.data(), HIP_SYMBOL(qs_dbg), qs.size() * 8));
        double qa[8] = {0};
        const int nf = F < 4096 ? F : 4096;
        for (int f = 0; f < nf; ++f) for (int k = 0; k < 8; ++k) qa[k] += (double)qs[(size_t)f * 8 + k] / nf;
        printf("select phases (cycles): vary %.0f hist0 %.0f digit-hist %.0f scan %.0f gather %.0f final %.0f\n",
               qa[0], qa[1], qa[2], qa[3], qa[4], qa[5]);
    }
    double acc[12] = {0};
    for (int f = 0; f < F; ++f) for (int k = 0; k < 12; ++k) acc[k] += (double)st[(size_t)f * 16 + k];
    printf("kernel %.4f ms;  mean cycles per workgroup (s_memtime):", ms / R);
    const char *nm[12] = {"load", "fwd0", "fwd1", "fwd2", "pointwise", "inverse", "mag", "quantiles", "rollsum", "rm:barrier", "stage", "store"};
    double tot = 0;
    for (int k = 0; k < 12; ++k) tot += acc[k] / F;
    for (int k = 0; k < 12; ++k) printf(" %s %.0f (%.1f%%)", nm[k], acc[k] / F, 100.0 * acc[k] / F / tot);
    printf("\n");
    CK(hipFree(dy)); CK(hipFree(denv)); CK(hipFree(dd)); CK(hipFree(da)); CK(hipFree(dt)); CK(hipFree(dst));
    if (dqv) CK(hipFree(dqv));
    return ms / R;
}

int main(int argc, char **argv) {
    const int F = argc > 1 ? atoi(argv[1]) : 1024;
    const int64_t nd = argc > 2 ? atoll(argv[2]) : 18124;
    std::vector<double> y((size_t)F * nd);
    unsigned long long s = 1;
    for (auto &v : y) { s = s * 6364136223846793005ull + 1442695040888963407ull; v = (double)(s >> 11) / 9007199254740992.0 - 0.5; }
    std::vector<double> e0, e1, e2, e3;
    run(F, nd, false, false, y, e0, false);
    run(F, nd, true, false, y, e1, false);
    run(F, nd, true, true, y, e2, false);
    run(F, nd, true, true, y, e3, true);
    double mx = 0, d = 0, d2 = 0, d3 = 0;
    for (size_t i = 0; i < e0.size(); ++i) {
        mx = fmax(mx, fabs(e0[i]));
        d = fmax(d, fabs(e0[i] - e1[i]));
        d2 = fmax(d2, fabs(e0[i] - e2[i]));
        d3 = fmax(d3, fabs(e0[i] - e3[i]));
    }
    printf("max |env_direct - env_X| / max|env|: mfma %.3e, rader %.3e, rader + const primes %.3e\n", d / mx,
           d2 / mx, d3 / mx);
    return 0;
}
