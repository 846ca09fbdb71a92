/*
 * rqbench.hip — phase timing of the final-floor rolling quantile
 * (k_rollq_wm_t<true>) on the bench's own inputs (tools/dump_floor_inputs.py),
 * checked bit for bit against the library's floor.
 *   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off [-DVARIANT...] tools/rqbench.hip -o tools/rqbench
 *   python tools/dump_floor_inputs.py 1024 native /tmp/floor_in.bin && ./tools/rqbench /tmp/floor_in.bin
 * Diagnostic builds: -DRQ_STOP_PRUNE / -DRQ_STOP_SORT end the kernel after
 * the pruning / the sort (phase costs by difference, e.g. with rocprofv3
 * --pmc SQ_INSTS_VALU; no output check), -DRQ_DIAG_Q prints per-block
 * statistics of the output phase (need, partial members, trips).
 */
#define BPMX_STAMPS 1
#include "../bpm_analysis_amd/csrc/k_rollq_wm.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace bpmx;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main(int argc, char **argv) {
    const char *path = argc > 1 ? argv[1] : "/tmp/floor_in.bin";
    FILE *fh = fopen(path, "rb");
    if (!fh) { printf("cannot open %s\n", path); return 1; }
    int64_t hdr[2];
    if (fread(hdr, 8, 2, fh) != 2) return 1;
    const int F = (int)hdr[0];
    const int64_t nd = hdr[1], N = (int64_t)F * nd;
    std::vector<double> env(N), floor_ref(N);
    std::vector<int32_t> ntr(F);
    std::vector<int64_t> tr(N);
    if (fread(env.data(), 8, N, fh) != (size_t)N || fread(ntr.data(), 4, F, fh) != (size_t)F ||
        fread(tr.data(), 8, N, fh) != (size_t)N || fread(floor_ref.data(), 8, N, fh) != (size_t)N) {
        printf("short file\n");
        return 1;
    }
    fclose(fh);
    std::vector<int64_t> doff(F + 1);
    for (int f = 0; f <= F; ++f) doff[f] = (int64_t)f * nd;
    std::vector<int32_t> run(F, 1);
    double *d_env, *d_out;
    int64_t *d_doff, *d_tr;
    int32_t *d_run, *d_an, *d_ntr, *d_full;
    uint16_t *d_pos;
    unsigned long long *d_st;
    CK(hipMalloc(&d_env, N * 8));
    CK(hipMalloc(&d_out, N * 8));
    CK(hipMalloc(&d_doff, (F + 1) * 8));
    CK(hipMalloc(&d_tr, N * 8));
    CK(hipMalloc(&d_run, F * 4));
    CK(hipMalloc(&d_an, F * 4));
    CK(hipMalloc(&d_ntr, F * 4));
    CK(hipMalloc(&d_full, F * 4));
    CK(hipMalloc(&d_pos, N * 2));
    CK(hipMalloc(&d_st, (size_t)F * 16 * 8));
    CK(hipMemcpy(d_env, env.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_doff, doff.data(), (F + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_tr, tr.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_run, run.data(), F * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ntr, ntr.data(), F * 4, hipMemcpyHostToDevice));
    RollqArgs a;
    a.dense = nullptr; a.doff = d_doff; a.troughs = d_tr; a.run = d_run; a.n_files = F; a.window = 3020;
    a.min_periods = 3; a.cap = 0; a.q = 0.2; a.out = d_out; a.allnan = d_an; a.stamps = d_st;
    a.wm_max = WM_MMAX; a.env = d_env; a.ntr = d_ntr; a.wm_chunk = 0; a.wm_fail = nullptr; a.wm_pos_ch = nullptr;
    a.vfirst = a.vlast = nullptr;
    {   /* env at each trough, beside the troughs (the library's trough values) */
        std::vector<double> tvh(N, 0.0);
        for (int f = 0; f < F; ++f)
            for (int j = 0; j < ntr[f]; ++j) tvh[(size_t)f * nd + j] = env[(size_t)f * nd + tr[(size_t)f * nd + j]];
        double *d_tv;
        CK(hipMalloc(&d_tv, N * 8));
        CK(hipMemcpy(d_tv, tvh.data(), N * 8, hipMemcpyHostToDevice));
        a.tv = d_tv;
    }
    const size_t lds = std::max(wm_layout(nd, true).total, wm_layout(nd, false).total);   /* the unpruned fallback runs in the same workgroup */
    CK(hipFuncSetAttribute((const void *)k_rollq_wm_t<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
        CK(hipMemset(d_st, 0, (size_t)F * 16 * 8));
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k_rollq_wm_t<true>, dim3(F), dim3(WM_T), lds, 0, a, d_pos, d_full);
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
    const char *names[16] = {"load", "count", "scan", "exchange", "q:bounds", "build", "q:skip+out", "cmpct+wait",
                             "p:tables", "p:hist", "p:prefix", "p:bstar", "p:thr", "p:keep", "q:cursor", "q:collect"};
    double tot = 0;
    for (int k = 0; k < 16; ++k) tot += sum[k];
#ifdef RQ_DIAG_M
    {
        std::vector<unsigned long long> ms(F);
        for (int f = 0; f < F; ++f) ms[f] = st[(size_t)f * 16 + 13];
        std::sort(ms.begin(), ms.end());
        printf("kept samples m: min %llu p10 %llu p50 %llu p90 %llu p99 %llu max %llu\n", ms[0], ms[F / 10], ms[F / 2],
               ms[F * 9 / 10], ms[F * 99 / 100], ms[F - 1]);
    }
#endif
#ifdef RQ_DIAG_W
    {
        double a[16] = {0}, mx[16] = {0};
        for (int f = 0; f < F; ++f)
            for (int k = 0; k < 16; ++k) {
                a[k] += (double)st[(size_t)f * 16 + k];
                mx[k] = std::max(mx[k], (double)st[(size_t)f * 16 + k]);
            }
        printf("output phase cycles per wave (mean / max over workgroups):");
        for (int k = 0; k < 16; ++k) printf(" w%d %.0f/%.0f", k, a[k] / F, mx[k]);
        printf("\n");
    }
#endif
#ifdef RQ_DIAG_Q
    {
        double a[8] = {0};
        for (int f = 0; f < F; ++f)
            for (int k = 0; k < 8; ++k) a[k] += (double)st[(size_t)f * 16 + 8 + k];
        printf("wave 0 per block: need %.2f, partial members %.2f, collect trips %.2f, cursor trips %.2f, collected %.2f (%.0f blocks)\n",
               a[1] / a[0], a[2] / a[0], a[3] / a[0], a[4] / a[0], a[5] / a[0], a[0]);
    }
#endif
    std::vector<int32_t> fl(F);
    CK(hipMemcpy(fl.data(), d_full, F * 4, hipMemcpyDeviceToHost));
    int nfull = 0;
    for (int f = 0; f < F; ++f) nfull += fl[f];
    printf("k_rollq_wm_t<1> F=%d nd=%ld lds=%zu: %.4f ms (best of 5); per-WG cycles %.0f; flagged full %d\n", F,
           (long)nd, lds, best, tot / F, nfull);
    for (int k = 0; k < 16; ++k)
        if (sum[k] > 0) printf("   %-10s %12.0f  %5.1f%%\n", names[k], sum[k] / F, 100.0 * sum[k] / tot);
#if defined(RQ_STOP_PRUNE) || defined(RQ_STOP_SORT)
    return 0;                                                /* phase-truncated diagnostic build: no outputs */
#endif
    std::vector<double> o(N);
    CK(hipMemcpy(o.data(), d_out, N * 8, hipMemcpyDeviceToHost));
    long bad = 0, checked = 0;
    for (int f = 0; f < F; ++f) {
        if (fl[f]) continue;
        for (int64_t i = 0; i < nd; ++i) {
            const double x = o[(size_t)f * nd + i], y = floor_ref[(size_t)f * nd + i];
            ++checked;
            if (!(x == y || (x != x && y != y))) {
                if (bad < 5) printf("  mismatch f=%d i=%ld got %.17g want %.17g\n", f, (long)i, x, y);
                ++bad;
            }
        }
    }
    printf("vs library floor: %ld of %ld outputs differ\n", bad, checked);
    return bad ? 2 : 0;
}
