/*
 * refbench.hip — phase timing of the reference-mode envelope (tools only):
 * k_ref_pick, then k_envelope_ref_t with s_memtime stamps (forward | backward
 * | rolling-mean chain, cycles of wave 0 of each workgroup), then
 * k_ref_env_mean; F x 60 s 44.1 kHz int16 mono, ds 146.
 *   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/refbench.hip -o tools/refbench
 */
#define BPMX_STAMPS 1
#include "../bpm_analysis_amd/csrc/k_envelope_ref.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
using namespace bpmx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char **argv) {
    const int F = argc > 1 ? atoi(argv[1]) : 1024;
    const int64_t frames = 2646000, ds = 146, nd = (frames + ds - 1) / ds;
    std::vector<int16_t> pcm((size_t)F * frames);
    unsigned s = 7;
    for (auto &v : pcm) { s = s * 1664525u + 1013904223u; v = (int16_t)(s >> 20); }
    std::vector<int64_t> foff(F + 1), doff(F + 1);
    for (int f = 0; f <= F; ++f) { foff[f] = (int64_t)f * frames; doff[f] = (int64_t)f * nd; }
    std::vector<int32_t> act(F, 1);
    void *dp; int64_t *dfo, *ddo; int32_t *da, *dch; double *scr, *env, *sums; unsigned long long *st;
    const size_t rows = (nd + 30 + 63) / 64 * 64;
    CK(hipMalloc(&dp, pcm.size() * 2)); CK(hipMalloc(&dfo, (F + 1) * 8)); CK(hipMalloc(&ddo, (F + 1) * 8));
    CK(hipMalloc(&da, F * 4)); CK(hipMalloc(&dch, F * 4)); CK(hipMalloc(&scr, rows * F * 8));
    CK(hipMalloc(&env, (size_t)F * nd * 8)); CK(hipMalloc(&sums, (size_t)F * nd * 8)); CK(hipMalloc(&st, (size_t)F * 16 * 8));
    CK(hipMemcpy(dp, pcm.data(), pcm.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dfo, foff.data(), (F + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(ddo, doff.data(), (F + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(da, act.data(), F * 4, hipMemcpyHostToDevice));
    EnvRefArgs a{};
    a.pcm = dp; a.foff = dfo; a.doff = ddo; a.active = da; a.n_files = F; a.dtype = BPMX_DT_I16; a.channels = 1;
    a.ds = (int32_t)ds; a.env_window = 30;
    const double b[5] = {0.0200833656, 0, -0.0401667311, 0, 0.0200833656}, aa[5] = {1, -3.5, 4.6, -2.7, 0.6};
    for (int i = 0; i < 5; ++i) { a.b[i] = b[i]; a.a[i] = aa[i]; }
    for (int i = 0; i < 4; ++i) a.zi[i] = 0.0;
    a.scratch = scr; a.env = env; a.y = nullptr; a.sums = sums; a.chain = dch; a.stamps = st;
    const dim3 gp((unsigned)((nd + 30 + 63) / 64), (unsigned)((F + 63) / 64)), g((F + 63) / 64);
    const dim3 gm((unsigned)((nd + 63) / 64), (unsigned)((F + 63) / 64));
    hipEvent_t e[4];
    for (auto &x : e) CK(hipEventCreate(&x));
    for (int it = 0; it < 2; ++it) {
        CK(hipEventRecord(e[0]));
        hipLaunchKernelGGL((k_ref_pick<BPMX_DT_I16, false>), gp, dim3(256), 0, 0, a);
        CK(hipEventRecord(e[1]));
        hipLaunchKernelGGL((k_envelope_ref_t<BPMX_DT_I16, false>), g, dim3(64), 0, 0, a);
        CK(hipEventRecord(e[2]));
        hipLaunchKernelGGL(k_ref_env_mean, gm, dim3(256), 0, 0, a);
        CK(hipEventRecord(e[3]));
        CK(hipEventSynchronize(e[3]));
    }
    float t[3];
    for (int i = 0; i < 3; ++i) CK(hipEventElapsedTime(&t[i], e[i], e[i + 1]));
    std::vector<unsigned long long> h((size_t)F * 16);
    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    double c[3] = {0, 0, 0};
    const int W = (F + 63) / 64;
    for (int w = 0; w < W; ++w) for (int k = 0; k < 3; ++k) c[k] += (double)h[(size_t)w * 16 + k] / W;
    printf("F %d nd %lld: pick %.3f ms, envelope %.3f ms, mean %.3f ms\n", F, (long long)nd, t[0], t[1], t[2]);
    printf("envelope phases (cycles, per step): forward %.0f (%.1f), backward %.0f (%.1f), chain %.0f (%.1f)\n",
           c[0], c[0] / (nd + 30), c[1], c[1] / (nd + 30), c[2], c[2] / nd);
    return 0;
}
