/*
 * k_bluestein.hip — the Hilbert transform of long recordings (native mode,
 * scipy.signal.hilbert as used by the north_star envelope |hilbert(y[::ds])|;
 * scipy/signal/_signaltools.py:2318) by Bluestein's chirp-z algorithm, for
 * every recording the fused in-LDS kernel (k_hilbert.hip) cannot hold.
 *
 * An N-point DFT of arbitrary N (C5's ragged lengths have large prime
 * factors) becomes a cyclic convolution of length L >= 2M - 1 (2^k or 3 * 2^k):
 *     X_k = c_k sum_n (x_n c_n) conj(c_(k-n)),   c_m = exp(-i pi m^2 / M),
 * computed as IFFT_L(FFT_L(x c) * FFT_L(b)) with b_m = conj(c_|m|) wrapped;
 * the inverse DFT uses conj(FFT_L(b)) (b is symmetric).  All recordings of
 * one (L, packing) group share two batched rocFFT plans
 * (forward, backward), so a ragged batch costs a handful of large batched
 * transforms instead of one small plan per distinct length.
 *
 * Even N is packed (the usual real-FFT trick): z_m = x_2m + i x_2m+1 over
 * M = N/2 points; between the forward and inverse DFTs one pass splits Z into
 * the real spectrum X, applies the Hilbert multiplier (-i X_k for
 * 0 < k < N/2, zero at 0 and N/2) and packs the half-length inverse, exactly
 * as k_hilbert_env's pointwise pass does.  Odd N runs unpacked over M = N.
 * The output is h = N * Im(analytic signal) (a C2R's scaling); k_native_env
 * then forms |y + i h/N| and the rolling mean.
 *
 *   k_blu_pre    a = z c (zero-padded to L); b (once per group geometry)
 *   rocFFT fwd   FFT(a) [, FFT(b)]
 *   k_blu_mul    FFT(a) * FFT(b)
 *   rocFFT bwd   -> L * (conv), read as Z_k = c_k conv_k
 *   k_blu_mid    Z -> X -> -i X -> packed G; a' = G conj(c) (zero-padded)
 *   rocFFT fwd, k_blu_mul (conj), rocFFT bwd
 *   k_blu_post   g_m = conj(c_m) conv_m / L -> h
 */
#include <map>
#include <mutex>
#include <tuple>

#include <rocfft/rocfft.h>

#include "bpmx_common.h"
#include "bpmx_kernels.h"
#include "bpmx_native.h"

namespace bpmx {

struct BluArgs {
    const double *yd;         /* decimated filtered signal, doff-indexed */
    double *hb;               /* out: N * Hilbert transform, doff-indexed */
    const int64_t *doff;
    const int32_t *files;     /* [nrec] recordings of the group */
    double2 *A, *B;           /* [nrec][L] work / FFT(b) */
    int32_t L, nrec, pack;
};

namespace {
/* c_m = exp(-i pi m^2 / M): m^2 reduced mod 2M exactly, then sincospi */
__device__ __forceinline__ double2 blu_chirp(int64_t m, int64_t M) {
    const int64_t r = (m * m) % (2 * M);
    double sn, cs;
    sincospi((double)r / (double)M, &sn, &cs);
    return make_double2(cs, -sn);
}
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cmulc(double2 a, double2 b) {   /* a * conj(b) */
    return make_double2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}
__device__ __forceinline__ double2 conj2(double2 a) { return make_double2(a.x, -a.y); }
__device__ __forceinline__ double2 add2(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 sub2(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 scale2(double2 a, double s) { return make_double2(a.x * s, a.y * s); }
}  // namespace

__global__ __launch_bounds__(256) void k_blu_pre(BluArgs A, int make_b) {
    const int r = blockIdx.y;
    const int f = A.files[r];
    const int64_t d0 = A.doff[f], N = A.doff[f + 1] - d0;
    const int64_t M = A.pack ? N / 2 : N, L = A.L;
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= L) return;
    const double *x = A.yd + d0;
    double2 *a = A.A + (int64_t)r * L;
    if (j < M) {
        const double2 z = A.pack ? make_double2(x[2 * j], x[2 * j + 1]) : make_double2(x[j], 0.0);
        a[j] = cmul(z, blu_chirp(j, M));
    } else {
        a[j] = make_double2(0.0, 0.0);
    }
    if (make_b) {
        double2 *b = A.B + (int64_t)r * L;
        b[j] = j < M ? conj2(blu_chirp(j, M)) : (j > L - M ? conj2(blu_chirp(L - j, M)) : make_double2(0.0, 0.0));
    }
}

__global__ __launch_bounds__(256) void k_blu_mul(BluArgs A, int conj_b) {
    const int r = blockIdx.y;
    const int64_t L = A.L, j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= L) return;
    double2 *a = A.A + (int64_t)r * L;
    const double2 b = A.B[(int64_t)r * L + j];
    a[j] = conj_b ? cmulc(a[j], b) : cmul(a[j], b);
}

/* forward DFT done (Z_k = c_k conv_k / L); Hilbert multiplier; inverse
 * pre-multiply.  Packed: one thread per pair (k, M - k), k <= M / 2. */
__global__ __launch_bounds__(256) void k_blu_mid(BluArgs A) {
    const int r = blockIdx.y;
    const int f = A.files[r];
    const int64_t N = A.doff[f + 1] - A.doff[f];
    const int64_t M = A.pack ? N / 2 : N, L = A.L;
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= L) return;
    double2 *a = A.A + (int64_t)r * L;
    const double invL = 1.0 / (double)L;
    if (j >= M) {                                            /* zero padding of the inverse's input */
        a[j] = make_double2(0.0, 0.0);
        return;
    }
    if (!A.pack) {                                           /* odd N: V_k = -i X_k (k < N/2), +i X_k (k > N/2) */
        const double2 X = scale2(cmul(blu_chirp(j, M), a[j]), invL);
        double2 V = j == 0 ? make_double2(0.0, 0.0) : (2 * j < N ? make_double2(X.y, -X.x) : make_double2(-X.y, X.x));
        a[j] = cmulc(V, blu_chirp(j, M));
        return;
    }
    if (2 * j > M) return;                                   /* the pair's other thread */
    const int64_t k = j, kp = M - j;                         /* kp == M stands for 0 (Z_M = Z_0) */
    const double2 Zk = scale2(cmul(blu_chirp(k, M), a[k]), invL);
    const double2 Zp = kp == M ? Zk : scale2(cmul(blu_chirp(kp, M), a[kp]), invL);
    /* X_k = (Z_k + conj Z_(M-k)) / 2 + t_k (Z_k - conj Z_(M-k)) / (2i),  t_k = exp(-2 pi i k / N) */
    auto spec = [&](int64_t q, double2 Zq, double2 Zr) -> double2 {
        double sn, cs;
        sincospi(2.0 * (double)q / (double)N, &sn, &cs);
        const double2 t = make_double2(cs, -sn);
        const double2 s = add2(Zq, conj2(Zr)), d = sub2(Zq, conj2(Zr));
        const double2 td = cmul(t, d);                      /* td / (2i) = (td.y, -td.x) / 2 */
        return make_double2(0.5 * (s.x + td.y), 0.5 * (s.y - td.x));
    };
    const double2 Xk = spec(k, Zk, Zp), Xp = spec(kp, Zp, Zk);
    /* W = -i X; zero at 0 and N/2 (k = 0 pairs with M) */
    const double2 Wk = k == 0 ? make_double2(0.0, 0.0) : make_double2(Xk.y, -Xk.x);
    const double2 Wp = (kp == M || kp == 0) ? make_double2(0.0, 0.0) : make_double2(Xp.y, -Xp.x);
    /* G_q = (W_q + conj W_(M-q)) + i e^(2 pi i q / N) (W_q - conj W_(M-q)) */
    auto pack = [&](int64_t q, double2 Wq, double2 Wr) -> double2 {
        double sn, cs;
        sincospi(2.0 * (double)q / (double)N, &sn, &cs);
        const double2 e = make_double2(-sn, cs);             /* i e^(2 pi i q / N) */
        return add2(add2(Wq, conj2(Wr)), cmul(e, sub2(Wq, conj2(Wr))));
    };
    a[k] = cmulc(pack(k, Wk, Wp), blu_chirp(k, M));
    if (kp < M && kp != k) a[kp] = cmulc(pack(kp, Wp, Wk), blu_chirp(kp, M));
}

__global__ __launch_bounds__(256) void k_blu_post(BluArgs A) {
    const int r = blockIdx.y;
    const int f = A.files[r];
    const int64_t d0 = A.doff[f], N = A.doff[f + 1] - d0;
    const int64_t M = A.pack ? N / 2 : N, L = A.L;
    const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (m >= M) return;
    const double2 g = scale2(cmulc(A.A[(int64_t)r * L + m], blu_chirp(m, M)), 1.0 / (double)L);
    double *h = A.hb + d0;
    if (A.pack) {
        h[2 * m] = g.x;
        h[2 * m + 1] = g.y;
    } else {
        h[m] = g.x;
    }
}

/* ---------------------------------------------------------------------- */
namespace {
struct C2cPlans {
    rocfft_plan fwd = nullptr, bwd = nullptr;
    size_t work = 0;
};
/* process-wide (contexts on any thread share plans): lookups and inserts under
 * g_c2c_mu; map nodes are never erased, so a returned pointer stays valid */
std::map<std::tuple<int, int64_t, int64_t>, C2cPlans> g_c2c;   /* (device, L, batch) */
std::mutex g_c2c_mu;

int rf_fail(const char *what, rocfft_status st) {
    return fail(BPMX_E_HIP, std::string(what) + " failed (rocfft status " + std::to_string((int)st) + ")");
}

int c2c_plans(int dev, int64_t L, int64_t batch, C2cPlans **out) {
    if (const int rc = rocfft_setup_once(); rc != BPMX_OK) return rc;
    const auto key = std::make_tuple(dev, L, batch);
    std::lock_guard<std::mutex> g(g_c2c_mu);
    auto it = g_c2c.find(key);
    if (it != g_c2c.end()) { *out = &it->second; return BPMX_OK; }
    C2cPlans p;
    const size_t len = (size_t)L;
    rocfft_status st = rocfft_plan_create(&p.fwd, rocfft_placement_inplace, rocfft_transform_type_complex_forward,
                                          rocfft_precision_double, 1, &len, (size_t)batch, nullptr);
    if (st != rocfft_status_success) return rf_fail("plan_create(c2c fwd)", st);
    st = rocfft_plan_create(&p.bwd, rocfft_placement_inplace, rocfft_transform_type_complex_inverse,
                            rocfft_precision_double, 1, &len, (size_t)batch, nullptr);
    if (st != rocfft_status_success) return rf_fail("plan_create(c2c bwd)", st);
    size_t w1 = 0, w2 = 0;
    rocfft_plan_get_work_buffer_size(p.fwd, &w1);
    rocfft_plan_get_work_buffer_size(p.bwd, &w2);
    p.work = std::max(w1, w2);
    *out = &g_c2c.emplace(key, p).first->second;
    return BPMX_OK;
}

int run_fft(bpmx_ctx *ctx, hipStream_t s, rocfft_plan plan, double2 *data, void *work, size_t wbytes,
            const char *label) {
    rocfft_execution_info info = nullptr;
    rocfft_execution_info_create(&info);
    rocfft_execution_info_set_stream(info, s);
    if (work) rocfft_execution_info_set_work_buffer(info, work, wbytes);
    void *io[1] = {data};
    Launch l(ctx, s, label);
    const rocfft_status st = rocfft_execute(plan, io, nullptr, info);
    rocfft_execution_info_destroy(info);
    if (st != rocfft_status_success) return rf_fail("rocfft_execute", st);
    return l.done();
}
}  // namespace

int bluestein_hilbert(bpmx_ctx *ctx, hipStream_t s, const double *yd, double *hb, const std::vector<int64_t> &doff,
                      const int64_t *d_doff, const std::vector<int32_t> &files) {
    if (files.empty()) return BPMX_OK;
    /* groups by (packing, L), in file order within a group */
    std::map<std::pair<int, int64_t>, std::vector<int32_t>> groups;
    for (int32_t f : files) {
        const int64_t N = doff[f + 1] - doff[f];
        const int pack = (N % 2) == 0;
        const int64_t M = pack ? N / 2 : N;
        /* L = 2^k or 3 * 2^k (both fast rocFFT lengths): ~1.2x the needed
         * 2M - 1 on average instead of ~1.4x, at most two groups per octave */
        int64_t L = 1;
        while (L < 2 * M - 1) L <<= 1;
        if ((L >> 2) * 3 >= 2 * M - 1 && L >= 4) L = (L >> 2) * 3;
        groups[{pack, L}].push_back(f);
    }
    /* host copies outlive the async uploads; the FFT(b) tables depend on the
     * group geometry only and are rebuilt when it changes */
    std::vector<int64_t> key;
    std::vector<int32_t> &hf = ctx->blu_files;
    hf.clear();
    size_t total = 0;
    for (auto &g : groups) {
        key.push_back(g.first.first);
        key.push_back(g.first.second);
        for (int32_t f : g.second) { key.push_back(doff[f + 1] - doff[f]); hf.push_back(f); }
        key.push_back(-1);
        total += (size_t)g.first.second * g.second.size();
    }
    int rc = BPMX_OK;
    bool grew = false;
    double2 *bufA = (double2 *)ctx->buf("blu_a", total * 16, &rc);
    double2 *bufB = (double2 *)ctx->buf("blu_b", total * 16, &rc, &grew);
    int32_t *d_files = (int32_t *)ctx->buf("blu_files", hf.size() * 4, &rc);
    if (rc != BPMX_OK) return rc;
    const bool make_b = grew || key != ctx->blu_key;
    ctx->blu_key.clear();                 /* set again only once every group's FFT(b) table is built */
    HIP_TRY(hipMemcpyAsync(d_files, hf.data(), hf.size() * 4, hipMemcpyHostToDevice, s));
    size_t off = 0, fo = 0;
    for (auto &g : groups) {
        const int64_t L = g.first.second;
        const int nrec = (int)g.second.size();
        C2cPlans *pl = nullptr;
        if ((rc = c2c_plans(ctx->device, L, nrec, &pl)) != BPMX_OK) return rc;
        void *work = pl->work ? ctx->buf("blu_work", pl->work, &rc) : nullptr;
        if (rc != BPMX_OK) return rc;
        BluArgs a;
        a.yd = yd; a.hb = hb; a.doff = d_doff; a.files = d_files + fo;
        a.A = bufA + off; a.B = bufB + off; a.L = (int32_t)L; a.nrec = nrec; a.pack = g.first.first;
        const dim3 grid((unsigned)((L + 255) / 256), (unsigned)nrec);
        LAUNCH(ctx, s, "k_blu_pre", k_blu_pre, grid, dim3(256), 0, s, a, make_b ? 1 : 0);
        if ((rc = run_fft(ctx, s, pl->fwd, a.A, work, pl->work, "blu_fft")) != BPMX_OK) return rc;
        if (make_b && (rc = run_fft(ctx, s, pl->fwd, a.B, work, pl->work, "blu_fft_b")) != BPMX_OK) return rc;
        LAUNCH(ctx, s, "k_blu_mul", k_blu_mul, grid, dim3(256), 0, s, a, 0);
        if ((rc = run_fft(ctx, s, pl->bwd, a.A, work, pl->work, "blu_ifft")) != BPMX_OK) return rc;
        LAUNCH(ctx, s, "k_blu_mid", k_blu_mid, grid, dim3(256), 0, s, a);
        if ((rc = run_fft(ctx, s, pl->fwd, a.A, work, pl->work, "blu_fft")) != BPMX_OK) return rc;
        LAUNCH(ctx, s, "k_blu_mul", k_blu_mul, grid, dim3(256), 0, s, a, 1);
        if ((rc = run_fft(ctx, s, pl->bwd, a.A, work, pl->work, "blu_ifft")) != BPMX_OK) return rc;
        LAUNCH(ctx, s, "k_blu_post", k_blu_post, grid, dim3(256), 0, s, a);
        off += (size_t)L * nrec;
        fo += nrec;
    }
    ctx->blu_key = key;
    return BPMX_OK;
}

}  // namespace bpmx
