/*
 * bpmx_native.h — native-mode (north_star ordering) envelope entry point.
 */
#ifndef BPMX_NATIVE_H
#define BPMX_NATIVE_H

#include <vector>

#include "bpmx_ctx.h"
#include "bpmx_kernels.h"

namespace bpmx {
int native_envelope(bpmx_ctx *ctx, const bpmx_params *P, const bpmx_batch *B, const bpmx_out *O, hipStream_t s,
                    int F, const std::vector<int64_t> &foff, const std::vector<int64_t> &doff, int64_t maxnd,
                    const int64_t *d_foff, const int64_t *d_doff, const int32_t *d_active,
                    const QuantArgs *qa = nullptr,    /* non-null: the fused Hilbert kernel also fills qa->qv */
                    const InitOutArgs *io = nullptr); /* non-null: k_native_carry resets the run's outputs */
/* k_bluestein.hip: hb = N * Hilbert transform of yd for the listed recordings */
/* rocfft_setup() exactly once per process (std::call_once), whatever thread gets there first */
int rocfft_setup_once();
/* k_longfft.hip: exact-length four-step Hilbert of long recordings */
bool longfft_supported(int64_t N);
int longfft_hilbert(bpmx_ctx *ctx, hipStream_t s, const double *yd, double *hb, const std::vector<int64_t> &doff,
                    const std::vector<int32_t> &files);
void longfft_free(bpmx_ctx *ctx);
int bluestein_hilbert(bpmx_ctx *ctx, hipStream_t s, const double *yd, double *hb, const std::vector<int64_t> &doff,
                      const int64_t *d_doff, const std::vector<int32_t> &files);
}

#endif
