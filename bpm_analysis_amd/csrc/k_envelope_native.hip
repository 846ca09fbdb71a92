/*
 * k_envelope_native.hip — native mode (placeholder until the block-state
 * sosfiltfilt + Hilbert kernels land).
 */
#include "bpmx_native.h"

namespace bpmx {
int native_envelope(bpmx_ctx *, const bpmx_params *, const bpmx_batch *, const bpmx_out *, hipStream_t, int,
                    const std::vector<int64_t> &, const std::vector<int64_t> &, int64_t, const int64_t *,
                    const int64_t *, const int32_t *) {
    return fail(BPMX_E_ARG, "native mode is not available in this build");
}
}  // namespace bpmx
