/*
 * bpmx_xlane.h — full-wave (64-lane) register shifts without LDS: DPP row
 * rotates for the in-row part, v_permlane16_swap / v_permlane32_swap (gfx950)
 * for the row crossings.  shift_up(x, d): lane l gets lane l-d; shift_down:
 * lane l gets lane l+d; lanes with no source get an unspecified value (the
 * callers mask them).  Every lane of the wave must be active.
 * tools/xlane_check.hip verifies them against __shfl_up/__shfl_down.
 */
#ifndef BPMX_XLANE_H
#define BPMX_XLANE_H

#include <hip/hip_runtime.h>
#include <cstdint>

namespace bpmx {

/* rows (16 lanes) moved up / down by one: row r gets row r-1 / r+1 */
__device__ __forceinline__ uint32_t xl_rows_up(uint32_t w) {
    const auto p16 = __builtin_amdgcn_permlane16_swap(w, w, false, false);   /* [0]: rows 1,3 <- 0,2; [1]: rows 0,2 <- 1,3 */
    const auto p32 = __builtin_amdgcn_permlane32_swap(p16[1], p16[1], false, false);  /* [0]: rows 2,3 <- rows 0,1 of p16[1] */
    return (threadIdx.x & 48) == 32 ? p32[0] : p16[0];
}
__device__ __forceinline__ uint32_t xl_rows_down(uint32_t w) {
    const auto p16 = __builtin_amdgcn_permlane16_swap(w, w, false, false);
    const auto p32 = __builtin_amdgcn_permlane32_swap(p16[0], p16[0], false, false);  /* [1]: rows 0,1 <- rows 2,3 of p16[0] */
    return (threadIdx.x & 48) == 16 ? p32[1] : p16[1];
}

template <int D>
__device__ __forceinline__ uint32_t xl_up32(uint32_t x) {
    if constexpr (D == 1) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, false);      /* wave_shr:1 */
    } else if constexpr (D < 16) {
        const uint32_t w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x120 + D, 0xf, 0xf, false);  /* row_ror:D */
        const uint32_t z = xl_rows_up(w);
        return (int)(threadIdx.x & 15) >= D ? w : z;
    } else if constexpr (D == 16) {
        return xl_rows_up(x);
    } else {
        static_assert(D == 32, "shift 1..16 or 32");
        return __builtin_amdgcn_permlane32_swap(x, x, false, false)[0];
    }
}
template <int D>
__device__ __forceinline__ uint32_t xl_down32(uint32_t x) {
    if constexpr (D == 1) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xf, 0xf, false);      /* wave_shl:1 */
    } else if constexpr (D < 16) {
        const uint32_t w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x120 + 16 - D, 0xf, 0xf, false);  /* row_ror:16-D */
        const uint32_t z = xl_rows_down(w);
        return (int)(threadIdx.x & 15) < 16 - D ? w : z;
    } else if constexpr (D == 16) {
        return xl_rows_down(x);
    } else {
        static_assert(D == 32, "shift 1..16 or 32");
        return __builtin_amdgcn_permlane32_swap(x, x, false, false)[1];
    }
}
template <int D>
__device__ __forceinline__ double xl_up(double v) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint64_t r = (uint64_t)xl_up32<D>((uint32_t)u) | ((uint64_t)xl_up32<D>((uint32_t)(u >> 32)) << 32);
    return __longlong_as_double((long long)r);
}
template <int D>
__device__ __forceinline__ double xl_down(double v) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint64_t r = (uint64_t)xl_down32<D>((uint32_t)u) | ((uint64_t)xl_down32<D>((uint32_t)(u >> 32)) << 32);
    return __longlong_as_double((long long)r);
}

}  // namespace bpmx

#endif
