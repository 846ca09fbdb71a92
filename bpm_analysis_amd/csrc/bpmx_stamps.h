/*
 * bpmx_stamps.h — optional in-kernel phase timing for the tools/kbench
 * harness.  Only builds with -DBPMX_STAMPS define anything; the library never
 * does.
 */
#ifndef BPMX_STAMPS_H
#define BPMX_STAMPS_H

/* Optional in-kernel phase timing (tools/kbench.hip builds with -DBPMX_STAMPS;
 * the library never does): thread 0 accumulates s_memtime deltas per phase. */
#ifdef BPMX_STAMPS
#define STAMP_DECL unsigned long long _st_acc[16] = {0}, _st_t = __builtin_amdgcn_s_memtime();
#define STAMP(k)                                                                  \
    do {                                                                          \
        if (threadIdx.x == 0) {                                                   \
            unsigned long long _t = __builtin_amdgcn_s_memtime();                 \
            _st_acc[k] += _t - _st_t;                                             \
            _st_t = _t;                                                           \
        }                                                                         \
    } while (0)
#define STAMP_FLUSH(ptr)                                                          \
    do {                                                                          \
        if (threadIdx.x == 0 && (ptr))                                            \
            for (int _k = 0; _k < 16; ++_k) (ptr)[blockIdx.x * 16 + _k] = _st_acc[_k]; \
    } while (0)
#else
#define STAMP_DECL
#define STAMP(k) do {} while (0)
#define STAMP_FLUSH(ptr) do {} while (0)
#endif

#endif
