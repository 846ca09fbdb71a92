/*
 * bpmx_synth.h — deterministic, integer-only synthetic heart-sound PCM.
 *
 * Shared verbatim by the device generator (bpmx.hip, kernel k_synth) and the
 * host generator (bpmx_synth_host, same .so), so a batch generated directly in
 * HBM is bit-identical to the one the CPU oracle sees.  Only integer
 * arithmetic is used: libm sin/exp are SIMD/ifunc-dispatched on x86 and may
 * differ in the last ulp between hosts, which would make "the same input"
 * differ between this container and the GPU box.
 *
 * Signal model (SURVEY.md §8(d) "Synthetic input"):
 *   - white-ish noise, sigma ~= 200 (Irwin-Hall sum of four 16-bit uniforms);
 *   - S1: 45 Hz tone under a (1-u^2)^4 bell of half-width 60 ms, amplitude 6000;
 *   - S2: 70 Hz tone, half-width 50 ms, amplitude 3500, 0.30*sqrt(RR) s after S1;
 *   - BPM ramps 75 -> 150 over the first half, 150 -> 90 over the second half;
 *   - +-2 % RR jitter per beat; clipped to int16.
 * The sine is a parabolic approximation; the waveform only has to look like a
 * heart-sound recording to the detector, not be a pure tone.
 */
#ifndef BPMX_SYNTH_H
#define BPMX_SYNTH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define BPMX_HD __host__ __device__
#else
#define BPMX_HD
#endif

#define BPMX_SYNTH_S1_HW_MS 60
#define BPMX_SYNTH_S2_HW_MS 50

BPMX_HD static inline uint64_t bpmx_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

BPMX_HD static inline int64_t bpmx_isqrt(int64_t v) {
    int64_t r = 0, bit = (int64_t)1 << 40;
    if (v <= 0) return 0;
    while (bit > v) bit >>= 2;
    while (bit != 0) {
        if (v >= r + bit) { v -= r + bit; r = (r >> 1) + bit; }
        else r >>= 1;
        bit >>= 2;
    }
    return r;
}

/* Beat onsets (frame indices) of file `seed`.  Returns the number of beats
 * written (<= cap).  Sequential by nature (each RR depends on the previous
 * onset), so the device runs it one lane per file. */
BPMX_HD static inline int bpmx_synth_beats(uint64_t seed, int64_t n_frames, int32_t fs,
                                           int64_t *s1, int64_t *s2, int cap) {
    int64_t t = (int64_t)fs * 300 / 1000;
    int64_t half = n_frames / 2;
    int k = 0;
    if (half < 1) half = 1;
    while (t < n_frames && k < cap) {
        int64_t bpm_m;                                  /* milli-BPM */
        if (t < half) bpm_m = 75000 + 75000 * t / half;
        else bpm_m = 150000 - 60000 * (t - half) / (n_frames - half > 0 ? n_frames - half : 1);
        int64_t rr = (int64_t)fs * 60000 / bpm_m;       /* frames */
        int64_t j = (int64_t)(bpmx_mix64(seed * 0x9E3779B97F4A7C15ull ^ ((uint64_t)k * 0xD1B54A32D192ED03ull)) % 4001) - 2000;
        rr = rr + rr * j / 100000;
        int64_t rr_ms = rr * 1000 / fs;
        int64_t d2 = bpmx_isqrt(rr_ms * 90) * fs / 1000; /* 0.30*sqrt(RR s) */
        s1[k] = t;
        s2[k] = t + d2;
        k++;
        t += rr > 1 ? rr : 1;
    }
    return k;
}

/* Parabolic sine of a Q32 phase, Q16 result in [-65536, 65536]. */
BPMX_HD static inline int64_t bpmx_psin(uint32_t ph) {
    int64_t x = (int64_t)(ph >> 15) & 0xFFFF;          /* position in the half cycle, Q16 */
    int64_t s = (4 * x * (65536 - x)) >> 16;
    return (ph & 0x80000000u) ? -s : s;
}

BPMX_HD static inline int64_t bpmx_burst(int64_t m, int64_t hw, int64_t freq, int32_t fs, int64_t amp) {
    if (m <= -hw || m >= hw) return 0;
    int64_t u = m * 65536 / hw;                        /* Q16 in (-1, 1) */
    int64_t t = 65536 - ((u * u) >> 16);
    int64_t t2 = (t * t) >> 16;
    int64_t w = (t2 * t2) >> 16;                       /* (1-u^2)^4, Q16 */
    int64_t mm = ((m % fs) + fs) % fs;
    uint32_t ph = (uint32_t)((((mm * freq) % fs) << 32) / fs);   /* Q32 phase of freq*m/fs */
    return (amp * ((w * bpmx_psin(ph)) >> 16)) >> 16;
}

/* One PCM sample (int16) of channel `ch` at frame n. */
BPMX_HD static inline int16_t bpmx_synth_sample(uint64_t seed, int ch, int64_t n, int32_t fs,
                                                const int64_t *s1, const int64_t *s2, int nb) {
    uint64_t h = bpmx_mix64((seed + 1) * 0x100000001B3ull ^ ((uint64_t)n * 2 + (uint64_t)ch) * 0xA24BAED4963EE407ull);
    int64_t u = (int64_t)(h & 0xFFFF) + (int64_t)((h >> 16) & 0xFFFF) + (int64_t)((h >> 32) & 0xFFFF) + (int64_t)(h >> 48);
    int64_t v = (u - 131070) * 200 / 37837;
    int64_t hw1 = (int64_t)fs * BPMX_SYNTH_S1_HW_MS / 1000;
    int64_t hw2 = (int64_t)fs * BPMX_SYNTH_S2_HW_MS / 1000;
    /* last beat whose S1 window has started */
    int lo = 0, hi = nb;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (s1[mid] - hw1 <= n) lo = mid + 1; else hi = mid;
    }
    int64_t a1 = ch ? 5250 : 6000, a2 = ch ? 3063 : 3500;
    for (int k = lo - 1; k >= 0 && k >= lo - 2; --k) {
        v += bpmx_burst(n - s1[k], hw1, 45, fs, a1);
        v += bpmx_burst(n - s2[k], hw2, 70, fs, a2);
    }
    if (v > 32767) v = 32767;
    if (v < -32768) v = -32768;
    return (int16_t)v;
}

#endif
