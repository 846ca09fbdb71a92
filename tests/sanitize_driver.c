/*
 * sanitize_driver.c — runs the CPU oracle (oracle/bpmx_oracle.c, test
 * infrastructure) under AddressSanitizer + UndefinedBehaviorSanitizer on
 * synthetic recordings and envelope edge cases (race detection /
 * sanitizers on the C restatement).  Built and run by
 * tests/test_oracle.py::test_oracle_under_sanitizers:
 *   gcc -fsanitize=address,undefined -fno-sanitize-recover=all -g -O1 ... tests/sanitize_driver.c -lm
 * Numerics are not checked here (the golden tests do that); any invalid access,
 * leak or UB aborts the run.
 */
#include "../oracle/bpmx_oracle.c"

#include <stdio.h>

/* bpm_analysis.py:1038-1044 at sr = 302 Hz */
static const double B302[5] = {0.7335490217285772, 0, -1.4670980434571543, 0, 0.7335490217285772};
static const double A302[5] = {1, 0.5483593718036774, -1.2760781922939408, -0.2863122443280344, 0.53940110028564};
static const double ZI302[4] = {-0.7335490217285773, -0.7335490217285773, 0.7335490217285772, 0.7335490217285772};
/* butter(2, [20, 150] / 22050, 'band', output='sos'); zi 0 */
static const double SOS44[12] = {8.465374494441103e-05, 1.6930748988882205e-04, 8.465374494441103e-05, 1,
                                 -1.9773752088985488, 0.9777429967935939,
                                 1, -2, 1, 1, -1.9963113905170433, 0.9963213432577561};
static const double SOSZI[4] = {0, 0, 0, 0};

static int detect_env(const double *env, int64_t n, const char *what) {
    bpmo_nf_params p = {15, 3020, 3, 0.1, 0.2, 4.0, 0.1};
    double *floor_v = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    int64_t *tr = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n / 2 + 2));
    int64_t *pk = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n / 2 + 2));
    int flags = 0;
    const int64_t nt = bpmo_noise_floor(env, n, &p, floor_v, tr, &flags);
    const int64_t np = bpmo_raw_peaks(env, n, floor_v, p.distance, 0.1, pk);
    printf("%-28s n=%8lld troughs=%5lld peaks=%5lld flags=%d\n", what, (long long)n, (long long)nt,
           (long long)np, flags);
    free(floor_v);
    free(tr);
    free(pk);
    return 0;
}

static void one_recording(uint64_t seed, int64_t frames, int32_t fs, int ch, int native) {
    int16_t *pcm = (int16_t *)malloc(sizeof(int16_t) * (size_t)(frames * ch));
    bpmo_synth(seed, frames, fs, ch, pcm);
    const int64_t ds = fs == 44100 ? 146 : 1;
    const int64_t nd = (frames + ds - 1) / ds;
    double *env = (double *)malloc(sizeof(double) * (size_t)nd);
    double *y = (double *)malloc(sizeof(double) * (size_t)nd);
    char what[64];
    if (!native) {
        const int64_t r = bpmo_preprocess_ref(pcm, 1, frames, ch, ds, B302, A302, ZI302, 30, y, env);
        snprintf(what, sizeof what, "reference %lld x %d", (long long)frames, ch);
        if (r > 0) detect_env(env, r, what);
        else printf("%-28s too short (padlen)\n", what);
    } else {
        double *yf = (double *)malloc(sizeof(double) * (size_t)frames);
        const int r = bpmo_sosfiltfilt(pcm, 1, frames, ch, SOS44, SOSZI, yf);
        snprintf(what, sizeof what, "native %lld x %d", (long long)frames, ch);
        if (r == 0) {
            for (int64_t j = 0; j < nd; ++j) y[j] = fabs(yf[j * ds]);
            bpmo_rolling_mean(y, nd, 30, 1, env);
            detect_env(env, nd, what);
        } else {
            printf("%-28s too short (padlen)\n", what);
        }
        free(yf);
    }
    free(env);
    free(y);
    free(pcm);
}

int main(void) {
    one_recording(1, 44100 * 20, 44100, 1, 0);
    one_recording(2, 44100 * 12 + 7, 44100, 2, 0);
    one_recording(3, 146 * 15, 44100, 1, 0);          /* Nd = 15: padlen */
    one_recording(4, 146 * 16 + 3, 44100, 1, 0);      /* smallest accepted */
    one_recording(5, 44100 * 10 + 1, 44100, 1, 1);
    one_recording(6, 10, 44100, 1, 1);                /* n <= 15: padlen */
    /* envelope edge cases: constant, tiny, one spike, ramps, windows longer than the recording */
    const int64_t sizes[] = {1, 2, 3, 16, 31, 500, 3019, 3021, 9000};
    for (size_t k = 0; k < sizeof sizes / sizeof sizes[0]; ++k) {
        const int64_t n = sizes[k];
        double *e = (double *)malloc(sizeof(double) * (size_t)n);
        for (int64_t i = 0; i < n; ++i) e[i] = 5.0;
        detect_env(e, n, "constant");
        for (int64_t i = 0; i < n; ++i) e[i] = (double)((i * 7919) % 101) + (i % 13 == 0 ? 300.0 : 0.0);
        detect_env(e, n, "pseudo-random + spikes");
        for (int64_t i = 0; i < n; ++i) e[i] = (double)i;
        detect_env(e, n, "ramp");
        free(e);
    }
    puts("SANITIZE OK");
    return 0;
}
