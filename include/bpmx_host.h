/*
 * bpmx_host.h — C ABI of the host-side beat stages (libbpmx_host.so, C++,
 * no GPU): what pixeru/bpm_analysis runs per file after the hot path, for the
 * batch path's host threads.
 *
 *   bpmx_beats  <- bpm_analysis.py:1734-1757 (analyze_wav_file stages 2-5):
 *                  _run_preliminary_pass (:1623-1652) -> PeakClassifier(...)
 *                  .classify_peaks() (:64-330) -> _refine_and_correct_peaks
 *                  (:1655-1698) -> calculate_bpm_series (:1463-1484)
 *
 * Inputs are the hot path's per-file outputs (bpmx.h: env, floor, raw peaks).
 * Outputs: the final beats, the smoothed BPM curve (beat times in s and BPM,
 * the rows of <base>_bpm_plot.csv before its NaN filter), the preliminary
 * pass' (start BPM, peak-BPM time, recovery end) and one label per raw peak.
 * Reentrant: no global state, callable from many host threads at once.
 */
#ifndef BPMX_HOST_H
#define BPMX_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BPMX_HOST_ABI_VERSION 1

enum bpmx_host_status {
    BPMX_HOST_OK = 0,
    BPMX_HOST_E_ARG = -1,        /* bad argument */
    BPMX_HOST_E_FEW_PEAKS = -2   /* < 2 raw peaks: the reference's refinement raises KeyError
                                    ('dynamic_noise_floor_series'); labels are still written */
};

/* labels per raw peak (tags_out) */
enum bpmx_beat_tag { BPMX_TAG_NONE = 0, BPMX_TAG_S1 = 1, BPMX_TAG_S2 = 2, BPMX_TAG_LONE_S1 = 3, BPMX_TAG_NOISE = 4 };

/* the DEFAULT_PARAMS keys the stages read (config.py), with the reference's
 * params.get() defaults applied by the caller */
typedef struct {
    double pairing_confidence_threshold, s1_s2_interval_cap_sec, s1_s2_interval_rr_fraction;
    double deviation_smoothing_factor;
    int64_t stability_history_window;
    double stability_confidence_floor, stability_confidence_ceiling;
    double s1_s2_boost_ratio, boost_amount_min, boost_amount_max, penalty_amount_min, penalty_amount_max;
    double s2_s1_ratio_low_bpm, s2_s1_ratio_high_bpm, contractility_bpm_low, contractility_bpm_high;
    double recovery_phase_duration_sec;
    double interval_penalty_start_factor, interval_penalty_full_factor, interval_max_penalty;
    int64_t enable_interval_penalty, cascade_reset_trigger_count;
    double min_bpm, max_bpm;
    double lone_s1_forward_check_pct, lone_s1_confidence_threshold, lone_s1_rhythm_weight, lone_s1_amplitude_weight;
    double rr_correction_threshold_pct, rr_correction_long_interval_pct;
    double penalty_waiver_strength_ratio, penalty_waiver_max_s2_s1_ratio;
    double output_smoothing_window_sec;
} bpmx_beat_params;

int bpmx_host_abi_version(void);

/* start_bpm_hint: NaN = None.  Caller-allocated outputs: final_out[n_peaks],
 * bpm_t_out / bpm_out[n_peaks], pass_out[3] (optional), tags_out[n_peaks]
 * (optional).  Returns BPMX_HOST_OK or a bpmx_host_status. */
int bpmx_beats(const double *env, int64_t n_env, const double *floor, const int64_t *peaks, int64_t n_peaks,
               int32_t sr, const bpmx_beat_params *params, double start_bpm_hint, int64_t *final_out,
               int64_t *n_final, double *bpm_t_out, double *bpm_out, int64_t *n_bpm, double *pass_out,
               int8_t *tags_out);

/* bpmx_beats over many recordings on `threads` host threads (a work queue of
 * files): per-file pointers and sizes, per-file status (bpmx_host_status);
 * pass_out is [n_files][3]. */
int bpmx_beats_batch(int32_t n_files, const double *const *env, const int64_t *n_env, const double *const *floor,
                     const int64_t *const *peaks, const int64_t *n_peaks, const int32_t *sr,
                     const bpmx_beat_params *params, double start_bpm_hint, int32_t threads,
                     int64_t *const *final_out, int64_t *n_final, double *const *bpm_t_out, double *const *bpm_out,
                     int64_t *n_bpm, double *pass_out, int8_t *const *tags_out, int32_t *status);

#ifdef __cplusplus
}
#endif

#endif /* BPMX_HOST_H */
