"""DEFAULT_PARAMS — the reference's parameter dict, same keys and values
(pixeru/bpm_analysis config.py:3-108), so callers can keep passing
``DEFAULT_PARAMS.copy()`` (gui.py:32, hugging-face-space/app.py:11).

Only eight keys reach the accelerated path:
downsample_factor, save_filtered_wav, min_peak_distance_sec,
peak_prominence_quantile, trough_prominence_quantile, noise_floor_quantile,
noise_window_sec, trough_rejection_multiplier.  The rest drive the host-side
classifier, corrections and reports of the reference and are carried through
unchanged.
"""

DEFAULT_PARAMS = dict(
    # preprocessing
    downsample_factor=300,
    save_filtered_wav=True,
    # feature detection
    min_peak_distance_sec=0.05,
    peak_prominence_quantile=0.1,
    trough_prominence_quantile=0.1,
    # noise floor
    noise_floor_quantile=0.20,
    noise_window_sec=10,
    trough_rejection_multiplier=4.0,
    # peak noise vetoing
    noise_confidence_threshold=0.6,
    trough_veto_multiplier=2.1,
    trough_noise_multiplier=3.0,
    strong_peak_override_ratio=6.0,
    # S1/S2 pairing and confidence
    pairing_confidence_threshold=0.50,
    s1_s2_interval_cap_sec=0.4,
    s1_s2_interval_rr_fraction=0.7,
    deviation_smoothing_factor=0.05,
    stability_history_window=20,
    stability_confidence_floor=0.60,
    stability_confidence_ceiling=1.25,
    s1_s2_boost_ratio=1.2,
    boost_amount_min=0.10,
    boost_amount_max=0.35,
    penalty_amount_min=0.10,
    penalty_amount_max=0.30,
    s2_s1_ratio_low_bpm=1.5,
    s2_s1_ratio_high_bpm=1.1,
    contractility_bpm_low=120.0,
    contractility_bpm_high=140.0,
    recovery_phase_duration_sec=120,
    interval_penalty_start_factor=1.0,
    interval_penalty_full_factor=1.4,
    interval_max_penalty=0.75,
    kickstart_check_threshold=0.3,
    kickstart_override_ratio=0.60,
    # rhythm plausibility
    min_bpm=40,
    max_bpm=240,
    rr_interval_max_decrease_pct=0.45,
    rr_interval_max_increase_pct=0.70,
    lone_s1_min_strength_ratio=0.30,
    lone_s1_forward_check_pct=0.50,
    lone_s1_confidence_threshold=0.50,
    lone_s1_rhythm_weight=0.65,
    lone_s1_amplitude_weight=0.35,
    # correction pass
    enable_correction_pass=False,
    rr_correction_threshold_pct=0.40,
    rr_correction_long_interval_pct=1.70,
    penalty_waiver_strength_ratio=4.0,
    penalty_waiver_max_s2_s1_ratio=2.5,
    # output / HRV / reporting
    output_smoothing_window_sec=5,
    hrv_window_size_beats=40,
    hrv_step_size_beats=5,
    plot_amplitude_scale_factor=250.0,
    plot_downsample_factor=1,
)
