"""bpm_analysis_amd — MI355X-native preprocessing + detection path of pixeru/bpm_analysis.

Filter -> envelope -> dynamic noise floor -> raw peaks, as hand-written HIP
kernels for gfx950 behind a C ABI (include/bpmx.h, bpm_analysis_amd/libbpmx.so),
with the reference's function names on top (dropin.py) and a batch engine
(engine.py), and the host beat stages on top (beats.py: classifier, refinement,
BPM curve and metrics).  See DESIGN.md.
"""
from .config import DEFAULT_PARAMS  # noqa: F401
from .dropin import (_calculate_dynamic_noise_floor, analyze_batch, detect, find_raw_peaks,  # noqa: F401
                     patch_reference, preprocess_audio)
from .engine import Detector, Result, default_detector  # noqa: F401
from .beats import PeakClassifier, analyze_recording, analyze_wav_file  # noqa: F401

__all__ = ["DEFAULT_PARAMS", "preprocess_audio", "_calculate_dynamic_noise_floor", "find_raw_peaks",
           "analyze_batch", "detect", "patch_reference", "Detector", "Result", "default_detector",
           "PeakClassifier", "analyze_recording", "analyze_wav_file"]
