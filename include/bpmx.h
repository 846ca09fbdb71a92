/*
 * bpmx.h — C ABI of the MI355X-native heartbeat preprocessing + detection path.
 *
 * One shared library (bpm_analysis_amd/libbpmx.so, HIP for gfx950) behind the
 * reference's own operator surface for this path.  The reference has no
 * plugin/FFI layer of its own (pure Python); these entry points
 * replace, one for one, the computation inside:
 *
 *   bpmx_run(stages=ENVELOPE)  <- bpm_analysis.py:1007-1062  preprocess_audio
 *                                 (wavfile.read result -> mean(axis=1) -> [::ds]
 *                                  -> butter/filtfilt -> |x| rolling mean)
 *   bpmx_run(stages=FLOOR)     <- bpm_analysis.py:1064-1117  _calculate_dynamic_noise_floor
 *   bpmx_run(stages=PEAKS)     <- bpm_analysis.py:223-229    PeakClassifier._find_raw_peaks
 *   bpmx_run(stages=ALL)       <- the three above in sequence, as analyze_wav_file
 *                                 runs them (bpm_analysis.py:1731-1732, :89)
 *   bpmx_synth / bpmx_synth_host   deterministic synthetic recordings (bench/tests)
 *
 * Plain C types only.  PCM and result arrays are DEVICE pointers (HBM); the
 * per-file frame offsets are a HOST array.  A batch shares one sample rate,
 * dtype and channel count; lengths may be ragged.  Filter coefficients
 * (butter / lfilter_zi / sosfilt_zi) are designed on the host exactly as the
 * reference designs them and passed in bpmx_params.
 *
 * Thread-safety: one bpmx_ctx per thread (or per stream); bpmx_last_error is
 * thread-local.  Calls may come from a non-main thread (gui.py:181-183).
 */
#ifndef BPMX_H
#define BPMX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BPMX_ABI_VERSION 2

/* sample formats of scipy.io.wavfile.read (bpm_analysis.py:1014) */
enum bpmx_dtype { BPMX_DT_U8 = 0, BPMX_DT_I16 = 1, BPMX_DT_I32 = 2, BPMX_DT_F32 = 3, BPMX_DT_F64 = 4 };

/* REFERENCE: the shipped pipeline, bit-exact (stride pick, b/a filtfilt at the
 *            decimated rate, rolling-mean envelope; bpm_analysis.py:1031-1054).
 * NATIVE:    the north_star ordering (sosfiltfilt at the native rate -> pick
 *            -> |Hilbert| -> rolling mean); envelope within 1e-9 relative of the
 *            scipy composition, detection stages identical. */
enum bpmx_mode { BPMX_MODE_REFERENCE = 0, BPMX_MODE_NATIVE = 1 };

enum bpmx_stage {
    BPMX_STAGE_ENVELOPE = 1, /* PCM -> env (and y)        */
    BPMX_STAGE_FLOOR = 2,    /* env -> floor, troughs     */
    BPMX_STAGE_PEAKS = 4,    /* env, floor -> raw peaks   */
    BPMX_STAGE_ALL = 7
};

/* return codes */
enum bpmx_status {
    BPMX_OK = 0,
    BPMX_E_ARG = -1,     /* bad argument (message in bpmx_last_error) */
    BPMX_E_HIP = -2,     /* HIP runtime error */
    BPMX_E_LIMIT = -3,   /* a size exceeds what the kernels support */
    BPMX_E_NODEV = -4    /* no usable gfx950 device */
};

/* per-file result flags (bpmx_out.flags) */
enum bpmx_file_flag {
    BPMX_F_STATIC_FLOOR = 1, /* < 5 troughs: constant quantile floor, troughs unsanitised (:1073-1077) */
    BPMX_F_DRAFT_FLOOR = 2,  /* <= 2 sanitised troughs: draft floor kept (:1107-1110) */
    BPMX_F_NAN_FLOOR = 4,    /* all-NaN floor replaced by quantile(env, 0.1) (:1113-1115) */
    BPMX_F_TOO_SHORT = 8,    /* Nd <= 15: scipy filtfilt raises ValueError; no outputs (its slices of the
                                output arrays are left as they were; counts are 0) */
    BPMX_F_BAD_WINDOW = 16,  /* noise_window < min_periods and >= 5 troughs: pandas rolling() raises
                                ValueError (:1085); floor/peaks of this recording are not meaningful */
    /* find_peaks' distance filter visits candidates in np.argsort(height) order
     * (scipy/signal/_peak_finding.py:976-978), which is unstable: for equal
     * heights the order is numpy's implementation detail (x86-simd-sort on
     * AVX-512, introsort elsewhere).  bpmx keeps the stable order (the later
     * index first among equals) and sets these bits exactly when that choice
     * decided a removal: some candidate was removed by an equal-height kept one
     * with no strictly higher kept one within `distance`.  Without the bit the
     * indices are those of every argsort order, so the reference's; with it
     * they may differ from the reference's on that machine. */
    BPMX_F_TROUGH_TIE = 32,  /* in the trough search find_peaks(-env) (:1070) */
    BPMX_F_PEAK_TIE = 64,    /* in the raw-peak search find_peaks(env, height=floor) (:227) */
    /* the distance filter of that search visited the candidates in the order
     * the caller supplied (bpmx_run_ordered: np.argsort of the heights, as
     * scipy's _select_by_peak_distance does); the matching TIE bit is then
     * never set, since the order is the reference's and nothing is left open */
    BPMX_F_TROUGH_ORDERED = 128,
    BPMX_F_PEAK_ORDERED = 256
};

enum bpmx_option {
    BPMX_OPT_ROLLQ_MERGE = 1, /* force the sorted-union rolling quantile (test/diagnostic; default picks the
                                 wavelet-matrix kernel for recordings of <= 18432 decimated samples) */
    BPMX_OPT_NATIVE_F64 = 2,  /* native mode: f64 VALU block projections instead of the exact-integer
                                 matrix-core kernel (test/diagnostic) */
    BPMX_OPT_HILBERT_ROCFFT = 4, /* native mode: rocFFT R2C/C2R Hilbert instead of the fused in-LDS transform
                                    (test/diagnostic; recordings the fused kernel cannot plan always use it) */
    BPMX_OPT_DRAFT_FULL = 8,     /* compute the draft floor (first rolling quantile) in full for every recording
                                    instead of deciding troughs from its bounds first (test/diagnostic) */
    BPMX_OPT_ROLLQ_NOPRUNE = 16, /* wavelet-matrix rolling quantile over every sample, without first dropping
                                    the samples no window's quantile can reach (test/diagnostic) */
    BPMX_OPT_DRAFT_GLOBAL_RANK = 32, /* draft-floor bounds from the recording-wide segment order even for
                                       recordings of > 512 troughs (test/diagnostic; default ranks per window) */
    BPMX_OPT_ROLLQ_GLOBAL = 64,  /* force the global-memory sorted-union rolling quantile (test/diagnostic;
                                    default: only for windows beyond the LDS kernel on long recordings) */
    BPMX_OPT_NATIVE_DMA = 128,   /* native mode, int16 mono without the matrix-core path: the LDS-DMA f64
                                    block kernel (default for int16 stereo) instead of the register-prefetch one */
    BPMX_OPT_PEAKS_GLOBAL = 256, /* find_peaks by sample walks over global memory (k_find_peaks) for every
                                    recording instead of the LDS-resident extrema (test/diagnostic) */
    BPMX_OPT_HILBERT_R2C = 512,  /* native mode, recordings outside the fused Hilbert kernel: one rocFFT
                                    R2C/C2R plan per distinct length instead of the batched Bluestein
                                    transform (test/diagnostic) */
    BPMX_OPT_REF_SERIAL_MEAN = 1024, /* reference mode: form the rolling mean's outputs inside the sequential
                                        pass instead of from its running sums in parallel (test/diagnostic) */
    BPMX_OPT_STATS = 2048,           /* count the run's path decisions for bpmx_stats (diagnostic) */
    BPMX_OPT_HILBERT_BLUESTEIN = 4096, /* native mode, long recordings: rocFFT Bluestein instead of the exact-
                                         length four-step transform (test/diagnostic) */
    BPMX_OPT_REF_NOSPLIT = 8192      /* reference mode: gather every decimated sample first, then the forward
                                        pass inside k_envelope_ref, instead of forward-pass row chunks
                                        overlapping the next chunks' gather on a side stream (diagnostic) */
};

/* bpmx_stats counters of the last run with BPMX_OPT_STATS */
enum bpmx_stat {
    BPMX_STAT_RAW_TROUGHS = 0,   /* raw troughs of the recordings whose draft floor was bracketed */
    BPMX_STAT_UNDECIDED = 1,     /* of those, troughs the bracket left open: draft evaluated there exactly */
    BPMX_STAT_FULL_DRAFT = 2,    /* trough chunks whose recording fell back to the whole draft floor */
    BPMX_NSTATS = 8
};

typedef struct bpmx_ctx bpmx_ctx;

typedef struct {
    int32_t mode;          /* bpmx_mode */
    int32_t stages;        /* bpmx_stage mask */
    int32_t dtype;         /* bpmx_dtype of the PCM */
    int32_t channels;      /* >= 1, frames are interleaved */
    int32_t fs;            /* native sample rate */
    int32_t ds;            /* downsample factor after the clamp (:1021-1029), >= 1 */
    int32_t sr;            /* decimated rate fs // ds (:1032) */
    int32_t env_window;    /* sr // 10 (:1053) */
    int32_t distance;      /* int(min_peak_distance_sec * sr) (:1066, :226), >= 1 */
    int32_t noise_window;  /* int(noise_window_sec * sr) (:1084) */
    int32_t min_periods;   /* 3 (:1085, :1105) */
    int32_t options;       /* bpmx_option bits (0 = defaults) */
    double trough_prom_q;  /* trough_prominence_quantile (:1067) */
    double peak_prom_q;    /* peak_prominence_quantile (:225) */
    double noise_floor_q;  /* noise_floor_quantile (:1075, :1085) */
    double fallback_q;     /* 0.1 (:1114) */
    double reject_mult;    /* trough_rejection_multiplier (:1091) */
    double ba_b[5], ba_a[5], ba_zi[4];  /* butter(2,[lo,hi],'band') at sr + lfilter_zi (reference mode) */
    double sos[12], sos_zi[4];          /* butter(...,output='sos') at fs + sosfilt_zi (native mode) */
} bpmx_params;

typedef struct {
    int32_t n_files;
    int32_t reserved;
    const void *pcm;              /* device: frames of all files back to back, interleaved channels.
                                     The library may read from the 16-byte boundary at or below pcm
                                     (an int16 base a whole number of frames past it is read from
                                     there; the bytes before pcm are read and discarded, never used),
                                     so that a recording's outputs do not depend on its alignment */
    const int64_t *frame_offsets; /* host: n_files+1 frame offsets into pcm */
} bpmx_batch;

/* Result arrays (device).  Per-file slices start at the decimated offsets
 * D_f = sum_{g<f} Nd_g, Nd_g = bpmx_decimated_length(frames_g, ds); every
 * array below has sum(Nd) elements, except the three per-file ones.
 * env / floor are inputs when the stage that produces them is not requested. */
typedef struct {
    double *env;        /* f64 envelope */
    double *floor;      /* f64 dynamic noise floor */
    double *y;          /* optional (NULL): filtered decimated signal (debug WAV, :1047-1060).
                         * Native mode: asking for it keeps a separate yd pass (~0.05 ms per
                         * 1024 x 60 s batch on MI355X); left NULL, the envelope kernel makes
                         * yd itself. */
    int64_t *troughs;   /* sanitised trough indices, per-file slice, n_troughs[f] valid */
    int64_t *peaks;     /* raw peak indices, per-file slice, n_peaks[f] valid */
    int32_t *n_troughs; /* [n_files] */
    int32_t *n_peaks;   /* [n_files] */
    int32_t *flags;     /* [n_files] bpmx_file_flag bits */
    int32_t *n_raw_troughs; /* optional [n_files]: troughs before sanitisation (:1099 log line) */
} bpmx_out;

int bpmx_abi_version(void);
const char *bpmx_last_error(void);

int bpmx_create(int device, bpmx_ctx **out);
void bpmx_destroy(bpmx_ctx *ctx);

/* ceil(n_frames / ds): length of x[::ds] (:1033) */
int64_t bpmx_decimated_length(int64_t n_frames, int32_t ds);

/* Run the requested stages over a batch, asynchronously on `stream`
 * (a hipStream_t; NULL = default stream). */
int bpmx_run(bpmx_ctx *ctx, const bpmx_params *params, const bpmx_batch *batch, const bpmx_out *out,
             void *stream);

/* Resolving decisive ties in the reference's own order (BPMX_F_*_TIE).
 *
 * scipy's distance filter (_peak_finding_utils._select_by_peak_distance,
 * called at scipy/signal/_peak_finding.py:976-980 from bpm_analysis.py:1070 and
 * :227) visits the candidates in np.argsort(x[peaks]) order, highest last
 * index first.  That order is numpy's, so only the host can produce it:
 * a run with cand[s] set writes each recording's candidate list of search s
 * (the local maxima, plateau midpoints, left by the height filter; ascending
 * positions, per-file slices at D_f, n_cand[s][f] of them); the host computes
 * rank = inverse of np.argsort(x[cand]) per recording; a run with rank[s] set
 * (and use_rank[s][f] != 0) then decides the distance filter of recording f by
 * rank alone — candidate k removes candidate j within `distance` iff
 * rank[k] > rank[j] and k is kept — which is scipy's greedy loop exactly.
 * Search 0 is the trough search find_peaks(-env) (:1070), 1 the raw-peak search
 * find_peaks(env, height=floor) (:227).  The candidates of a search depend only
 * on env (and the floor for search 1), so a rank computed from one run's list
 * applies to any run on the same env (and floor).  All pointers are device
 * pointers and optional (NULL: that part is not used); a run with an order
 * object takes the one-workgroup find_peaks kernel for every recording.  Meant
 * for the few recordings that carry a TIE bit (engine.Detector.resolve_ties).
 */
typedef struct {
    int32_t *cand[2];           /* out: candidate positions, sum(Nd) entries, per-file slices at D_f */
    int32_t *n_cand[2];         /* out: [n_files] candidate counts (with cand[s]) */
    const int32_t *rank[2];     /* in: per candidate (same order as cand), its index in np.argsort(x[cand]) */
    const int32_t *use_rank[2]; /* in: [n_files] nonzero = recording f's slice of rank[s] is set */
} bpmx_peak_order;

/* bpmx_run with a find_peaks visiting order / candidate export (above); order
 * NULL = bpmx_run.  Never pipelined. */
int bpmx_run_ordered(bpmx_ctx *ctx, const bpmx_params *params, const bpmx_batch *batch, const bpmx_out *out,
                     const bpmx_peak_order *order, void *stream);

/* Synthetic int16 recordings straight into HBM: file f gets seed seed0+f,
 * frames [frame_offsets[f], frame_offsets[f+1]) of pcm (device). */
int bpmx_synth(bpmx_ctx *ctx, uint64_t seed0, int32_t n_files, const int64_t *frame_offsets, int32_t fs,
               int32_t channels, int16_t *pcm, void *stream);
/* The same generator on the host (bit-identical). */
void bpmx_synth_host(uint64_t seed, int64_t n_frames, int32_t fs, int32_t channels, int16_t *out);

/* Per-kernel device timing with HIP events recorded on the launch stream.
 * bpmx_profile(ctx, 1) starts recording; bpmx_profile_read() synchronises,
 * and writes "name launches total_ms\n" lines into buf (returns bytes). */
int bpmx_profile(bpmx_ctx *ctx, int on);
int bpmx_profile_read(bpmx_ctx *ctx, char *buf, int len);
/* Record events only around launches labelled `label` (NULL or "": every
 * launch), so a timed run can carry one kernel's device time without
 * bracketing every launch. */
int bpmx_profile_only(bpmx_ctx *ctx, const char *label);

/* Pipelined runs: batches of at least 2 * chunks recordings with ENVELOPE and
 * a detection stage run as `chunks` consecutive groups of recordings; group
 * k's envelope runs on an internal stream restricted to env_cus CUs (0: no
 * restriction) while group k-1's detection runs beside it (on an internal
 * stream restricted to det_cus other CUs when det_cus > 0, else on the
 * caller's stream), so the HBM-bound envelope kernels overlap the
 * latency-bound detection kernels.  Same outputs as an unpipelined run: every
 * index, count and flag identical, env, y and floor bit-identical, in both
 * modes (a recording's outputs do not depend on where its PCM lies: an int16
 * base a whole number of frames past a 16-byte boundary is read from that
 * boundary, so a chunk keeps the matrix-core block kernel).
 * Pipeline sub-contexts share the root context's side streams, which carry no
 * CU mask.  chunks = 0 (the default) turns it off.  Waits for the device. */
int bpmx_set_pipeline(bpmx_ctx *ctx, int chunks, int env_cus, int det_cus);

/* Counters (enum bpmx_stat) of the last bpmx_run on ctx that had
 * BPMX_OPT_STATS set: waits for that run, copies min(n, BPMX_NSTATS) of them
 * into out (zeros if none), returns BPMX_NSTATS or an error code. */
int bpmx_stats(bpmx_ctx *ctx, int64_t *out, int n);

#ifdef __cplusplus
}
#endif

#endif /* BPMX_H */
