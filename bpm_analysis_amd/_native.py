"""ctypes binding of libbpmx.so (include/bpmx.h).

The shared library is built in-tree (``bpm_analysis_amd/libbpmx.so``, see
``csrc/Makefile`` / ``__graft_entry__.build()``).  There is no fallback: if the
library is missing or cannot be loaded this module raises, so a GPU run can
never silently compute on the CPU.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# BPMX_LIB: another build of the same library (diagnostic A/B runs of kernel variants)
LIB_PATH = os.environ.get("BPMX_LIB") or os.path.join(_HERE, "libbpmx.so")

ABI_VERSION = 2

DT_U8, DT_I16, DT_I32, DT_F32, DT_F64 = 0, 1, 2, 3, 4
MODE_REFERENCE, MODE_NATIVE = 0, 1
STAGE_ENVELOPE, STAGE_FLOOR, STAGE_PEAKS, STAGE_ALL = 1, 2, 4, 7
F_STATIC_FLOOR, F_DRAFT_FLOOR, F_NAN_FLOOR, F_TOO_SHORT, F_BAD_WINDOW = 1, 2, 4, 8, 16
F_TROUGH_TIE, F_PEAK_TIE = 32, 64      # decisive height tie in find_peaks' distance filter (bpmx.h)
F_TROUGH_ORDERED, F_PEAK_ORDERED = 128, 256   # that filter ran in the caller's np.argsort order (bpmx_run_ordered)
OPT_ROLLQ_MERGE = 1
OPT_NATIVE_F64 = 2
OPT_HILBERT_ROCFFT = 4
OPT_DRAFT_FULL = 8
OPT_ROLLQ_NOPRUNE = 16
OPT_DRAFT_GLOBAL_RANK = 32
OPT_ROLLQ_GLOBAL = 64
OPT_NATIVE_DMA = 128
OPT_PEAKS_GLOBAL = 256
OPT_HILBERT_R2C = 512
OPT_REF_SERIAL_MEAN = 1024
OPT_STATS = 2048
OPT_HILBERT_BLUESTEIN = 4096
OPT_REF_NOSPLIT = 8192
STAT_RAW_TROUGHS, STAT_UNDECIDED, STAT_FULL_DRAFT, NSTATS = 0, 1, 2, 8
OK, E_ARG, E_HIP, E_LIMIT, E_NODEV = 0, -1, -2, -3, -4

EXPORTS = ["bpmx_abi_version", "bpmx_last_error", "bpmx_create", "bpmx_destroy", "bpmx_decimated_length",
           "bpmx_run", "bpmx_run_ordered", "bpmx_synth", "bpmx_synth_host", "bpmx_profile", "bpmx_profile_read", "bpmx_profile_only",
           "bpmx_stats", "bpmx_set_pipeline"]


class Params(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("stages", ctypes.c_int32), ("dtype", ctypes.c_int32),
                ("channels", ctypes.c_int32), ("fs", ctypes.c_int32), ("ds", ctypes.c_int32),
                ("sr", ctypes.c_int32), ("env_window", ctypes.c_int32), ("distance", ctypes.c_int32),
                ("noise_window", ctypes.c_int32), ("min_periods", ctypes.c_int32), ("options", ctypes.c_int32),
                ("trough_prom_q", ctypes.c_double), ("peak_prom_q", ctypes.c_double),
                ("noise_floor_q", ctypes.c_double), ("fallback_q", ctypes.c_double),
                ("reject_mult", ctypes.c_double),
                ("ba_b", ctypes.c_double * 5), ("ba_a", ctypes.c_double * 5), ("ba_zi", ctypes.c_double * 4),
                ("sos", ctypes.c_double * 12), ("sos_zi", ctypes.c_double * 4)]


class Batch(ctypes.Structure):
    _fields_ = [("n_files", ctypes.c_int32), ("reserved", ctypes.c_int32), ("pcm", ctypes.c_void_p),
                ("frame_offsets", ctypes.POINTER(ctypes.c_int64))]


class Out(ctypes.Structure):
    _fields_ = [("env", ctypes.c_void_p), ("floor", ctypes.c_void_p), ("y", ctypes.c_void_p),
                ("troughs", ctypes.c_void_p), ("peaks", ctypes.c_void_p), ("n_troughs", ctypes.c_void_p),
                ("n_peaks", ctypes.c_void_p), ("flags", ctypes.c_void_p), ("n_raw_troughs", ctypes.c_void_p)]


class PeakOrder(ctypes.Structure):
    """bpmx_peak_order: per search (0 = troughs, 1 = raw peaks) the candidate
    export and the caller's visiting ranks (device pointers or None)."""
    _fields_ = [("cand", ctypes.c_void_p * 2), ("n_cand", ctypes.c_void_p * 2),
                ("rank", ctypes.c_void_p * 2), ("use_rank", ctypes.c_void_p * 2)]


class BpmxError(RuntimeError):
    """A libbpmx failure.  ``code`` is the BPMX_E_* status (None when raised by
    the host side).  Only argument and size-limit errors belong to the
    recordings of one call (``per_file``); a HIP or device failure means the
    GPU path itself failed and must stop the run."""

    def __init__(self, msg: str = "", code: int = None):
        super().__init__(msg)
        self.code = code

    @property
    def per_file(self) -> bool:
        return self.code in (E_ARG, E_LIMIT)


class BpmxArgError(BpmxError, ValueError):
    """BPMX_E_ARG: an argument the reference's own calls reject with ValueError
    (scipy find_peaks' distance check, pandas' rolling-window checks); the
    message is the library's, which repeats the reference-side wording."""


_lib = None


def load() -> ctypes.CDLL:
    """Load libbpmx.so (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise BpmxError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                        f"or `make -C bpm_analysis_amd/csrc` (there is no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    P, I32, I64, U64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    L.bpmx_abi_version.restype = ctypes.c_int
    L.bpmx_last_error.restype = ctypes.c_char_p
    L.bpmx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    L.bpmx_create.restype = ctypes.c_int
    L.bpmx_destroy.argtypes = [P]
    L.bpmx_destroy.restype = None
    L.bpmx_decimated_length.argtypes = [I64, I32]
    L.bpmx_decimated_length.restype = I64
    L.bpmx_run.argtypes = [P, ctypes.POINTER(Params), ctypes.POINTER(Batch), ctypes.POINTER(Out), P]
    L.bpmx_run.restype = ctypes.c_int
    L.bpmx_run_ordered.argtypes = [P, ctypes.POINTER(Params), ctypes.POINTER(Batch), ctypes.POINTER(Out),
                                   ctypes.POINTER(PeakOrder), P]
    L.bpmx_run_ordered.restype = ctypes.c_int
    L.bpmx_synth.argtypes = [P, U64, I32, ctypes.POINTER(ctypes.c_int64), I32, I32, P, P]
    L.bpmx_synth.restype = ctypes.c_int
    L.bpmx_synth_host.argtypes = [U64, I64, I32, I32, P]
    L.bpmx_synth_host.restype = None
    L.bpmx_profile.argtypes = [P, ctypes.c_int]
    L.bpmx_profile.restype = ctypes.c_int
    L.bpmx_profile_read.argtypes = [P, ctypes.c_char_p, ctypes.c_int]
    L.bpmx_profile_read.restype = ctypes.c_int
    L.bpmx_profile_only.argtypes = [P, ctypes.c_char_p]
    L.bpmx_profile_only.restype = ctypes.c_int
    L.bpmx_stats.argtypes = [P, ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
    L.bpmx_stats.restype = ctypes.c_int
    L.bpmx_set_pipeline.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.bpmx_set_pipeline.restype = ctypes.c_int
    if L.bpmx_abi_version() != ABI_VERSION:
        raise BpmxError(f"libbpmx ABI {L.bpmx_abi_version()} != expected {ABI_VERSION}; rebuild")
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != OK:
        msg = load().bpmx_last_error().decode(errors="replace")
        if rc == E_ARG:
            raise BpmxArgError(msg, rc)
        raise BpmxError(f"{what} failed ({rc}): {msg}", rc)
