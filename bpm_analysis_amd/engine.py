"""Batch engine: device buffers (torch), the C-ABI call, per-file results.

PyTorch is used here only as plumbing — device memory, streams and copies.
All arithmetic runs in libbpmx.so's HIP kernels.

A batch is a set of recordings with one sample rate, sample format and
channel count (the reference processes one WAV at a time: gui.py:202-251; a
batch is the MI355X unit of work).  Lengths may be ragged.  Recordings are
laid out back to back in HBM; results use the decimated offsets
``doff[f] = sum(Nd[:f])``.
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import _native as N
from .design import Design, design, detect_design, dtype_code, make_params

MODES = {"reference": N.MODE_REFERENCE, "native": N.MODE_NATIVE}


def _torch():
    import torch
    return torch


_TORCH_DT = None


def torch_dtype(np_dtype):
    global _TORCH_DT
    torch = _torch()
    if _TORCH_DT is None:
        _TORCH_DT = {np.dtype(np.uint8): torch.uint8, np.dtype(np.int16): torch.int16,
                     np.dtype(np.int32): torch.int32, np.dtype(np.float32): torch.float32,
                     np.dtype(np.float64): torch.float64}
    return _TORCH_DT[np.dtype(np_dtype)]


@dataclass
class Result:
    """Device-resident outputs of one batch (torch tensors on the GPU)."""
    sr: int
    ds: int
    frame_offsets: np.ndarray      # host int64 [F+1]
    doff: np.ndarray               # host int64 [F+1] decimated offsets
    env: "object"
    floor: "object"
    y: "object"
    troughs: "object"
    peaks: "object"
    n_troughs: "object"
    n_peaks: "object"
    n_raw_troughs: "object"
    flags: "object"

    @property
    def n_files(self) -> int:
        return len(self.doff) - 1

    def to_host(self) -> List[dict]:
        """Per-file numpy views after one D2H copy of each array."""
        env = self.env.cpu().numpy()
        floor = self.floor.cpu().numpy() if self.floor is not None else None
        y = self.y.cpu().numpy() if self.y is not None else None
        tr = self.troughs.cpu().numpy() if self.troughs is not None else None
        pk = self.peaks.cpu().numpy() if self.peaks is not None else None
        ntr = self.n_troughs.cpu().numpy()
        npk = self.n_peaks.cpu().numpy()
        nraw = self.n_raw_troughs.cpu().numpy()
        flags = self.flags.cpu().numpy()
        out = []
        for f in range(self.n_files):
            a, b = int(self.doff[f]), int(self.doff[f + 1])
            if flags[f] & N.F_TOO_SHORT:
                b = a           # no outputs (include/bpmx.h): empty slices, not the buffers' old contents
            out.append(dict(
                sr=self.sr, env=env[a:b], floor=None if floor is None else floor[a:b],
                y=None if y is None else y[a:b],
                troughs=None if tr is None else tr[a:a + int(ntr[f])].copy(),
                peaks=None if pk is None else pk[a:a + int(npk[f])].copy(),
                n_raw_troughs=int(nraw[f]), flags=int(flags[f])))
        return out


class Detector:
    """One libbpmx context on one GPU.

    Threading (the reference is called from a GUI worker thread, gui.py:181-187,
    and Gradio may call concurrently): ``run`` enqueues under ``lock`` on the
    caller's current stream; the host entry points (``run_host``,
    ``run_env_host``) hold the lock from upload to download on the detector's
    own stream, so a context's scratch is never shared by two calls in flight.
    ``default_detector`` gives each thread its own Detector (context + stream),
    so concurrent threads also run concurrently on the GPU."""

    def __init__(self, device: int = 0):
        torch = _torch()
        if not torch.cuda.is_available():
            raise N.BpmxError("no GPU visible to torch: the bpmx path runs only on an MI355X (gfx950)")
        self.L = N.load()
        self.device = torch.device("cuda", device)
        torch.cuda.set_device(self.device)
        torch.empty(1, device=self.device)      # initialise the HIP runtime on this device
        ctx = ctypes.c_void_p()
        N.check(self.L.bpmx_create(device, ctypes.byref(ctx)), "bpmx_create")
        self.ctx = ctx
        self.lock = threading.RLock()
        self._stream = None

    def close(self):
        if getattr(self, "ctx", None):
            self.L.bpmx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ #
    def host_stream(self):
        """The stream of the host entry points (created on first use)."""
        if self._stream is None:
            self._stream = _torch().cuda.Stream(self.device)
        return self._stream

    def stream_handle(self) -> ctypes.c_void_p:
        return ctypes.c_void_p(_torch().cuda.current_stream(self.device).cuda_stream)

    def alloc(self, frame_offsets: Sequence[int], ds: int, sr: int, want_y: bool = False,
              want_floor: bool = True, want_troughs: bool = True, want_peaks: bool = True) -> Result:
        torch = _torch()
        fo = np.ascontiguousarray(frame_offsets, dtype=np.int64)
        lens = np.diff(fo)
        nd = np.where(lens > 0, (lens + ds - 1) // ds, 0)
        doff = np.zeros(len(fo), dtype=np.int64)
        doff[1:] = np.cumsum(nd)
        tot, F = int(doff[-1]), len(fo) - 1
        dev = self.device
        e = lambda dt: torch.empty(max(tot, 1), dtype=dt, device=dev)
        return Result(sr=sr, ds=ds, frame_offsets=fo, doff=doff, env=e(torch.float64),
                      floor=e(torch.float64) if want_floor else None, y=e(torch.float64) if want_y else None,
                      troughs=e(torch.int64) if want_troughs else None, peaks=e(torch.int64) if want_peaks else None,
                      n_troughs=torch.zeros(F, dtype=torch.int32, device=dev),
                      n_peaks=torch.zeros(F, dtype=torch.int32, device=dev),
                      n_raw_troughs=torch.zeros(F, dtype=torch.int32, device=dev),
                      flags=torch.zeros(F, dtype=torch.int32, device=dev))

    def run(self, pcm, frame_offsets: Sequence[int], fs: int, params: dict, mode: str = "reference",
            stages: int = N.STAGE_ALL, channels: int = 1, out: Optional[Result] = None, want_y: bool = False,
            d: Optional[Design] = None, log: bool = False, options: int = 0,
            order: Optional[N.PeakOrder] = None) -> Result:
        """Run `stages` over a device batch.  `pcm` is a CUDA tensor (or None when
        ENVELOPE is not requested and `out.env` already holds the envelopes).
        `order`: bpmx_run_ordered's candidate export / visiting ranks (see
        ``resolve_ties``)."""
        if d is None:
            d = design(fs, params, log=log)
        fo = np.ascontiguousarray(frame_offsets, dtype=np.int64)
        if out is None:
            out = self.alloc(fo, d.ds, d.sr, want_y=want_y)
        if pcm is not None:
            np_dt = {v: k for k, v in _torch_np_map().items()}[pcm.dtype]
            dt = dtype_code(np_dt)
            assert pcm.is_cuda and pcm.is_contiguous()
            assert pcm.numel() >= int(fo[-1]) * channels, "pcm shorter than frame_offsets[-1] * channels"
            pcm_ptr = pcm.data_ptr()
        else:
            dt, pcm_ptr = N.DT_I16, None
        p = make_params(d, params, MODES[mode], stages, dt, channels)
        p.options = options
        b = N.Batch()
        b.n_files = len(fo) - 1
        b.pcm = pcm_ptr
        b.frame_offsets = fo.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
        o = N.Out()
        ptr = lambda t: None if t is None else t.data_ptr()
        o.env, o.floor, o.y = ptr(out.env), ptr(out.floor), ptr(out.y)
        o.troughs, o.peaks = ptr(out.troughs), ptr(out.peaks)
        o.n_troughs, o.n_peaks, o.flags = ptr(out.n_troughs), ptr(out.n_peaks), ptr(out.flags)
        o.n_raw_troughs = ptr(out.n_raw_troughs)
        with self.lock:
            if order is None:
                N.check(self.L.bpmx_run(self.ctx, ctypes.byref(p), ctypes.byref(b), ctypes.byref(o),
                                        self.stream_handle()), "bpmx_run")
            else:
                N.check(self.L.bpmx_run_ordered(self.ctx, ctypes.byref(p), ctypes.byref(b), ctypes.byref(o),
                                                ctypes.byref(order), self.stream_handle()), "bpmx_run_ordered")
        return out

    def resolve_ties(self, out: Result, params: dict, stages: int = N.STAGE_ALL, options: int = 0) -> int:
        """Re-decide find_peaks' distance filter in numpy's own argsort order for
        the recordings of `out` that carry a decisive-tie bit (F_TROUGH_TIE /
        F_PEAK_TIE), so their troughs, floor and raw peaks are the reference's
        on this machine.

        scipy visits the distance filter's candidates in ``np.argsort(x[peaks])``
        order (``_select_by_peak_distance``, scipy/signal/_peak_finding.py:976-980,
        called from bpm_analysis.py:1070 and :227).  Among equal heights that
        order is numpy's implementation detail, so it is computed here, by numpy,
        from the candidate list the library exports; the library then decides the
        filter by those ranks (include/bpmx.h ``bpmx_run_ordered``).  Troughs
        first: a new trough set changes the floor and so the peak search's
        candidates, whose order is taken after.  The flagged recordings run as a
        sub-batch (ds = 1, envelopes gathered on the device); their results are
        written back into `out` and their flags carry F_*_ORDERED instead of
        F_*_TIE.  `options`: the run's bpmx_option bits, forwarded to the
        sub-batch runs (BPMX_OPT_STATS, which bpmx_run_ordered rejects, masked
        off) so they take the same floor kernels as the original run.  Returns
        the number of recordings re-run (0: nothing to do, no launch).
        Synchronises the current stream."""
        torch = _torch()
        det_st = stages & (N.STAGE_FLOOR | N.STAGE_PEAKS)
        bits = (N.F_TROUGH_TIE if det_st & N.STAGE_FLOOR else 0) | (N.F_PEAK_TIE if det_st & N.STAGE_PEAKS else 0)
        if not bits:
            return 0
        flags = out.flags.cpu().numpy()
        sel = np.flatnonzero(flags & bits)
        if sel.size == 0:
            return 0
        F = int(sel.size)
        lens = out.doff[sel + 1] - out.doff[sel]
        fo = np.zeros(F + 1, dtype=np.int64)
        fo[1:] = np.cumsum(lens)
        tot = int(fo[-1])
        d = detect_design(out.sr, params)
        dev = self.device
        idx = torch.from_numpy(np.concatenate([np.arange(out.doff[f], out.doff[f + 1]) for f in sel])).to(dev)
        sub = self.alloc(fo, 1, d.sr)
        sub.env.copy_(out.env[idx])
        if not det_st & N.STAGE_FLOOR:
            sub.floor.copy_(out.floor[idx])
        env_h = sub.env.cpu().numpy()
        i32 = lambda k: torch.zeros(max(k, 1), dtype=torch.int32, device=dev)
        cand, ncand = [i32(tot), i32(tot)], [i32(F), i32(F)]
        rank, use = [i32(tot), i32(tot)], [i32(F), i32(F)]

        def order(export, ranked):
            o = N.PeakOrder()
            for s in export:
                o.cand[s], o.n_cand[s] = cand[s].data_ptr(), ncand[s].data_ptr()
            for s in ranked:
                o.rank[s], o.use_rank[s] = rank[s].data_ptr(), use[s].data_ptr()
            return o

        def set_ranks(s, files, sign):
            c, nc = cand[s].cpu().numpy(), ncand[s].cpu().numpy()
            r, u = np.zeros(max(tot, 1), dtype=np.int32), np.zeros(F, dtype=np.int32)
            for k in files:
                a, m = int(fo[k]), int(nc[k])
                x = env_h[a:int(fo[k + 1])]
                x = -x if sign < 0 else x                     # find_peaks(-env) negates the array (:1070)
                perm = np.argsort(x[c[a:a + m]])              # the call _select_by_peak_distance makes
                r[a + perm] = np.arange(m, dtype=np.int32)
                u[k] = 1
            rank[s].copy_(torch.from_numpy(r))
            use[s].copy_(torch.from_numpy(u))

        opts = options & ~N.OPT_STATS
        run = lambda st, o: self.run(None, fo, d.sr, params, stages=st, out=sub, d=d, order=o, options=opts)
        ranked = set()
        if det_st & N.STAGE_FLOOR and (flags[sel] & N.F_TROUGH_TIE).any():
            run(det_st, order({0}, ()))
            set_ranks(0, np.flatnonzero(flags[sel] & N.F_TROUGH_TIE), -1.0)
            ranked.add(0)
        run(det_st, order({1} if det_st & N.STAGE_PEAKS else (), ranked))
        fl = sub.flags.cpu().numpy().copy()
        if det_st & N.STAGE_PEAKS and (fl & N.F_PEAK_TIE).any():
            p2 = np.flatnonzero(fl & N.F_PEAK_TIE)
            set_ranks(1, p2, 1.0)
            run(N.STAGE_PEAKS, order((), {1}))
            pb = N.F_PEAK_TIE | N.F_PEAK_ORDERED
            fl = (fl & ~pb) | (sub.flags.cpu().numpy() & pb)
        if det_st & N.STAGE_FLOOR:
            out.floor[idx] = sub.floor[:tot]
            out.troughs[idx] = sub.troughs[:tot]
            out.n_troughs[sel] = sub.n_troughs
            out.n_raw_troughs[sel] = sub.n_raw_troughs
        if det_st & N.STAGE_PEAKS:
            out.peaks[idx] = sub.peaks[:tot]
            out.n_peaks[sel] = sub.n_peaks
        out.flags[torch.from_numpy(sel).to(dev)] = torch.from_numpy(fl).to(dev)
        return F

    def tie_check_start(self, out: Result):
        """Start the flags read-back that ``tie_check_finish`` decides on: an
        asynchronous copy of ``out.flags`` into pinned host memory and an event
        behind it on the current stream, so the host need not wait for the run
        before queuing the next one (a batch pipeline keeps two ``Result`` sets
        and checks run k while run k + 1 is queued)."""
        torch = _torch()
        host = torch.empty(out.flags.shape, dtype=out.flags.dtype, pin_memory=True)
        host.copy_(out.flags, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return host, ev

    def tie_check_finish(self, handle, out: Result, params: dict, stages: int = N.STAGE_ALL,
                         options: int = 0) -> int:
        """Wait for the read-back ``tie_check_start`` began; if any recording of
        `out` carries a decisive-tie bit, re-decide them (``resolve_ties``: a
        launch and a host sort only then).  Returns the recordings re-run."""
        host, ev = handle
        ev.synchronize()
        bits = N.F_TROUGH_TIE | N.F_PEAK_TIE
        if not (host.numpy() & bits).any():
            return 0
        return self.resolve_ties(out, params, stages, options)

    def synth(self, frame_offsets: Sequence[int], fs: int, channels: int = 1, seed0: int = 0,
              seeds: Optional[Sequence[int]] = None):
        """Synthetic int16 batch generated in HBM (bit-identical to bpmx_synth_host):
        recording f gets seed ``seed0 + f``, or ``seeds[f]`` when given."""
        torch = _torch()
        fo = np.ascontiguousarray(frame_offsets, dtype=np.int64)
        pcm = torch.empty(int(fo[-1]) * channels, dtype=torch.int16, device=self.device)
        runs = [(seed0, 0, len(fo) - 1)] if seeds is None else [(int(sd), f, f + 1) for f, sd in enumerate(seeds)]
        with self.lock:
            for sd, a, b in runs:
                sub = np.ascontiguousarray(fo[a:b + 1])
                N.check(self.L.bpmx_synth(self.ctx, sd, b - a, sub.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                          fs, channels, ctypes.c_void_p(pcm.data_ptr()), self.stream_handle()),
                        "bpmx_synth")
        return pcm

    def profile(self, on: bool):
        N.check(self.L.bpmx_profile(self.ctx, 1 if on else 0), "bpmx_profile")

    def profile_only(self, label: str = ""):
        """Restrict profiling events to launches labelled `label` ("" = all)."""
        N.check(self.L.bpmx_profile_only(self.ctx, label.encode()), "bpmx_profile_only")

    def profile_read(self) -> dict:
        buf = ctypes.create_string_buffer(1 << 16)
        n = self.L.bpmx_profile_read(self.ctx, buf, len(buf))
        if n < 0:
            N.check(n, "bpmx_profile_read")
        out = {}
        for line in buf.value.decode().splitlines():
            name, cnt, ms = line.rsplit(" ", 2)
            out[name] = (int(cnt), float(ms))
        return out

    def set_pipeline(self, chunks: int, env_cus: int = 0, det_cus: int = 0):
        """bpmx_set_pipeline: overlap chunk k's envelope with chunk k-1's detection (0 = off)."""
        N.check(self.L.bpmx_set_pipeline(self.ctx, chunks, env_cus, det_cus), "bpmx_set_pipeline")

    def stats(self) -> dict:
        """Path counters of the last run with options | OPT_STATS (bpmx_stats)."""
        buf = (ctypes.c_int64 * N.NSTATS)()
        rc = self.L.bpmx_stats(self.ctx, buf, N.NSTATS)
        if rc < 0:
            N.check(rc, "bpmx_stats")
        return {"raw_troughs": int(buf[N.STAT_RAW_TROUGHS]), "undecided": int(buf[N.STAT_UNDECIDED]),
                "full_draft_chunks": int(buf[N.STAT_FULL_DRAFT])}

    # ------------------------------------------------------------------ #
    def run_host(self, recordings: List[np.ndarray], fs: int, params: dict, mode: str = "reference",
                 stages: int = N.STAGE_ALL, want_y: bool = False, log: bool = False,
                 options: int = 0, longest_first: bool = True, resolve_ties: bool = False) -> List[dict]:
        """Host arrays in, per-file host results out (H2D + run + D2H).

        A ragged batch runs longest recording first (shard.longest_first: LPT
        over the CUs, since recording f is workgroup f of every per-recording
        kernel); results come back in the caller's order.  `resolve_ties`:
        decisive find_peaks ties re-decided in numpy's order (``resolve_ties``;
        the drop-in entry points set it)."""
        torch = _torch()
        if not recordings:
            return []
        if longest_first and len({r.shape[0] for r in recordings}) > 1:
            from .shard import longest_first as _lf
            perm = _lf([r.shape[0] for r in recordings])
            res = self.run_host([recordings[i] for i in perm], fs, params, mode=mode, stages=stages,
                                want_y=want_y, log=log, options=options, longest_first=False,
                                resolve_ties=resolve_ties)
            out: List[dict] = [None] * len(recordings)
            for k, i in enumerate(perm):
                out[i] = res[k]
            return out
        dt = recordings[0].dtype
        ch = 1 if recordings[0].ndim == 1 else recordings[0].shape[1]
        for r in recordings:
            if r.dtype != dt or (1 if r.ndim == 1 else r.shape[1]) != ch:
                raise ValueError("a batch needs one sample format and channel count")
        fo = np.zeros(len(recordings) + 1, dtype=np.int64)
        fo[1:] = np.cumsum([r.shape[0] for r in recordings])
        host = np.concatenate([np.ascontiguousarray(r).reshape(-1) for r in recordings])
        with self.lock, torch.cuda.stream(self.host_stream()):
            pcm = torch.from_numpy(host).to(self.device)
            res = self.run(pcm, fo, fs, params, mode=mode, stages=stages, channels=ch, want_y=want_y, log=log,
                           options=options)
            if resolve_ties:
                self.resolve_ties(res, params, stages, options)
            out = res.to_host()          # .cpu() waits for this stream only
            self.host_stream().synchronize()
        return out

    def run_env_host(self, envs: List[np.ndarray], sr: int, params: dict, stages: int,
                     floors: Optional[List[np.ndarray]] = None, options: int = 0,
                     resolve_ties: bool = False) -> List[dict]:
        """Detection stages on host envelopes (drop-in for the env-level functions)."""
        torch = _torch()
        fo = np.zeros(len(envs) + 1, dtype=np.int64)
        fo[1:] = np.cumsum([len(e) for e in envs])   # ds = 1: offsets == decimated offsets
        d = detect_design(sr, params)
        with self.lock, torch.cuda.stream(self.host_stream()):
            out = self.alloc(fo, 1, d.sr)
            out.env.copy_(torch.from_numpy(np.concatenate(envs).astype(np.float64)).to(self.device))
            if floors is not None:
                out.floor.copy_(torch.from_numpy(np.concatenate(floors).astype(np.float64)).to(self.device))
            self.run(None, fo, d.sr, params, stages=stages, out=out, d=d, options=options)
            if resolve_ties:
                self.resolve_ties(out, params, stages, options)
            res = out.to_host()
            self.host_stream().synchronize()
        return res


class BatchPipeline:
    """Batches of one geometry through the path back to back, batch k + 1's
    ENVELOPE stage overlapping batch k's detection (FLOOR | PEAKS and the
    decisive-tie check).

    Reference mode's envelope is three bit-exact sequential passes (DF2T
    forward and backward, pandas' Kahan rolling mean, bpm_analysis.py:1045-1054)
    with one lane per recording: 1024 recordings are 16 waves, so for ~2.8 ms
    per batch 240 of the 256 CUs idle, and the detection after it fills the
    chip for ~1.3 ms.  Two library contexts on two HIP streams run the two
    halves of consecutive batches at the same time (the streams' kernels do
    overlap on MI355X: tools/overlap_probe), so a stream of batches costs
    max(envelope, detection) per batch instead of their sum.  ``depth`` result
    sets rotate; batch k's envelope waits (an event, no host wait) until the
    detection that last used its result set is done.

    ``submit(pcm)`` enqueues one batch and returns its Result (complete once
    ``finish`` or a later ``submit`` has checked it); ``finish()`` drains.
    Every batch's outputs equal a single ``Detector.run`` of all stages."""

    def __init__(self, device: int, frame_offsets: Sequence[int], fs: int, params: dict, mode: str = "reference",
                 channels: int = 1, options: int = 0, depth: int = 2, d: Optional[Design] = None,
                 det_free_cus: int = 48, env_priority: bool = True, env_masked: bool = False):
        torch = _torch()
        self.fo = np.ascontiguousarray(frame_offsets, dtype=np.int64)
        self.fs, self.params, self.mode, self.channels, self.options = fs, params, mode, channels, options
        self.d = d if d is not None else design(fs, params, log=False)
        self.env_det, self.det_det = Detector(device), Detector(device)
        # The envelope chain is a sequence of small launches: each needs a free
        # CU when it starts, and a detection kernel's workgroups hold a whole
        # CU's LDS for ~0.1 ms each.  So the detection stream leaves
        # `det_free_cus` CUs out of its mask (spread over the XCDs), and the
        # envelope stream has the higher priority for the CUs that do free up.
        if env_masked:
            self.s_env = cu_masked_stream(self.env_det.device, det_free_cus, only=True)
        else:
            self.s_env = torch.cuda.Stream(self.env_det.device, priority=-1 if env_priority else 0)
        self.s_det = cu_masked_stream(self.det_det.device, det_free_cus)
        self._own = [s for s in (self.s_env, self.s_det) if isinstance(s, torch.cuda.ExternalStream)]
        self.outs = [self.det_det.alloc(self.fo, self.d.ds, self.d.sr) for _ in range(max(2, depth))]
        self.ev_free = [None] * len(self.outs)
        self.pending = None
        self.k = 0
        self.ties_resolved = 0

    def _check(self, pend):
        """Batch `pend`'s tie check (its read-back was queued behind its
        detection); a resolution runs on the detection stream and re-marks
        when the batch's result set is free."""
        if pend is None:
            return
        torch = _torch()
        h, o, i = pend
        with torch.cuda.stream(self.s_det):
            r = self.det_det.tie_check_finish(h, o, self.params, N.STAGE_FLOOR | N.STAGE_PEAKS, self.options)
            if r:
                ev = torch.cuda.Event()
                ev.record(self.s_det)
                self.ev_free[i] = ev
        self.ties_resolved += r

    def submit(self, pcm) -> Result:
        torch = _torch()
        i = self.k % len(self.outs)
        o = self.outs[i]
        with torch.cuda.stream(self.s_env):
            if self.ev_free[i] is not None:
                self.s_env.wait_event(self.ev_free[i])
            self.env_det.run(pcm, self.fo, self.fs, self.params, mode=self.mode, stages=N.STAGE_ENVELOPE,
                             channels=self.channels, out=o, d=self.d, options=self.options)
            ev_env = torch.cuda.Event()
            ev_env.record(self.s_env)
        with torch.cuda.stream(self.s_det):
            self.s_det.wait_event(ev_env)
            self.det_det.run(None, self.fo, self.fs, self.params, mode=self.mode,
                             stages=N.STAGE_FLOOR | N.STAGE_PEAKS, channels=self.channels, out=o, d=self.d,
                             options=self.options)
            h = self.det_det.tie_check_start(o)
            ev_free = torch.cuda.Event()
            ev_free.record(self.s_det)
            self.ev_free[i] = ev_free
        # batch k - 1's tie check, with batch k's envelope and detection already queued
        prev, self.pending = self.pending, (h, o, i)
        self._check(prev)
        self.k += 1
        return o

    def finish(self):
        torch = _torch()
        prev, self.pending = self.pending, None
        self._check(prev)
        self.s_env.synchronize()
        self.s_det.synchronize()
        torch.cuda.current_stream(self.det_det.device).wait_stream(self.s_det)

    def close(self):
        """Drain, free both contexts and destroy the CU-masked stream(s): a
        stream left to the HIP runtime's exit-time teardown can outlive the
        tools that hooked it (rocprofv3 faulted there)."""
        if self.env_det is None:
            return
        self.s_env.synchronize()
        self.s_det.synchronize()
        self.env_det.close()
        self.det_det.close()
        for s in self._own:
            destroy_stream(s)
        self._own, self.env_det, self.det_det = [], None, None


def destroy_stream(s):
    """hipStreamDestroy of a stream cu_masked_stream made (torch does not own
    an ExternalStream's handle)."""
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipStreamDestroy(ctypes.c_void_p(s.cuda_stream))
    if rc != 0:
        raise N.BpmxError(f"hipStreamDestroy failed ({rc})")


def cu_masked_stream(device, free_cus: int, only: bool = False):
    """A torch stream on `device` whose kernels avoid the first `free_cus` CUs
    of the mask (or, with `only`, run on those alone).  hipExtStreamCreateWithCUMask:
    bit c of the mask is the (c / 8)-th CU of XCD c % 8, so the first
    `free_cus` bits are the same share of every XCD.  free_cus <= 0: an
    ordinary stream."""
    torch = _torch()
    if free_cus <= 0:
        return torch.cuda.Stream(device)
    hip = ctypes.CDLL("libamdhip64.so")
    total = torch.cuda.get_device_properties(device).multi_processor_count
    words = (total + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in (range(0, min(free_cus, total)) if only else range(min(free_cus, total), total)):
        mask[c // 32] |= 1 << (c % 32)
    st = ctypes.c_void_p()
    with torch.cuda.device(device):
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise N.BpmxError(f"hipExtStreamCreateWithCUMask failed ({rc})")
    return torch.cuda.ExternalStream(st.value, device=device)


def _torch_np_map():
    torch = _torch()
    return {np.dtype(np.uint8): torch.uint8, np.dtype(np.int16): torch.int16, np.dtype(np.int32): torch.int32,
            np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64}


class _PerThread(threading.local):
    def __init__(self):
        self.dets = {}


_default = _PerThread()


def default_detector(device: int = 0) -> Detector:
    """This thread's Detector on `device` (created on first use, in this thread:
    gui.py runs the analysis on a daemon worker thread, gui.py:181-187)."""
    det = _default.dets.get(device)
    if det is None:
        det = _default.dets[device] = Detector(device)
    return det
