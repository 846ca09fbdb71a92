"""Placement of ragged batches: recordings over ranks, and their
order inside one GPU batch.

Recordings are independent (no exchange), so placement is pure scheduling:

* ``lpt_partition`` — longest-processing-time-first over ranks: recordings in
  descending length, each to the rank with the least total so far (ties to
  the lower rank).  Every rank computes the same partition from the same
  lengths, so no collective is needed to agree on it.  Greedy LPT is within
  4/3 of the optimal makespan.
* ``longest_first`` — the order a rank hands its recordings to one
  ``bpmx_run``: the per-recording kernels give recording f workgroup f and the
  hardware dispatches workgroups in index order, so longest-first is LPT over
  the CUs and a long recording never starts last (the ragged C5 tail).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np


def longest_first(lengths: Sequence[int]) -> np.ndarray:
    """Permutation putting the longest recordings first (stable for equal lengths)."""
    n = np.asarray(lengths, dtype=np.int64)
    return np.argsort(-n, kind="stable")


def lpt_partition(lengths: Sequence[int], world: int) -> List[List[int]]:
    """Recording indices per rank; each rank's list is longest first."""
    if world < 1:
        raise ValueError("world must be >= 1")
    n = np.asarray(lengths, dtype=np.int64)
    load = np.zeros(world, dtype=np.int64)
    parts: List[List[int]] = [[] for _ in range(world)]
    for i in longest_first(n):
        r = int(np.argmin(load))                    # first minimum: ties go to the lower rank
        parts[r].append(int(i))
        load[r] += n[i]
    return parts


def makespan(lengths: Sequence[int], parts: List[List[int]]) -> int:
    n = np.asarray(lengths, dtype=np.int64)
    return max((int(n[p].sum()) if p else 0) for p in parts)


# ---------------------------------------------------------------- sharded runner
def _lengths(items) -> List[int]:
    """Frames per recording: array rows, or the WAV header of a path (memory-mapped, not read)."""
    out = []
    for it in items:
        if isinstance(it, str):
            from scipy.io import wavfile
            import warnings
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                _, a = wavfile.read(it, mmap=True)
            out.append(int(a.shape[0]))
            del a
        else:
            out.append(int(np.asarray(it).shape[0]))
    return out


def _load(it, fs):
    if isinstance(it, str):
        from .dropin import _read_wav
        return _read_wav(it)
    return fs, np.asarray(it)


def _detect_local(items, idx, fs, params, mode, detector):
    """The hot path over this rank's recordings: one ragged batch per (rate,
    sample format, channels), as dropin.analyze_wav_files groups them."""
    from . import _native as N
    from .design import design
    from .dropin import DISTANCE_MSG, PADLEN_MSG, _file_error
    res = {}
    groups = {}
    data = {}
    for i in idx:
        try:
            f, a = _load(items[i], fs)
        except Exception as exc:                        # unreadable file: reported for that file only
            res[i] = {"error": exc}
            continue
        data[i] = (f, a)
        groups.setdefault((int(f), a.dtype.str, 1 if a.ndim == 1 else a.shape[1]), []).append(i)
    for (f, _, _), ids in groups.items():
        d = None
        try:
            d = design(f, params, log=False)
            if d.distance < 1:
                raise ValueError(DISTANCE_MSG)
            out = detector.run_host([data[i][1] for i in ids], f, params, mode=mode, stages=N.STAGE_ALL,
                                    resolve_ties=True)
        except (ValueError, N.BpmxError) as exc:
            if isinstance(exc, N.BpmxError) and not exc.per_file:
                raise                                   # HIP / device failure: the rank fails, not the files
            for i in ids:
                short = d is not None and -(-data[i][1].shape[0] // d.ds) <= 15
                res[i] = {"error": ValueError(PADLEN_MSG) if short else exc}
            continue
        for i, r in zip(ids, out):
            err = _file_error(r["flags"], params, d.sr)
            res[i] = {"error": err} if err is not None else r
    return res


NMETA = 5          # per-file slab header: item index, raw peaks, final beats, BPM points, flags


def _pad_rows(rows: List[np.ndarray], width: int, fill, dtype) -> np.ndarray:
    out = np.full((len(rows), max(width, 1)), fill, dtype=dtype)
    for k, r in enumerate(rows):
        out[k, :len(r)] = r
    return out


def run_sharded(items: Sequence, params: dict, fs: Optional[int] = None, mode: str = "native",
                start_bpm_hint: Optional[float] = None, beats="native", detector=None,
                group=None, host_threads: int = 0, chunk_frames: int = 1 << 30) -> Optional[List[dict]]:
    """A ragged batch of independent recordings over the ranks of a
    torch.distributed process group (one process per GPU); the
    per-file loop it replaces is gui.py:202-251.

    * ``items``: WAV paths (each rank reads only its own files) or host PCM
      arrays at rate ``fs``; every rank passes the same list.
    * Placement: ``lpt_partition`` of the frame counts; every rank derives it
      from the same lengths, so no plan is exchanged.
    * Per rank: the hot path on its GPU (``detector``: an engine.Detector; one
      ragged batch per rate/format/channel group, cut into chunks of about
      ``chunk_frames`` frames), and the host beat stages of each chunk on
      ``host_threads`` host threads while the GPU runs the next chunk
      (``beats="native"``: libbpmx_host.so, beats.analyze_fast;
      ``"python"``: beats.analyze_recording; False: raw peaks only).
    * Result gather to rank 0 (RCCL under the "nccl" backend, gloo on CPU):
      one int64 slab [files, 4 + raw peaks + final beats] and one f64 slab
      [files, 2 x BPM-curve points] per rank, padded to the widest over all
      ranks (caps agreed by one all_reduce(MAX)); errors as objects.

    Returns, on rank 0, one dict per item in order: ``raw_peaks``,
    ``final_peaks``, ``bpm_times``, ``bpm`` (the smoothed curve that
    ``<base>_bpm_plot.csv`` holds, bpm_analysis.py:1463-1484), ``flags``,
    ``rank``, or ``error``; None on the other ranks."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if detector is None:
        from .engine import Detector
        detector = Detector(int(os.environ.get("LOCAL_RANK", "0")))
    lengths = _lengths(items)
    mine = lpt_partition(lengths, world)[rank]
    if host_threads <= 0:
        try:
            host_threads = max(1, min(16, len(os.sched_getaffinity(0))))
        except AttributeError:
            host_threads = 1
    chunks, cur, acc = [], [], 0                       # longest first (LPT order), ~chunk_frames each
    for i in mine:
        cur.append(i)
        acc += lengths[i]
        if acc >= chunk_frames:
            chunks.append(cur)
            cur, acc = [], 0
    if cur:
        chunks.append(cur)

    def host_stage(idx, det_res):
        out = []
        for i in idx:
            r = det_res[i]
            if "error" in r:
                out.append(FileResult(i, error=r["error"]))
                continue
            pk = np.asarray(r["peaks"], dtype=np.int64)
            if not beats:
                out.append(FileResult(i, raw_peaks=pk, flags=int(r["flags"])))
                continue
            if beats == "python":
                from .beats import analyze_recording
                try:
                    a = analyze_recording(r["env"], r["sr"], r["floor"], r["troughs"], pk, params, start_bpm_hint)
                except Exception as exc:               # per file, as the GUI loop catches it (gui.py:247-251)
                    out.append(FileResult(i, error=exc))
                    continue
                out.append(FileResult.from_analysis(i, pk, int(r["flags"]), a))
                continue
            from . import _host
            a = _host.beats(r["env"], r["sr"], r["floor"], pk, bparams, start_bpm_hint)
            if "error" in a:
                out.append(FileResult(i, error=a["error"]))
            else:
                out.append(FileResult(i, pk, a["final_peaks"], a["bpm_times"], a["bpm"], int(r["flags"])))
        return out

    bparams = None
    if beats and beats != "python":
        from . import _host
        bparams = _host.beat_params(params)
    from concurrent.futures import ThreadPoolExecutor
    rows: List[FileResult] = []
    with ThreadPoolExecutor(host_threads) as ex:
        futs = []
        for idx in chunks:                             # the GPU runs chunk k+1 while host threads take chunk k
            det_res = _detect_local(items, idx, fs, params, mode, detector)
            per = max(1, len(idx) // host_threads)
            futs += [ex.submit(host_stage, idx[a:a + per], det_res) for a in range(0, len(idx), per)]
        for fu in futs:
            rows += fu.result()
    dev = detector.device if (dist.is_initialized() and dist.get_backend(group) == "nccl") else None
    return gather_file_results(rows, len(items), group=group, device=dev)


class FileResult:
    """One recording's record for the result gather."""

    def __init__(self, index: int, raw_peaks=None, final_peaks=None, bpm_times=None, bpm=None, flags: int = 0,
                 error=None):
        self.index, self.flags, self.error = index, flags, error
        self.raw_peaks = np.zeros(0, np.int64) if raw_peaks is None else np.asarray(raw_peaks, np.int64)
        self.final_peaks = np.zeros(0, np.int64) if final_peaks is None else np.asarray(final_peaks, np.int64)
        self.bpm_times = np.zeros(0) if bpm_times is None else np.asarray(bpm_times, np.float64)
        self.bpm = np.zeros(0) if bpm is None else np.asarray(bpm, np.float64)

    @classmethod
    def from_analysis(cls, index: int, raw_peaks, flags: int, a: dict) -> "FileResult":
        """From beats.analyze_recording's dict: final beats and the smoothed BPM
        curve (the series ``<base>_bpm_plot.csv`` holds, bpm_analysis.py:1463-1484)."""
        m = a["final_metrics"]
        times = curve = None
        if m is not None and not m["smoothed_bpm"].empty:
            times, curve = m["bpm_times"], m["smoothed_bpm"].values
        return cls(index, raw_peaks, a["final_peaks"], times, curve, flags)


def gather_file_results(rows: List[FileResult], n_items: int, group=None, device=None) -> Optional[List[dict]]:
    """The final result gather: every rank's records to rank 0 as
    one int64 slab [files, NMETA + raw peaks + final beats] and one f64 slab
    [files, 2 x BPM-curve points], padded to the widest over all ranks (the caps
    agreed by one all_reduce(MAX)); RCCL under the "nccl" backend (``device``:
    this rank's GPU), gloo on CPU.  Errors travel as objects.  Returns the
    records in item order on rank 0 (None elsewhere)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    dev = device if device is not None else torch.device("cpu")
    caps = torch.tensor([len(rows), max([len(x.raw_peaks) for x in rows], default=0),
                         max([len(x.final_peaks) for x in rows], default=0),
                         max([len(x.bpm) for x in rows], default=0)], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(caps, op=dist.ReduceOp.MAX, group=group)
    nf, cp, cf, cb = (int(x) for x in caps.tolist())
    rows = list(rows) + [FileResult(-1)] * (nf - len(rows))
    meta = [[x.index, -1 if x.error is not None else len(x.raw_peaks), len(x.final_peaks), len(x.bpm), x.flags]
            for x in rows]
    islab = np.concatenate([np.asarray(meta, np.int64).reshape(nf, NMETA),
                            _pad_rows([x.raw_peaks for x in rows], cp, -1, np.int64),
                            _pad_rows([x.final_peaks for x in rows], cf, -1, np.int64)], axis=1)
    fslab = np.concatenate([_pad_rows([x.bpm_times for x in rows], cb, np.nan, np.float64),
                            _pad_rows([x.bpm for x in rows], cb, np.nan, np.float64)], axis=1)
    ti = torch.from_numpy(np.ascontiguousarray(islab)).to(dev)
    tf = torch.from_numpy(np.ascontiguousarray(fslab)).to(dev)
    errors = {x.index: x.error for x in rows if x.error is not None}
    if world > 1:
        gi = [torch.empty_like(ti) for _ in range(world)] if rank == 0 else None
        gf = [torch.empty_like(tf) for _ in range(world)] if rank == 0 else None
        dist.gather(ti, gi, dst=0, group=group)
        dist.gather(tf, gf, dst=0, group=group)
        ge = [None] * world if rank == 0 else None
        dist.gather_object(errors, ge, dst=0, group=group)
    else:
        gi, gf, ge = [ti], [tf], [errors]
    if rank != 0:
        return None
    cpf = max(cp, 1)
    out: List[dict] = [None] * n_items
    for r, (si, sf) in enumerate(zip(gi, gf)):
        si, sf = si.cpu().numpy(), sf.cpu().numpy()
        cb1 = sf.shape[1] // 2
        for row_i, row_f in zip(si, sf):
            i, npk, nfin, nb, flags = (int(x) for x in row_i[:NMETA])
            if i < 0:
                continue
            if npk < 0:
                out[i] = {"error": ge[r][i], "rank": r}
                continue
            o = NMETA + cpf
            out[i] = {"raw_peaks": row_i[NMETA:NMETA + npk].copy(), "final_peaks": row_i[o:o + nfin].copy(),
                      "bpm_times": row_f[:nb].copy(), "bpm": row_f[cb1:cb1 + nb].copy(), "flags": flags, "rank": r}
    return out
