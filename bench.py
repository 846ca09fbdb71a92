"""Benchmark: audio-samples/sec of filter + envelope + noise floor + peaks
(BASELINE.json metric) on a synthetic batch of 1024 x 60 s 44.1 kHz mono int16
recordings per GPU, inputs resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode native|reference]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One process per GPU; files are sharded (weak scaling: every rank processes its
own 1024 recordings, no data-path collective).  After the timed steps every
file's raw peaks, final beats and BPM curve go to rank 0 over RCCL (the only
collective besides the max-time all_reduce).  Rank 0 prints one JSON line.

`python bench.py --gpus N` without WORLD_SIZE in the environment starts the N
ranks itself (a `torch.distributed.run` child process, before anything touches
the GPU) and exits with its status; a rank whose WORLD_SIZE differs from
--gpus refuses to run.  `--cpu-stub` (tests only) swaps the GPU detector for
tests/bench_stub.py's oracle-backed double over gloo, so the multi-rank path
runs on a CPU-only host; its line says so and is never a measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "audio-samples/sec (filter+envelope+peaks), 1024x60s@44.1kHz batch, 1 & 8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# flags both sides report: static / draft / NaN floor (BPMX_F_TOO_SHORT and
# BPMX_F_BAD_WINDOW are library-side input checks, compared by the tests)
FLOOR_FLAGS = 1 | 2 | 4 | 32 | 64      # fallbacks and the decisive-tie reports (bpmx.h)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", default="native", choices=["native", "reference"])
    ap.add_argument("--files", type=int, default=1024, help="recordings per GPU (weak scaling, the default line)")
    ap.add_argument("--files-total", type=int, default=0,
                    help="strong scaling: this many recordings in the whole job, split evenly over the ranks "
                         "(BASELINE C4: --gpus 8 --files-total 4096; the metric's 1024-file batch at any N: 1024); "
                         "0: --files per GPU")
    ap.add_argument("--secs", type=float, default=60.0)
    ap.add_argument("--fs", type=int, default=44100)
    ap.add_argument("--cpu-files", type=int, default=-1, help="CPU baseline sample size (-1: auto, 0: skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pcie-steps", type=int, default=3, help="steps of the PCIe-inclusive side measurement (0: skip)")
    ap.add_argument("--host-beat-files", type=int, default=16,
                    help="files of the side measurement of the host beat stages (0: skip)")
    ap.add_argument("--options", type=int, default=0, help="bpmx_option bits (diagnostics; 0 = defaults)")
    ap.add_argument("--tie-check", default="on", choices=["on", "off"],
                    help="the timed step's decisive-tie check (off: diagnostic A/B of its cost only)")
    ap.add_argument("--batch-pipeline", default="auto", choices=["auto", "on", "off"],
                    help="timed steps through engine.BatchPipeline (batch k+1's envelope beside batch k's "
                         "detection, two contexts and streams); auto: on in reference mode")
    ap.add_argument("--contexts", type=int, default=4,
                    help="side measurement: the batch split over K contexts on K streams (0: skip)")
    ap.add_argument("--exact-steps", type=int, default=5,
                    help="side measurement: steps with the input-dependent exact shortcuts off "
                         "(BPMX_OPT_DRAFT_FULL | BPMX_OPT_ROLLQ_NOPRUNE; 0: skip)")
    ap.add_argument("--workload", default="metric", choices=["metric", "c5"],
                    help="metric: BASELINE's headline (1024 x 60 s 44.1 kHz mono per GPU); c5: BASELINE config C5, "
                         "64 x U[10, 30] min 96 kHz stereo per GPU (512 over 8 GPUs), ragged, LPT over ranks")
    ap.add_argument("--parity-files", type=int, default=16,
                    help="N > 1: files per rank checked against the oracle (N = 1 checks every file)")
    ap.add_argument("--c5-files", type=int, default=512,
                    help="C5: recordings in the whole job (LPT over the ranks; BASELINE C5 is 512 over 8 GPUs)")
    ap.add_argument("--c5-chunk-gb", type=float, default=48.0,
                    help="C5: a rank's recordings run in HBM-resident chunks of at most this much PCM")
    ap.add_argument("--c5-contexts", type=int, default=3,
                    help="C5: a chunk's recordings run as this many LPT-balanced sub-batches on as many library "
                         "contexts and streams, so one sub-batch's latency-bound kernels fill another's gaps "
                         "(3: the box's GPU_MAX_HW_QUEUES = 4 leaves three hardware queues beside the null "
                         "stream's; a fourth stream shares one and serialises)")
    ap.add_argument("--c5-parity-files", type=int, default=-1,
                    help="C5: each rank's shortest recordings checked against the oracle (-1: every recording of "
                         "the rank; ~15 s of 16-thread oracle time per 64 recordings)")
    ap.add_argument("--dropin-files", type=int, default=3,
                    help="side measurement: per-file latency of the reference's call sequence through the "
                         "drop-in on 60 s WAV files (0: skip)")
    ap.add_argument("--undecided-mult", type=float, default=1.0,
                    help="side measurement: the step with trough_rejection_multiplier set to this, which leaves "
                         "many troughs inside the draft-floor bracket (decided by draft_point); 0: skip")
    ap.add_argument("--real-env-steps", type=int, default=5,
                    help="side measurement: the detection stages (noise floor + raw peaks) on 60 s windows of a "
                         "real recording's envelope (the reference's vulpine sample, tests/golden) beside the "
                         "same stages on the synthetic batch's envelopes (0: skip)")
    ap.add_argument("--cpu-stub", action="store_true",
                    help="TESTS ONLY: oracle-backed detector (tests/bench_stub.py) over gloo on CPU ranks")
    a = ap.parse_args(argv)
    if a.cpu_stub:          # the side measurements need device memory and streams
        a.pcie_steps = a.contexts = a.exact_steps = a.dropin_files = a.real_env_steps = 0
        a.undecided_mult = 0.0
        a.c5_contexts = 1
    return a


def launch_ranks(argv, n: int) -> int:
    """`--gpus N` without a launcher: start N ranks as one torch.distributed.run
    child (one process per GPU, rendezvous on 127.0.0.1) and return its exit
    status.  Runs before anything initialises the GPU; never exec."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(cmd, env=env)


def setup_rank(args):
    """(world, rank, local rank, detector, backend) of this process.  Refuses a
    world size other than --gpus, so a line never claims GPUs it did not use."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; refusing to report")
    backend = "gloo" if args.cpu_stub else "nccl"
    if args.cpu_stub:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from bench_stub import StubDetector as Detector
    else:
        from bpm_analysis_amd.engine import Detector
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    return world, rank, local, Detector(local), backend


def sync(det):
    """Wait for the detector's device (no-op for the CPU stub)."""
    if det.device.type == "cuda":
        import torch
        torch.cuda.synchronize(det.device)


def algorithmic_bytes(mode: str, n_files: int, n_frames: int, nd: int, ds: int, channels: int = 1) -> dict:
    """Algorithmic HBM bytes PER STEP of each kernel label (summed over its
    launches in one step): the bytes the algorithm must
    move, not what the implementation happens to move.  Uniform lengths."""
    return algorithmic_bytes_total(mode, n_files, n_files * n_frames, n_files * nd, channels)


def algorithmic_bytes_total(mode: str, F: int, frames: int, nd: int, channels: int = 1) -> dict:
    """The same for a ragged batch: F recordings, `frames` frames and `nd`
    decimated samples in total."""
    nb = nd - F
    common = {
        "k_quantile": nd * 8,                          # env read once
        "k_quantile_reg": nd * 8,
        "k_block_stats": nd * 8,
        "k_find_peaks[troughs]": nd * 8,
        "k_find_peaks[peaks]": nd * 16,                # env + floor
        "k_draft_bounds": nd // 76 * 16,               # ~1 raw trough per 76 samples x (position, value)
        # the noise floor after the draft bracket (k_floor_wm: sanitize, the final rolling
        # quantile interpolated in-kernel from the kept troughs' values, the fallbacks): floor
        # out; the full-draft pass (k_rollq_wm) runs only for recordings whose bracket stayed
        # open past draft_point (none on this workload)
        "k_floor_wm": nd * 8,
        "k_rollq_wm": 0,
        "k_rollq_wm[full]": 0,                          # unpruned variant: recordings the pruned one flags (none here)
        "k_init_out": 0,
        "k_rolling_quantile": nd * 16,
        "k_floor_final": 0, "k_sanitize": 0, "k_interp": 0,
    }
    if mode == "native":
        return dict(common, **{
            "k_native_blocks": frames * channels * 2,                 # every PCM sample read once
            "k_native_carry": nb // 64 * 128 + F * 64 * 16 * 8,       # tile carries in/out, partial tile
            "k_native_yd": nb * (8 + 8),                              # gamma in, yd out
            "k_hilbert_env": nd * (8 + 8),                            # yd in, env out (transform in LDS)
        })
    # reference: the picked samples, y kept in scratch (written fwd, rewritten bwd, read twice), env written once
    return dict(common, **{"k_envelope_ref": nd * channels * 2 + (nd + 30 * F) * 8 * 4 + nd * 8})


# launch labels -> kernel names in the rocprofv3 PMC summary
PMC_NAMES = {"k_native_blocks": ("k_native_blocks_mfma", "k_native_blocks_dma", "k_native_blocks_i16",
                                 "k_native_blocks_gen"),
             "k_rollq_wm": ("k_rollq_wm_t",),
             "k_find_peaks[troughs]": ("k_find_peaks[troughs]", "k_find_peaks_lds", "k_find_peaks"),
             "k_find_peaks[peaks]": ("k_find_peaks[peaks]", "k_find_peaks_lds", "k_find_peaks")}


def pmc_traffic(mode: str, kernel: str, workload: str, launches_per_step: float):
    """HBM bytes per step of `kernel` from the committed rocprofv3 PMC summary
    (tools/pmc_traffic.py: mean bytes per dispatch, FETCH_SIZE doubled per the
    gfx950 calibration) times its launches per step, or None."""
    path = os.path.join(REPO, "profiles", f"pmc_traffic_{mode}.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    if d.get("workload") != workload:
        return None
    for name in PMC_NAMES.get(kernel, (kernel,)):
        k = d.get("kernels", {}).get(name)
        if k is not None:
            return int(k["hbm_bytes_per_launch"] * launches_per_step)
    return None


def cpu_threads():
    """(threads used, CPUs in this process's affinity mask, os.cpu_count()).

    The CPU leg runs one thread per CPU of the affinity mask, capped by
    OMP_NUM_THREADS when that is set: the GPU pool sets it to the host-CPU
    share of one GPU (16), and os.cpu_count() there shows the whole machine."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    share = int(omp) if omp.isdigit() and int(omp) > 0 else aff
    return max(1, min(aff, share)), aff, os.cpu_count() or aff


def _cpu_model() -> str:
    cpu = platform.processor() or platform.machine()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return cpu


def oracle_outputs(mode: str, fs: int, n_frames: int, seeds, params: dict, threads: int):
    """The oracle (C restatement of the reference path) on the recordings with
    the given seeds: (per-file dicts, wall seconds of the detection itself).
    Input synthesis is untimed; each worker drops its PCM after use."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O
    d = O.derive(fs, params)
    with ThreadPoolExecutor(threads) as ex:
        pcms = list(ex.map(lambda s: O.synth(int(s), n_frames, fs, 1), seeds))

    def one(k):
        pcm = pcms[k]
        env = O.preprocess_ref(pcm, d) if mode == "reference" else O.preprocess_native(pcm, d)
        fl, tr, flags = O.noise_floor(env, d, params)
        pk = O.raw_peaks(env, fl, d, params)
        pcms[k] = None
        return {"env": env, "floor": fl, "troughs": tr, "peaks": pk, "flags": flags}

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        outs = list(ex.map(one, range(len(pcms))))
    return outs, time.perf_counter() - t0


TIE_BITS = 32 | 64                      # BPMX_F_TROUGH_TIE | BPMX_F_PEAK_TIE: decisive tie left open
ORDERED_BITS = 128 | 256                # BPMX_F_*_ORDERED: re-decided in numpy's argsort order


def numpy_order_expected(o: dict, fs: int, params: dict) -> dict:
    """The oracle's troughs, floor, flags and peaks for the oracle envelope
    o["env"] with find_peaks' distance filter in numpy's own argsort order
    (what a tie-resolved GPU recording must equal, bpm_analysis.py:1070 / :227)."""
    from oracle import oracle as O
    d = O.derive(fs, params)
    e = np.ascontiguousarray(o["env"])
    fl, tr, flags, _ = O.noise_floor_numpy_order(e, d, params)
    pk = O.find_peaks_numpy_order(e, height=fl, distance=d.distance,
                                  prominence=O.quantile(e, params["peak_prominence_quantile"]))
    return dict(o, floor=fl, troughs=tr, peaks=pk, flags=int(flags))


def compare_outputs(gpu: list, cpu: list, exact_env: bool, fs: int = 0, params: dict | None = None) -> dict:
    """Per-file parity of the GPU batch against the oracle: every trough and
    peak index and the fallback flags bit-exact; env and floor bit-exact in
    reference mode, within 1e-9 x max|env| in native mode (north_star asks for
    1e-5 relative).  A GPU recording re-decided in numpy's order (an ORDERED
    flag bit) is compared with the numpy-order oracle instead (needs `fs` and
    `params`); one still carrying a decisive-tie bit counts in
    `ties_unresolved`, and `ok` requires none.  Returns counts over files and
    the worst relative errors."""
    n = len(cpu)
    pe = te = fe = 0
    env_rel = floor_rel = 0.0
    bad = []
    unresolved = resolved = 0
    for f, (g, o) in enumerate(zip(gpu, cpu)):
        gfl = int(g["flags"])
        unresolved += bool(gfl & TIE_BITS)
        if gfl & ORDERED_BITS:
            resolved += 1
            if params is not None:
                o = numpy_order_expected(o, fs, params)
        scale = float(np.max(np.abs(o["env"]))) or 1.0
        de = float(np.max(np.abs(g["env"] - o["env"]))) / scale
        df = np.abs(g["floor"] - o["floor"])
        df = float(np.nanmax(df)) / scale if np.any(np.isfinite(df)) else 0.0
        if not np.array_equal(np.isnan(g["floor"]), np.isnan(o["floor"])):
            df = float("inf")
        env_rel, floor_rel = max(env_rel, de), max(floor_rel, df)
        p_ok = np.array_equal(g["peaks"], o["peaks"])
        t_ok = np.array_equal(g["troughs"], o["troughs"])
        fmask = FLOOR_FLAGS & ~TIE_BITS if gfl & ORDERED_BITS else FLOOR_FLAGS
        f_ok = (gfl & fmask) == (int(o["flags"]) & fmask)
        pe += p_ok
        te += t_ok
        fe += f_ok
        if not (p_ok and t_ok and f_ok) and len(bad) < 8:
            bad.append(f)
    tol = 0.0 if exact_env else 1e-9
    return {"files": n, "peaks_equal": pe, "troughs_equal": te, "flags_equal": fe,
            "env_max_rel": env_rel, "floor_max_rel": floor_rel, "env_tol": tol,
            "ties_resolved": resolved, "ties_unresolved": unresolved,
            "ok": pe == n and te == n and fe == n and env_rel <= tol and floor_rel <= tol and unresolved == 0,
            "mismatched_files": bad}


def cpu_baseline(mode: str, fs: int, n_frames: int, seed0: int, n_files: int, params: dict, gpu_host: list):
    """The CPU oracle on exactly the GPU batch's recordings (seeds seed0 + f),
    timed, and the GPU outputs compared against it file by file."""
    threads, aff, ncpu = cpu_threads()
    outs, dt = oracle_outputs(mode, fs, n_frames, [seed0 + f for f in range(n_files)], params, threads)
    parity = compare_outputs(gpu_host[:n_files], outs, exact_env=(mode == "reference"), fs=fs, params=params)
    base = {"value": n_files * n_frames / dt, "unit": "audio-samples/s", "cores": threads, "kind": "port",
            "affinity_cpus": aff, "os_cpu_count": ncpu,
            "sample": f"the GPU batch's own {n_files} recordings (seeds {seed0}..{seed0 + n_files - 1}, "
                      f"{n_frames / fs:.0f} s {fs} Hz mono int16), {mode} mode, oracle/bpmx_oracle.c + numpy FFT "
                      f"on {threads} threads of {_cpu_model()}; {dt:.2f} s wall"}
    return base, parity


def shard_seed0(rank: int, files_per_gpu: int) -> int:
    """Weak scaling: rank r synthesises files r*F .. r*F+F-1 (disjoint shards)."""
    return rank * files_per_gpu


def shard_files(args, rank: int, world: int):
    """(first recording index = seed, recordings on this rank, recordings in the job).

    Weak scaling (default): --files per rank, rank r holding r*F .. r*F+F-1.
    Strong scaling (--files-total T): the job's T equal-length recordings split
    into contiguous, as-even-as-possible runs (the LPT placement of equal
    lengths, gui.py:202-251's loop sharded); a rank may hold none."""
    if args.files_total > 0:
        lo, hi = rank * args.files_total // world, (rank + 1) * args.files_total // world
        return lo, hi - lo, args.files_total
    return shard_seed0(rank, args.files), args.files, world * args.files


def reduce_results(elapsed: float, n_peaks, world: int, rank: int):
    """Max wall time over ranks, and the final result gather: every shard's
    per-file raw-peak counts to rank 0 (RCCL on the GPU box, gloo in the CPU
    tests).  The only collectives of the job."""
    import torch
    import torch.distributed as dist
    if world <= 1:
        return elapsed, int(n_peaks.sum())
    tt = torch.tensor([elapsed], dtype=torch.float64, device=n_peaks.device)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    counts = n_peaks.sum(dtype=torch.int64).reshape(1)     # ranks may hold different file counts (--files-total)
    gathered = [torch.empty_like(counts) for _ in range(world)] if rank == 0 else None
    dist.gather(counts, gathered, dst=0)
    total = int(sum(int(g.sum()) for g in gathered)) if rank == 0 else 0
    return float(tt.item()), total


def c5_lengths(n_files: int, fs: int = 96000, seed: int = 2025):
    """BASELINE config C5: recordings of U[10, 30] minutes (whole seconds), seeded."""
    rng = np.random.default_rng(seed)
    return (rng.integers(600, 1801, size=n_files) * fs).astype(np.int64)


def c5_chunks(lengths, mine, channels: int, budget_bytes: int):
    """A rank's recordings (longest first) cut into HBM-resident chunks of at
    most `budget_bytes` of int16 PCM (at least one recording each)."""
    chunks, cur, acc = [], [], 0
    for i in mine:
        b = int(lengths[i]) * channels * 2
        if cur and acc + b > budget_bytes:
            chunks.append(cur)
            cur, acc = [], 0
        cur.append(int(i))
        acc += b
    if cur:
        chunks.append(cur)
    return chunks


def run_c5(args):
    """Side workload (never the driver's headline): BASELINE config C5, 512
    ragged 10-30 min 96 kHz stereo int16 recordings in the whole job (strong
    scaling: `--c5-files` is fixed whatever N), native mode.  Recordings are
    placed over ranks by shard.lpt_partition of the frame counts (every rank
    derives the same placement) and each rank synthesises its own in HBM (seed
    = global recording index).  A rank runs its recordings longest first in
    chunks of at most `--c5-chunk-gb` of PCM (512 recordings are ~236 GB, the
    whole of one GPU's HBM at N = 1); each chunk is resident before its timed
    steps, and a step is one pass over every chunk.  Chunk rounds are
    bracketed by barriers, so the step time is the slowest rank's.  Prints one
    JSON line."""
    import torch
    import torch.distributed as dist

    from bpm_analysis_amd import DEFAULT_PARAMS
    from bpm_analysis_amd.design import design
    from bpm_analysis_amd.shard import FileResult, gather_file_results, lpt_partition

    world, rank, local, det, backend = setup_rank(args)
    params = dict(DEFAULT_PARAMS, save_filtered_wav=False)
    fs, ch = 96000, 2
    K = max(1, args.c5_contexts)
    dets = [det] + [type(det)(local) for _ in range(K - 1)]
    streams = [torch.cuda.Stream(det.device) for _ in range(K)] if K > 1 else [None]
    lengths = c5_lengths(args.c5_files, fs)
    mine = lpt_partition(lengths, world)[rank]
    d = design(fs, params, log=False)
    chunks = c5_chunks(lengths, mine, ch, int(args.c5_chunk_gb * 2 ** 30))
    n_rounds = len(chunks)
    if world > 1:                       # every rank takes part in every chunk round
        t = torch.tensor([n_rounds], dtype=torch.int64, device=det.device if backend == "nccl" else None)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        n_rounds = int(t.item())
    npar = len(mine) if args.c5_parity_files < 0 else args.c5_parity_files
    pick = set(sorted(mine, key=lambda i: lengths[i])[:npar]) if not args.no_cpu else set()
    kept, rows, kprof = {}, [], {}
    ties_c5 = [0]                       # recordings the steps' tie checks re-decided
    frames = nd_tot = 0
    elapsed = 0.0
    for ci in range(n_rounds):
        idx = chunks[ci] if ci < len(chunks) else []
        step = None
        if idx:
            # the chunk as K LPT-balanced sub-batches, one per context and stream
            subs = []
            for k, g in enumerate(lpt_partition(lengths[idx], K)):
                if not g:
                    continue
                gi = [idx[j] for j in g]
                fo = np.concatenate([[0], np.cumsum(lengths[gi])]).astype(np.int64)
                pcm = dets[k].synth(fo, fs, ch, seeds=[100_000 + i for i in gi])
                out = dets[k].alloc(fo, d.ds, d.sr)
                frames += int(fo[-1])
                nd_tot += int(out.doff[-1])
                subs.append((k, gi, fo, pcm, out))

            def run_sub(sub):
                k, _, fo, pcm, out = sub
                dets[k].run(pcm, fo, fs, params, mode="native", channels=ch, out=out, d=d, options=args.options)

            def step():
                # every sub-batch's run, then its decisive-tie check (engine.resolve_ties)
                checks = []
                for sub in subs:
                    if streams[sub[0]] is None:
                        run_sub(sub)
                        checks.append((sub, dets[sub[0]].tie_check_start(sub[4]), None))
                    else:
                        with torch.cuda.stream(streams[sub[0]]):
                            run_sub(sub)
                            checks.append((sub, dets[sub[0]].tie_check_start(sub[4]), streams[sub[0]]))
                for sub, h, st in checks:
                    if st is None:
                        ties_c5[0] += dets[sub[0]].tie_check_finish(h, sub[4], params, 7, args.options)
                    else:
                        with torch.cuda.stream(st):
                            ties_c5[0] += dets[sub[0]].tie_check_finish(h, sub[4], params, 7, args.options)

            # per-kernel profile: the sub-batches one after another (untimed)
            for sub in subs:
                dk = dets[sub[0]]
                dk.profile(True)
                for _ in range(max(1, args.warmup)):
                    run_sub(sub)
                sync(dk)
                dk.profile(False)
                for kn, (c, t) in dk.profile_read().items():
                    c0, t0 = kprof.get(kn, (0, 0.0))
                    kprof[kn] = (c0 + c, t0 + t)
            step()
            sync(det)
        if world > 1:
            dist.barrier()
        sync(det)
        t0 = time.perf_counter()
        if step is not None:
            for _ in range(args.steps):
                step()
        sync(det)
        if world > 1:
            dist.barrier()
        elapsed += time.perf_counter() - t0
        if idx:
            for k, gi, fo, pcm, out in subs:
                host = out.to_host()
                for j, i in enumerate(gi):
                    rows.append(FileResult(i, raw_peaks=host[j]["peaks"], flags=host[j]["flags"]))
                    if i in pick:
                        kept[i] = {kk: (v.copy() if isinstance(v, np.ndarray) else v) for kk, v in host[j].items()}
                del host
            del subs, step
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=det.device if backend == "nccl" else None)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    # parity: this rank's shortest recordings against the oracle (bounded CPU time)
    parity = None
    if pick:
        from oracle import oracle as O
        order = sorted(pick)

        def one(i):
            o = O.detect(O.synth(100_000 + i, int(lengths[i]), fs, ch), fs, params, mode="native")
            return {kk: o[kk] for kk in ("env", "floor", "troughs", "peaks", "flags")}

        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max(1, min(len(order), cpu_threads()[0]))) as ex:
            outs = list(ex.map(one, order))
        parity = compare_outputs([kept[i] for i in order], outs, exact_env=False, fs=fs, params=params)
        parity["files_checked_rank0"] = order
        parity["tie_flagged_in_steps"] = ties_c5[0]
        if world > 1:
            cnt = torch.tensor([parity["files"], parity["peaks_equal"], parity["troughs_equal"],
                                parity["flags_equal"], 0 if parity["ok"] else 1, parity["ties_unresolved"],
                                parity["ties_resolved"], ties_c5[0]], dtype=torch.float64,
                               device=det.device if backend == "nccl" else None)
            dist.all_reduce(cnt)
            c = [int(x) for x in cnt.tolist()]
            parity.update(files=c[0], peaks_equal=c[1], troughs_equal=c[2], flags_equal=c[3],
                          ok=c[4] == 0, ranks=world, ties_unresolved=c[5], ties_resolved=c[6],
                          tie_flagged_in_steps=c[7])
    allres = gather_file_results(rows, len(lengths), device=det.device if (world > 1 and backend == "nccl") else None)
    if rank == 0:
        ms = elapsed / args.steps * 1e3
        total = int(lengths.sum()) * ch
        wsteps = max(1, args.warmup)
        kernels = {k: {"launches": c, "avg_ms": round(t / c, 4), "share": round(t / wsteps / ms, 4)}
                   for k, (c, t) in sorted(kprof.items())}
        roof = None
        if "k_native_blocks" in kprof:
            c, t = kprof["k_native_blocks"]
            kms = t / wsteps
            ach = frames * ch * 2 / (kms / 1e3) / 1e9
            roof = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None, "kernel": "k_native_blocks",
                    "kernel_ms_per_step_rank0": round(kms, 4), "algorithmic_bytes_per_step_rank0": frames * ch * 2}
        step_bytes = total * 2
        line = {"metric": "audio-samples/sec (filter+envelope+peaks), C5: 512 x 10-30 min 96 kHz stereo over 8 GPUs",
                "value": total / (elapsed / args.steps), "unit": "audio-samples/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "f64",
                "data": "cpu-stub (tests only; not a measurement)" if args.cpu_stub else "synthetic",
                "config": {"workload": f"C5: {len(lengths)} x U[10,30] min 96000 Hz stereo int16 recordings in the "
                                       f"job, LPT over {world} ranks, HBM-resident chunks of <= "
                                       f"{args.c5_chunk_gb:g} GiB PCM, each as {K} LPT sub-batches on {K} "
                                       f"contexts/streams, native mode",
                           "recordings_rank0": len(mine), "chunks_rank0": len(chunks), "frames_rank0": frames,
                           "decimated_rank0": nd_tot, "parallelism": f"file-sharded x{world}"},
                "roofline": roof,
                "pipeline": {"hbm_bytes_per_step": step_bytes,
                             "achieved_GBps": round(step_bytes / (ms / 1e3) / 1e9, 1),
                             "frac_of_peak": round(step_bytes / (ms / 1e3) / 1e9 / (HBM_PEAK_GBS * world), 5)},
                "parity": parity, "kernels_rank0": kernels,
                "result_gather": {"files": sum(1 for r in allres if r is not None),
                                  "peaks": int(sum(len(r["raw_peaks"]) for r in allres
                                                   if r is not None and "raw_peaks" in r))}}
        print(json.dumps(line), flush=True)
    for x in dets[1:]:
        x.close()
    if world > 1:
        dist.destroy_process_group()


def dropin_latency(device: int, n_files: int, fs: int, secs: float, params: dict, mode: str) -> dict:
    """Per-file latency of the reference's own call sequence for one WAV
    (`analyze_wav_file`, bpm_analysis.py:1731-1740): preprocess_audio ->
    _calculate_dynamic_noise_floor -> PeakClassifier._find_raw_peaks twice
    (preliminary pass :1635 and main pass :1740, both via :89), through the
    drop-in (dropin.py) on 60 s int16 WAVs written to a temporary directory.
    Side measurement beside BASELINE's 28.9 ms/file (reference, one core, the
    first three calls); the beat stages in between are not timed here."""
    import tempfile

    import torch
    from scipy.io import wavfile

    from bpm_analysis_amd import dropin
    from bpm_analysis_amd.engine import default_detector
    det = default_detector(device)
    n = int(round(secs * fs))
    p = dict(params, save_filtered_wav=False, bpmx_mode=mode)
    times = []
    with tempfile.TemporaryDirectory() as tmp:
        paths = []
        for f in range(n_files + 1):              # file 0 warms up the path (plans, scratch)
            fo = np.array([0, n], dtype=np.int64)
            pcm = det.synth(fo, fs, 1, seed0=50_000 + f).cpu().numpy()
            path = os.path.join(tmp, f"dropin_{f}.wav")
            wavfile.write(path, fs, pcm)
            paths.append(path)
        torch.cuda.synchronize(det.device)
        for k, path in enumerate(paths):
            t0 = time.perf_counter()
            env, sr = dropin.preprocess_audio(path, p, tmp)
            floor, troughs = dropin._calculate_dynamic_noise_floor(env, sr, p)
            pk1 = dropin.find_raw_peaks(env, sr, p, floor.values)
            pk2 = dropin.find_raw_peaks(env, sr, p, floor.values)
            dt = time.perf_counter() - t0
            if k > 0:
                times.append(dt)
            assert np.array_equal(pk1, pk2)
    return {"mode": mode, "files": n_files, "ms_per_file": round(float(np.median(times)) * 1e3, 3),
            "ms_min": round(min(times) * 1e3, 3), "calls": "preprocess_audio + _calculate_dynamic_noise_floor "
            "+ 2 x _find_raw_peaks (WAV read included)", "reference_ms_per_file_1core": 28.9}


def main(args):
    import torch
    import torch.distributed as dist

    from bpm_analysis_amd import DEFAULT_PARAMS
    from bpm_analysis_amd.design import design

    world, rank, local, det, backend = setup_rank(args)
    cdev = det.device if backend == "nccl" else None          # collectives' tensors: the GPU under RCCL
    params = dict(DEFAULT_PARAMS)
    params["save_filtered_wav"] = False
    fs = args.fs
    seed0, F, total_files = shard_files(args, rank, world)
    if F < 1:
        raise SystemExit(f"bench.py: rank {rank} holds no recording (--files-total {args.files_total} over {world})")
    n = int(round(args.secs * fs))
    d = design(fs, params, log=False)
    fo = np.arange(F + 1, dtype=np.int64) * n
    pcm = det.synth(fo, fs, 1, seed0=seed0)
    out = det.alloc(fo, d.ds, d.sr)
    nd = -(-n // d.ds)

    def step(o=None):
        det.run(pcm, fo, fs, params, mode=args.mode, out=out if o is None else o, d=d, options=args.options)

    # The timed step is the drop-in's whole contract: the run, then the
    # decisive-tie check (engine.resolve_ties: recordings whose find_peaks
    # distance filter met equal heights are re-decided in numpy's argsort
    # order, bpm_analysis.py:1070 / :227).  Two result sets alternate, so the
    # check of step k (a flags read-back; a launch only when a bit is set)
    # waits for step k while step k + 1 is already queued.
    from bpm_analysis_amd import _native as N
    outs_pp = [out, det.alloc(fo, d.ds, d.sr)]
    ties = {"raised": 0, "resolved": 0}

    def run_steps(k_steps):
        pend = None
        for k in range(k_steps):
            o = outs_pp[k & 1]
            step(o)
            if args.tie_check == "off":
                continue
            h = det.tie_check_start(o)
            if pend is not None:
                r = det.tie_check_finish(pend[0], pend[1], params, N.STAGE_ALL, args.options)
                ties["raised"] += r
            pend = (h, o)
        if pend is not None:
            ties["raised"] += det.tie_check_finish(pend[0], pend[1], params, N.STAGE_ALL, args.options)
        return outs_pp[(k_steps - 1) & 1] if k_steps > 0 else out

    abytes = algorithmic_bytes(args.mode, F, n, nd, d.ds)
    # warmup with every launch bracketed by events: picks the dominant kernel
    det.profile(True)
    run_steps(args.warmup)
    sync(det)
    det.profile(False)
    wprof = {k: v for k, v in det.profile_read().items() if k in abytes}
    dom = max(wprof, key=lambda k: wprof[k][1]) if wprof else ""
    if world > 1:
        dist.barrier()
    # timed steps: events around the dominant kernel's launches only, so the
    # step time carries no per-launch event overhead
    # Reference mode's envelope is a few waves of sequential passes, so a
    # stream of batches runs batch k+1's envelope beside batch k's detection
    # (engine.BatchPipeline, two contexts on two streams): a step is still one
    # batch through every stage and its tie check, the K steps overlap.
    piped = args.batch_pipeline == "on" or (args.batch_pipeline == "auto" and args.mode == "reference")
    piped = piped and not args.cpu_stub
    pipe = None
    if piped:
        from bpm_analysis_amd.engine import BatchPipeline
        pipe = BatchPipeline(local, fo, fs, params, mode=args.mode, options=args.options, d=d)
        for _ in range(2):
            pipe.submit(pcm)
        pipe.finish()
        pipe.ties_resolved = 0
        for x in (pipe.env_det, pipe.det_det):
            x.profile_only(dom)
            x.profile(True)
    else:
        det.profile_only(dom)
        det.profile(True)
    sync(det)
    ties["raised"] = 0
    t0 = time.perf_counter()
    if piped:
        for _ in range(args.steps):
            last = pipe.submit(pcm)
        pipe.finish()
    else:
        last = run_steps(args.steps)
    sync(det)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    if piped:
        prof = {}
        for x in (pipe.env_det, pipe.det_det):
            x.profile(False)
            for k, (c, tms) in x.profile_read().items():
                c0, t_0 = prof.get(k, (0, 0.0))
                prof[k] = (c0 + c, t_0 + tms)
        ties["raised"] = pipe.ties_resolved
    else:
        det.profile(False)
        prof = det.profile_read()
    gpu_host = last.to_host()          # the timed steps' outputs (checked against the oracle below)
    ties_timed = dict(ties)
    if pipe is not None:
        pipe.close()
        del pipe
    elapsed, total_peaks = reduce_results(t1 - t0, out.n_peaks, world, rank)
    # per-kernel table from a separate, untimed pass with every launch bracketed
    det.profile_only("")
    det.profile(True)
    kprof_steps = max(3, min(args.steps, 10))
    for _ in range(kprof_steps):
        step()
    sync(det)
    det.profile(False)
    kprof = det.profile_read()

    # PCIe-inclusive rate: the same step with the PCM handed over in
    # pinned host memory and copied to HBM inside the timed region.  Reported
    # beside `value`, never as it.
    pcie = None
    if args.pcie_steps > 0:
        host = pcm.cpu().pin_memory()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for _ in range(args.pcie_steps):
            pcm.copy_(host, non_blocking=True)
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t2) / args.pcie_steps
        pcie = {"value": F * n / dt, "unit": "audio-samples/s", "ms_per_step": dt * 1e3,
                "h2d_bytes_per_step": F * n * 2, "steps": args.pcie_steps, "per_gpu": True}
        del host

    # Side measurement (never `value`): the same batch as K sub-batches on K
    # library contexts and K streams, so the latency-bound per-recording
    # kernels of one sub-batch fill the tails of another's.  Outputs are
    # compared with the timed batch's file by file, array by array.
    multi = None
    if args.contexts > 1 and F % args.contexts == 0:
        from bpm_analysis_amd.engine import Detector
        K, per = args.contexts, F // args.contexts
        dets = [det] + [Detector(local) for _ in range(K - 1)]
        streams = [torch.cuda.Stream(det.device) for _ in range(K)]
        fok = np.arange(per + 1, dtype=np.int64) * n
        outs = [dets[k].alloc(fok, d.ds, d.sr) for k in range(K)]
        views = [pcm[k * per * n:(k + 1) * per * n] for k in range(K)]

        def mstep():
            for k in range(K):
                with torch.cuda.stream(streams[k]):
                    dets[k].run(views[k], fok, fs, params, mode=args.mode, out=outs[k], d=d, options=args.options)

        for _ in range(2):
            mstep()
        torch.cuda.synchronize()
        tm0 = time.perf_counter()
        msteps = max(3, min(args.steps, 10))
        for _ in range(msteps):
            mstep()
        torch.cuda.synchronize()
        mdt = (time.perf_counter() - tm0) / msteps
        mhost = [r for o in outs for r in o.to_host()]
        same = all(np.array_equal(a[k], b[k], equal_nan=(k in ("env", "floor")))
                   for a, b in zip(mhost, gpu_host) for k in ("env", "floor", "troughs", "peaks")) and \
            all(a["flags"] == b["flags"] for a, b in zip(mhost, gpu_host))
        multi = {"contexts": K, "value": F * n / mdt, "unit": "audio-samples/s", "ms_per_step": mdt * 1e3,
                 "steps": msteps, "per_gpu": True, "outputs_identical": bool(same),
                 "compared": "env, floor, troughs, peaks, flags of every file vs the timed batch"}
        for x in dets[1:]:
            x.close()
        del outs, views, streams, mhost

    # Side measurement (never `value`): the same step with the two exact but
    # input-dependent shortcuts off (draft-floor bracket, final-floor pruning),
    # i.e. the step a recording that defeats them costs.  Outputs must not change.
    exact = None
    if args.exact_steps > 0:
        ref = [x.clone() for x in (out.floor, out.troughs, out.peaks, out.n_troughs, out.n_peaks, out.flags)]
        opt = args.options | 8 | 16       # BPMX_OPT_DRAFT_FULL | BPMX_OPT_ROLLQ_NOPRUNE
        det.run(pcm, fo, fs, params, mode=args.mode, out=out, d=d, options=opt)
        torch.cuda.synchronize()
        te0 = time.perf_counter()
        for _ in range(args.exact_steps):
            det.run(pcm, fo, fs, params, mode=args.mode, out=out, d=d, options=opt)
        torch.cuda.synchronize()
        edt = (time.perf_counter() - te0) / args.exact_steps
        same = all(torch.equal(a, b) if a.dtype != torch.float64 else
                   torch.equal(a.nan_to_num(-1.0), b.nan_to_num(-1.0))
                   for a, b in zip(ref, (out.floor, out.troughs, out.peaks, out.n_troughs, out.n_peaks, out.flags)))
        exact = {"options": opt, "value": F * n / edt, "unit": "audio-samples/s", "ms_per_step": edt * 1e3,
                 "steps": args.exact_steps, "per_gpu": True, "outputs_identical": bool(same)}
        del ref

    # Side measurement (never `value`): a batch whose troughs the draft-floor
    # bracket does not decide (the synthetic generator leaves none open; real
    # recordings such as the vulpine sample leave ~17 %).  Lowering
    # trough_rejection_multiplier puts many troughs near the threshold; they are
    # then decided from the exact draft value at the trough (draft_point).  The
    # same parameters with the draft computed in full must give identical outputs.
    undecided = None
    if args.undecided_mult > 0 and args.exact_steps > 0:
        from bpm_analysis_amd import _native as N
        pu = dict(params, trough_rejection_multiplier=args.undecided_mult)
        det.run(pcm, fo, fs, pu, mode=args.mode, out=out, d=d, options=args.options | N.OPT_STATS)
        stt = det.stats()
        res = {}
        for name, opt in (("default", args.options), ("draft_full", args.options | N.OPT_DRAFT_FULL),
                          ("draft_full_noprune", args.options | N.OPT_DRAFT_FULL | N.OPT_ROLLQ_NOPRUNE)):
            det.run(pcm, fo, fs, pu, mode=args.mode, out=out, d=d, options=opt)
            torch.cuda.synchronize()
            tu0 = time.perf_counter()
            for _ in range(args.exact_steps):
                det.run(pcm, fo, fs, pu, mode=args.mode, out=out, d=d, options=opt)
            torch.cuda.synchronize()
            res[name] = {"options": opt, "ms_per_step": (time.perf_counter() - tu0) / args.exact_steps * 1e3,
                         "outputs": [x.clone() for x in (out.floor, out.troughs, out.peaks, out.n_troughs,
                                                         out.n_peaks, out.flags)]}
        base = res["default"]["outputs"]
        for name in res:
            o = res[name].pop("outputs")
            res[name]["outputs_identical_to_default"] = bool(all(
                torch.equal(a.nan_to_num(-1.0), b.nan_to_num(-1.0)) if a.dtype == torch.float64 else torch.equal(a, b)
                for a, b in zip(base, o)))
        undecided = {"trough_rejection_multiplier": args.undecided_mult, "raw_troughs": stt["raw_troughs"],
                     "undecided_troughs": stt["undecided"],
                     "undecided_frac": stt["undecided"] / max(1, stt["raw_troughs"]),
                     "full_draft_chunks": stt["full_draft_chunks"], "steps": args.exact_steps, "per_gpu": True,
                     **res}
        del base

    # Side measurement (never `value`): the detection stages on REAL envelopes.
    # The synthetic generator's recordings leave no trough inside the draft
    # bracket and prune well; a real recording does neither as well.  Two
    # envelopes of the reference's own vulpine sample (tests/golden/vulpine.npz,
    # 377 s at 302 Hz): "reference" = its reference-pipeline envelope (rolling
    # mean of |filtfilt|, the 20-150 Hz ripple kept), "native_style" =
    # rolling mean of |hilbert| of its filtered, decimated signal (the sample
    # WAV itself), i.e. what native mode computes, made on the host as input.
    # Each is cut into F windows of the batch's decimated length at spread
    # offsets; FLOOR | PEAKS run on them and, for comparison, on the timed
    # batch's synthetic envelopes.  Recordings with a decisive tie are counted
    # and re-decided in numpy's order (engine.resolve_ties), timed apart; a
    # sample of windows is checked against the numpy-order oracle.
    real = None
    if rank == 0 and args.real_env_steps > 0 and args.mode == "native":
        import pandas as pd
        import scipy.signal as ssig
        from bpm_analysis_amd import _native as N
        from bpm_analysis_amd.design import detect_design
        g = np.load(os.path.join(REPO, "tests", "golden", "vulpine.npz"), allow_pickle=False)
        sr = int(g["sr"])
        if sr == d.sr and len(g["env"]) > nd:
            sources = {
                "reference": np.ascontiguousarray(g["env"], dtype=np.float64),
                "native_style": pd.Series(np.abs(ssig.hilbert(g["pcm"].astype(np.float64)))).rolling(
                    sr // 10, min_periods=1, center=True).mean().to_numpy(),
            }
            fr = np.arange(F + 1, dtype=np.int64) * nd
            dr = detect_design(sr, params)
            st = N.STAGE_FLOOR | N.STAGE_PEAKS
            out_d = det.alloc(fr, 1, sr)

            def det_time(o):
                det.run(None, fr, sr, params, stages=st, out=o, d=dr, options=args.options)
                torch.cuda.synchronize()
                tr0 = time.perf_counter()
                for _ in range(args.real_env_steps):
                    det.run(None, fr, sr, params, stages=st, out=o, d=dr, options=args.options)
                torch.cuda.synchronize()
                return (time.perf_counter() - tr0) / args.real_env_steps * 1e3

            out_d.env.copy_(out.env)
            real = {"recordings": F, "samples_per_recording": nd, "sr": sr, "steps": args.real_env_steps,
                    "stages": "FLOOR | PEAKS (noise floor, troughs, raw peaks)",
                    "windows": "offsets (k * 997) mod (len - Nd), k < recordings",
                    "synthetic_envelopes_ms_per_batch": det_time(out_d)}
            from oracle import oracle as O
            od = O.derive(fs, params)
            for name, env0 in sources.items():
                starts = [(k * 997) % (len(env0) - nd) for k in range(F)]
                out_d.env.copy_(torch.from_numpy(np.concatenate([env0[s0:s0 + nd] for s0 in starts])).to(det.device))
                ms_r = det_time(out_d)
                det.run(None, fr, sr, params, stages=st, out=out_d, d=dr, options=args.options | N.OPT_STATS)
                stt = det.stats()
                fl = out_d.flags.cpu().numpy()
                n_tie = int(np.count_nonzero(fl & (N.F_TROUGH_TIE | N.F_PEAK_TIE)))
                torch.cuda.synchronize()
                tt0 = time.perf_counter()
                n_res = det.resolve_ties(out_d, params, st)
                torch.cuda.synchronize()
                t_res = (time.perf_counter() - tt0) * 1e3
                rhost = out_d.to_host()
                pick = sorted(set(np.linspace(0, F - 1, min(F, 8)).astype(int).tolist()))
                ok = 0
                for k in pick:
                    e = np.ascontiguousarray(env0[starts[k]:starts[k] + nd])
                    of, ot, ofl, _ = O.noise_floor_numpy_order(e, od, params)
                    opk = O.find_peaks_numpy_order(e, height=of, distance=od.distance,
                                                   prominence=O.quantile(e, params["peak_prominence_quantile"]))
                    r = rhost[k]
                    ok += int(np.array_equal(r["troughs"], ot) and np.array_equal(r["peaks"], opk) and
                              np.array_equal(r["floor"], of, equal_nan=True) and (r["flags"] & 7) == (ofl & 7))
                real[name] = {"ms_per_batch": ms_r, "raw_troughs": stt["raw_troughs"],
                              "undecided_troughs": stt["undecided"],
                              "undecided_frac": stt["undecided"] / max(1, stt["raw_troughs"]),
                              "full_draft_chunks": stt["full_draft_chunks"], "tie_flagged_recordings": n_tie,
                              "ties_resolved": n_res, "tie_resolution_ms": t_res,
                              "parity": {"files": len(pick), "equal_to_numpy_order_oracle": ok}}
            del out_d

    # Parity of the timed batch against the oracle on the same recordings.  N = 1:
    # every file, in the cpu_baseline leg below.  N > 1: a bounded sample of
    # every rank's shard, counts summed over ranks; rank 0's sample, timed on
    # its share of the host's cores, is that rank's cpu_baseline.
    parity = cpu = None
    if world > 1 and args.parity_files > 0 and not args.no_cpu:
        lw = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        th_all, aff, ncpu = cpu_threads()
        # OMP_NUM_THREADS, when set, is already this process's share (the launcher
        # passes it to every rank); otherwise split the affinity mask over the ranks
        th = th_all if os.environ.get("OMP_NUM_THREADS", "").isdigit() else max(1, th_all // max(1, lw))
        pick = sorted(set(np.linspace(0, F - 1, min(F, args.parity_files)).astype(int).tolist()))
        seeds = [seed0 + f for f in pick]
        outs, odt = oracle_outputs(args.mode, fs, n, seeds, params, th)
        pr = compare_outputs([gpu_host[f] for f in pick], outs, exact_env=(args.mode == "reference"), fs=fs,
                             params=params)
        cnt = torch.tensor([pr["files"], pr["peaks_equal"], pr["troughs_equal"], pr["flags_equal"],
                            pr["ties_unresolved"], pr["ties_resolved"], ties_timed["raised"]],
                           dtype=torch.float64, device=cdev)
        worst = torch.tensor([pr["env_max_rel"], pr["floor_max_rel"]], dtype=torch.float64, device=cdev)
        dist.all_reduce(cnt)
        dist.all_reduce(worst, op=dist.ReduceOp.MAX)
        c, w = cnt.tolist(), worst.tolist()
        parity = {"files": int(c[0]), "ranks": world, "files_per_rank": len(pick), "peaks_equal": int(c[1]),
                  "troughs_equal": int(c[2]), "flags_equal": int(c[3]), "env_max_rel": w[0], "floor_max_rel": w[1],
                  "env_tol": pr["env_tol"], "ties_unresolved": int(c[4]), "ties_resolved": int(c[5]),
                  "tie_flagged_in_timed_steps": int(c[6]),
                  "ok": c[1] == c[0] and c[2] == c[0] and c[3] == c[0] and max(w) <= pr["env_tol"] and c[4] == 0}
        if rank == 0:
            cpu = {"value": len(pick) * n / odt, "unit": "audio-samples/s", "cores": th, "kind": "port",
                   "per_rank": True, "rank": 0, "affinity_cpus": aff, "os_cpu_count": ncpu,
                   "sample": f"rank 0's parity sample: {len(pick)} of its {F} recordings (seeds {seeds[0]}.."
                             f"{seeds[-1]}, {n / fs:.0f} s {fs} Hz mono int16), {args.mode} mode, "
                             f"oracle/bpmx_oracle.c + numpy FFT on {th} threads of {_cpu_model()} ({lw} ranks "
                             f"on this node, each on its share), while the other ranks ran theirs; "
                             f"{odt:.2f} s wall"}

    # Side measurement (never `value`): the host beat stages (beats.py: classifier,
    # refinement, BPM curve, metrics — SURVEY 8(f) rows 1 and 3) on the first
    # files of this batch's GPU outputs, one core.  Outside the north-star metric.
    # Every rank's files then go to rank 0 in the final result gather (SURVEY
    # 8(e)): raw peaks of every file, and final beats + the smoothed BPM curve of
    # the files whose beat stages ran.
    from bpm_analysis_amd.shard import FileResult, gather_file_results
    rows = [FileResult(seed0 + f, raw_peaks=gpu_host[f]["peaks"], flags=gpu_host[f]["flags"]) for f in range(F)]
    host_beats = None
    if args.host_beat_files > 0:
        from bpm_analysis_amd import beats
        # native stages (libbpmx_host.so) on every file of the batch, over the
        # rank's host threads: their beats and BPM curves go into the gather
        hth = max(1, cpu_threads()[0] // int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
        th0 = time.perf_counter()
        fast = beats.analyze_fast(gpu_host, params, threads=hth)
        ndt = time.perf_counter() - th0
        for f, a in enumerate(fast):
            if "error" not in a:
                rows[f] = FileResult(seed0 + f, gpu_host[f]["peaks"], a["final_peaks"], a["bpm_times"], a["bpm"],
                                     gpu_host[f]["flags"])
        # the Python stages (beats.py: also HRV, slopes, debug strings) on a sample, one core
        res = gpu_host[:args.host_beat_files]
        th1 = time.perf_counter()
        done = beats.analyze_many(res, params)
        hdt = time.perf_counter() - th1
        same = all(np.array_equal(d["final_peaks"], a["final_peaks"]) for d, a in zip(done, fast)
                   if "error" not in d and "error" not in a)
        host_beats = {"native": {"files": F, "threads": hth, "files_per_s": F / ndt, "ms_per_file_per_thread":
                                 ndt / F * hth * 1e3, "wall_ms": ndt * 1e3,
                                 "final_beats": int(sum(len(a["final_peaks"]) for a in fast if "error" not in a))},
                      "python": {"files": len(res), "cores": 1, "files_per_s": len(res) / hdt,
                                 "ms_per_file": hdt / len(res) * 1e3,
                                 "final_beats": int(sum(len(r["final_peaks"]) for r in done if "error" not in r))},
                      "native_equals_python": bool(same)}
    tg0 = time.perf_counter()
    allres = gather_file_results(rows, total_files, device=cdev if world > 1 else None)
    gathered = None
    if rank == 0:
        got = [r for r in allres if r is not None]
        gathered = {"ranks": world, "files": len(got), "peaks": int(sum(len(r["raw_peaks"]) for r in got)),
                    "bpm_curves": int(sum(1 for r in got if len(r["bpm"]))),
                    "bpm_points": int(sum(len(r["bpm"]) for r in got)),
                    "final_beats": int(sum(len(r["final_peaks"]) for r in got)),
                    "ranks_seen": sorted({int(r["rank"]) for r in got}),
                    "ms": round((time.perf_counter() - tg0) * 1e3, 2)}

    # Side measurement (never `value`): one recording at a time through the
    # drop-in, as the reference's analyze_wav_file calls it (rank 0 only).
    dropin = None
    if rank == 0 and args.dropin_files > 0:
        dropin = {m: dropin_latency(local, args.dropin_files, fs, args.secs, params, m)
                  for m in ("reference", "native")}

    if rank == 0:
        ms = elapsed / args.steps * 1e3
        value = total_files * n / (elapsed / args.steps)
        strong = args.files_total > 0
        if strong:
            workload = (f"{total_files} x {args.secs:g} s {fs} Hz mono int16 recordings in the job over {world} "
                        f"GPU(s), {args.mode} mode (filter+envelope+noise floor+raw peaks)")
        else:
            workload = (f"{F} x {args.secs:g} s {fs} Hz mono int16 recordings per GPU, {args.mode} mode "
                        f"(filter+envelope+noise floor+raw peaks)")
        # dominant kernel = the largest share of the step (summed over its launches,
        # from the warmup pass); its roofline point is per step: algorithmic bytes of
        # all its launches in a step / its time per step, the HIP-event total over
        # the TIMED steps / steps
        timed = {k: v for k, v in prof.items() if k in abytes}
        roof = None
        if dom and dom in timed:
            cnt, tot = timed[dom]
            per_step_s = tot / args.steps / 1e3
            ach = abytes[dom] / per_step_s / 1e9
            roof = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 5),
                    "traffic": pmc_traffic(args.mode, dom, workload, cnt / args.steps),
                    "traffic_source": f"profiles/pmc_traffic_{args.mode}.json: rocprofv3 --pmc FETCH_SIZE / "
                                      "WRITE_SIZE passes of this command (tools/pmc_traffic.py), committed; "
                                      "read here, not measured in this run",
                    "kernel": dom, "kernel_ms_per_step": round(per_step_s * 1e3, 4),
                    "launches_per_step": cnt / args.steps, "algorithmic_bytes_per_step": abytes[dom]}
        kernels = {}
        for k, (c, t) in sorted(kprof.items()):
            kernels[k] = {"launches": c, "avg_ms": round(t / c, 4),
                          "share": round(t / kprof_steps / ms, 4)}
            if abytes.get(k):
                kernels[k]["algo_GBps"] = round(abytes[k] / (t / kprof_steps / 1e3) / 1e9, 1)
                tr = pmc_traffic(args.mode, k, workload, c / kprof_steps)
                if tr:
                    kernels[k]["pmc_bytes_per_step"] = tr
        # whole-step view of the north-star roofline: PCM bytes (read once) / step time
        step_bytes = F * n * 2
        pipeline = {"hbm_bytes_per_step": step_bytes, "per_gpu": True,
                    "achieved_GBps": round(step_bytes / (ms / 1e3) / 1e9, 1),
                    "frac_of_peak": round(step_bytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 5)}
        if world == 1 and not args.no_cpu and args.cpu_files != 0:
            nfc = args.cpu_files if args.cpu_files > 0 else F
            cpu, parity = cpu_baseline(args.mode, fs, n, seed0, nfc, params, gpu_host)
            # recordings the timed steps' tie check re-decided (summed over the
            # steps; 0 on the synthetic batch: no decisive tie), and those left open
            parity["tie_flagged_in_timed_steps"] = ties_timed["raised"]
            parity["tie_check"] = ("every timed step: flags read back, tied recordings re-decided in numpy's "
                                   "argsort order (engine.resolve_ties)")
        line = {
            "metric": METRIC, "value": value, "unit": "audio-samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None, "dtype": "f64",
            "data": "cpu-stub (tests only; not a measurement)" if args.cpu_stub else "synthetic",
            "config": {"workload": workload, "files_total": total_files,
                       "files_per_gpu": F, "frames_per_file": n, "decimated_per_file": nd, "mode": args.mode,
                       "parallelism": f"file-sharded x{world}",
                       "batch_pipeline": bool(piped)},
            "roofline": roof, "cpu_baseline": cpu, "parity": parity,
            "gpu_vs_cpu": (value / cpu["value"]) if cpu else None,
            "pipeline": pipeline, "pcie_inclusive": pcie, "kernels": kernels, "total_raw_peaks": total_peaks,
            "result_gather": gathered, "multi_context": multi, "exact_no_shortcuts": exact,
            "host_beat_stages": host_beats, "dropin_latency": dropin, "draft_undecided": undecided,
            "real_envelope_detection": real,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    _args = parse()
    if _args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if not _args.cpu_stub:
            import torch
            if torch.cuda.device_count() < _args.gpus:      # counts devices without initialising them
                raise SystemExit(f"bench.py: --gpus {_args.gpus} but {torch.cuda.device_count()} GPU(s) visible")
        sys.exit(launch_ranks(sys.argv[1:], _args.gpus))
    if _args.workload == "c5":
        run_c5(_args)
    else:
        main(_args)
