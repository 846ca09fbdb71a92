"""Multi-rank path of bench.py on CPU (gloo, world size 2): disjoint file
shards, max-over-ranks timing and the rank-0 gather of per-file results."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    counts = torch.arange(4, dtype=torch.int32) + 10 * rank      # per-file peak counts of this shard
    elapsed, total = bench.reduce_results(1.0 + rank, counts, world, rank)
    # result gather: file f of rank r holds peaks 100*r + f*1000 + [0, counts[f])
    from bpm_analysis_amd.shard import FileResult, gather_file_results
    rows = [FileResult(4 * rank + f, raw_peaks=100 * rank + 1000 * f + torch.arange(int(counts[f])).numpy())
            for f in range(4)]
    got = gather_file_results(rows, 4 * world)
    summary = None
    if rank == 0:
        summary = [[got[4 * r + f]["raw_peaks"].tolist() for f in range(4)] for r in range(world)]
    q.put((rank, elapsed, total, bench.shard_seed0(rank, 4), summary))
    dist.destroy_process_group()


def test_two_rank_gather_and_max_time():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, e0, t0, s0, g0), (r1, e1, t1, s1, g1) = res
    assert g1 is None and len(g0) == 2
    for r in range(2):
        for f in range(4):
            n = f + 10 * r
            assert g0[r][f] == [100 * r + 1000 * f + k for k in range(n)]
    assert e0 == e1 == 2.0                        # max over ranks
    assert t0 == (0 + 1 + 2 + 3) + (10 + 11 + 12 + 13) and t1 == 0
    assert (s0, s1) == (0, 4)                     # disjoint synthetic shards


def test_single_rank_passthrough():
    import bench
    e, t = bench.reduce_results(3.5, torch.tensor([1, 2, 3]), 1, 0)
    assert e == 3.5 and t == 6


def test_algorithmic_bytes_native_reads_pcm_once():
    import bench
    ab = bench.algorithmic_bytes("native", 1024, 2646000, 18124, 146)
    assert ab["k_native_blocks"] == 1024 * 2646000 * 2
    assert set(ab) >= {"k_floor_wm", "k_rollq_wm", "k_native_carry", "k_hilbert_env", "k_find_peaks[peaks]"}


def _lpt_worker(rank, world, port, q):
    """Every rank derives the same LPT placement from the lengths alone."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import numpy as np
    from bpm_analysis_amd.shard import lpt_partition
    rng = np.random.default_rng(5)
    lengths = (rng.integers(10, 31, size=37) * 60 * 96000).tolist()     # C5-like: 10-30 min at 96 kHz
    mine = lpt_partition(lengths, world)[rank]
    got = [None] * world
    dist.all_gather_object(got, mine)
    q.put((rank, got, lengths))
    dist.destroy_process_group()


def test_two_rank_lpt_placement():
    import numpy as np
    from bpm_analysis_amd.shard import longest_first, lpt_partition, makespan
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_lpt_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, parts, lengths = outs[0]
    assert all(o[1] == parts for o in outs)                     # ranks agree without exchanging a plan
    flat = sorted(i for part in parts for i in part)
    assert flat == list(range(len(lengths)))                    # each recording exactly once
    n = np.asarray(lengths)
    assert makespan(lengths, parts) <= n.sum() / world + n.max()   # greedy LPT bound
    for part in parts:                                          # each rank's list is longest first
        assert list(n[part]) == sorted(n[part], reverse=True)
    assert list(longest_first([3, 5, 5, 1])) == [1, 2, 0, 3]     # stable among equal lengths
    assert lpt_partition([7, 7, 7, 7], 2) == [[0, 2], [1, 3]]


class _OracleDetector:
    """Test double for engine.Detector on CPU ranks: the oracle computes the hot
    path so the gloo test exercises placement, the host beat stages and the
    gather (the GPU detector is covered by the -m gpu tests)."""
    device = torch.device("cpu")

    def run_host(self, recs, fs, params, mode="native", stages=7, resolve_ties=False):
        from oracle import oracle as O
        ds = O.derive(fs, params).ds
        out = []
        for r in recs:
            if -(-len(r) // ds) <= 15:                  # the library's BPMX_F_TOO_SHORT, in both modes
                out.append({"flags": 8})
                continue
            o = O.detect(r, fs, params, mode=mode)
            out.append({k: o[k] for k in ("env", "floor", "troughs", "peaks", "sr", "flags")})
        return out


def _sharded_items():
    from oracle import oracle as O
    lens = [44100 * s for s in (25, 12, 31, 18, 9, 22)] + [146 * 15]          # ragged; the last is too short
    return [O.synth(40 + i, n, 44100, 1) for i, n in enumerate(lens)]


def _sharded_worker(rank, world, port, q, beats):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bpm_analysis_amd import DEFAULT_PARAMS
    from bpm_analysis_amd.shard import lpt_partition, run_sharded
    items = _sharded_items()
    params = dict(DEFAULT_PARAMS, save_filtered_wav=False)
    res = run_sharded(items, params, fs=44100, mode="native", detector=_OracleDetector(), beats=beats,
                      host_threads=2, chunk_frames=44100 * 30)     # several GPU chunks per rank
    q.put((rank, res, lpt_partition([len(x) for x in items], world)))
    dist.destroy_process_group()


@pytest.mark.parametrize("stages", ["native", "python"])
def test_two_rank_sharded_runner_gathers_peaks_and_bpm_curves(stages):
    """shard.run_sharded over 2 gloo ranks: LPT placement, per-rank detection in
    chunks with the host beat stages (native C++ or Python) on host threads,
    and the rank-0 gather of raw peaks, final beats and the smoothed BPM
    curve, equal to the single-process result file by file."""
    import numpy as np
    from bpm_analysis_amd import DEFAULT_PARAMS, beats
    from oracle import oracle as O
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_sharded_worker, args=(r, world, port, q, stages)) for r in range(world)]
    for p in ps:
        p.start()
    outs = sorted((q.get(timeout=300) for _ in range(world)), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, res, parts), (_, res1, _) = outs
    assert res1 is None and len(res) == 7
    params = dict(DEFAULT_PARAMS, save_filtered_wav=False)
    for i, pcm in enumerate(_sharded_items()):
        r = res[i]
        assert r["rank"] == (0 if i in parts[0] else 1)
        if i == 6:
            assert isinstance(r["error"], ValueError) and "padlen" in str(r["error"])
            continue
        o = O.detect(pcm, 44100, params, mode="native")
        a = beats.analyze_recording(o["env"], o["sr"], o["floor"], o["troughs"], o["peaks"], params)
        m = a["final_metrics"]
        assert np.array_equal(r["raw_peaks"], o["peaks"])
        assert np.array_equal(r["final_peaks"], a["final_peaks"])
        assert np.array_equal(r["bpm_times"], np.asarray(m["bpm_times"]))
        assert np.array_equal(r["bpm"], m["smoothed_bpm"].values)
        assert r["flags"] == o["flags"] and len(r["bpm"]) > 5


def _bench_json(stdout: str) -> dict:
    import json
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("workload", ["metric", "strong", "c5"])
def test_bench_launches_n_ranks(workload):
    """`python bench.py --gpus 2` starts two ranks itself (torch.distributed.run
    child, gloo under --cpu-stub), reports n_gpus 2 and gathers both ranks'
    files to rank 0; parity and the CPU baseline are kept at N > 1."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--cpu-stub", "--steps", "1", "--warmup", "1"]
    if workload == "metric":
        cmd += ["--files", "3", "--secs", "6", "--parity-files", "2", "--host-beat-files", "1"]
    elif workload == "strong":   # BASELINE C4's shape (--files-total over the ranks), 5 recordings in the job
        cmd += ["--files-total", "5", "--secs", "6", "--parity-files", "3", "--host-beat-files", "1"]
    else:   # 5 recordings of 10-30 min at 96 kHz stereo are too much oracle work: shrink via the chunk budget only
        cmd += ["--workload", "c5", "--c5-files", "2", "--c5-chunk-gb", "0.001"]     # parity: every recording
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=repo)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _bench_json(r.stdout)
    assert line["n_gpus"] == 2 and line["data"].startswith("cpu-stub")
    assert line["parity"]["ok"] and line["parity"]["ranks"] == 2
    if workload == "metric":
        assert line["result_gather"]["files"] == 6 and line["result_gather"]["ranks_seen"] == [0, 1]
        assert line["cpu_baseline"]["per_rank"] and line["cpu_baseline"]["rank"] == 0
        assert line["parity"]["files"] == 4
    elif workload == "strong":
        # ranks hold recordings 0-1 and 2-4; every one checked and gathered once
        assert line["scaling"] == "strong" and line["config"]["files_total"] == 5
        assert line["config"]["files_per_gpu"] == 2
        assert line["result_gather"]["files"] == 5 and line["result_gather"]["ranks_seen"] == [0, 1]
        assert line["parity"]["files"] == 5
        assert abs(line["value"] - 5 * 6 * 44100 / (line["ms_per_step"] / 1e3)) <= 1e-6 * line["value"]
    else:
        assert line["result_gather"]["files"] == 2 and line["scaling"] == "strong"
        assert line["parity"]["files"] == 2


def test_bench_refuses_world_mismatch():
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--cpu-stub"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=repo)
    assert r.returncode != 0 and "refusing" in r.stderr
