"""C5 shard step (64 x U[10, 30] min 96 kHz stereo, bench.c5_lengths) with its
recordings run concurrently (tools only):

  * pipeline shapes (bpmx_set_pipeline: chunk k's detection overlaps chunk
    k+1's envelope), and
  * K sub-batches on K contexts and streams (LPT by length),

each timed over `steps` steps and compared array by array with the plain
one-stream run.

    python tools/c5_concurrency.py [steps] [files]
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    files = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    import torch
    import bench
    from bpm_analysis_amd import DEFAULT_PARAMS
    from bpm_analysis_amd.design import design
    from bpm_analysis_amd.engine import Detector
    det = Detector(0)
    fs, ch = 96000, 2
    params = dict(DEFAULT_PARAMS, save_filtered_wav=False)
    lengths = np.sort(bench.c5_lengths(files, fs))[::-1]
    fo = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    d = design(fs, params, log=False)
    pcm = det.synth(fo, fs, ch, seeds=[100_000 + i for i in range(len(lengths))])
    keys = ("env", "floor", "troughs", "peaks")

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    def same(a_list, b_list):
        return all(np.array_equal(a[k], b[k], equal_nan=k in ("env", "floor")) for a, b in zip(a_list, b_list)
                   for k in keys) and all(a["flags"] == b["flags"] for a, b in zip(a_list, b_list))

    out = det.alloc(fo, d.ds, d.sr)
    base_ms = timed(lambda: det.run(pcm, fo, fs, params, mode="native", channels=ch, out=out, d=d))
    ref = out.to_host()
    rows = [{"shape": "plain", "ms_per_step": round(base_ms, 3)}]
    print(json.dumps(rows[-1]), flush=True)
    for shape in ((2, 0, 0), (4, 0, 0), (8, 0, 0)):
        det.set_pipeline(*shape)
        ms = timed(lambda: det.run(pcm, fo, fs, params, mode="native", channels=ch, out=out, d=d))
        rows.append({"shape": "pipeline", "chunks": shape[0], "ms_per_step": round(ms, 3),
                     "identical": bool(same(out.to_host(), ref))})
        print(json.dumps(rows[-1]), flush=True)
    det.set_pipeline(0, 0, 0)
    frame_bytes = 2 * ch
    for K in (2, 4):
        # LPT over K groups of whole recordings (contiguous in the batch: groups
        # are the interleaved sorted lengths, so take views per recording set)
        groups = [[] for _ in range(K)]
        load = [0] * K
        for i in range(len(lengths)):
            k = int(np.argmin(load))
            groups[k].append(i)
            load[k] += int(lengths[i])
        # contiguous sub-batches: copy each group's recordings together once
        dets = [det] + [Detector(0) for _ in range(K - 1)]
        streams = [torch.cuda.Stream(det.device) for _ in range(K)]
        subs = []
        for k, g in enumerate(groups):
            g = sorted(g)
            parts = [pcm[int(fo[i]) * ch:int(fo[i + 1]) * ch] for i in g]
            sp = torch.cat(parts)
            sfo = np.concatenate([[0], np.cumsum(lengths[g])]).astype(np.int64)
            subs.append((g, sp, sfo, dets[k].alloc(sfo, d.ds, d.sr)))

        def mstep():
            for k, (g, sp, sfo, so) in enumerate(subs):
                with torch.cuda.stream(streams[k]):
                    dets[k].run(sp, sfo, fs, params, mode="native", channels=ch, out=so, d=d)

        ms = timed(mstep)
        got = [None] * len(lengths)
        for g, sp, sfo, so in subs:
            for i, h in zip(g, so.to_host()):
                got[i] = h
        rows.append({"shape": "contexts", "K": K, "ms_per_step": round(ms, 3), "identical": bool(same(got, ref))})
        print(json.dumps(rows[-1]), flush=True)
        for x in dets[1:]:
            x.close()
        del subs, streams
        torch.cuda.empty_cache()
    print(json.dumps({"summary": rows, "pcm_GB": round(int(fo[-1]) * frame_bytes / 1e9, 3)}))


if __name__ == "__main__":
    main()
