"""Per-kernel time of the ENVELOPE stage alone on the C5 shard (tools only):
64 x U[10, 30] min 96 kHz stereo int16 (bench.c5_lengths).  Used with
BPMX_LIB=build_var/libbpmx_<variant>.so to time phase-skipping builds of the
block kernel (their outputs are meaningless, so only the envelope stage runs).

    python tools/c5_env_prof.py [steps]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    import torch
    import bench
    from bpm_analysis_amd import DEFAULT_PARAMS, _native as N
    from bpm_analysis_amd.design import design
    from bpm_analysis_amd.engine import Detector
    det = Detector(0)
    fs, ch = 96000, 2
    params = dict(DEFAULT_PARAMS, save_filtered_wav=False)
    lengths = bench.c5_lengths(64, fs)
    lengths = np.sort(lengths)[::-1]
    fo = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    d = design(fs, params, log=False)
    pcm = det.synth(fo, fs, ch, seeds=[100_000 + i for i in range(len(lengths))])
    out = det.alloc(fo, d.ds, d.sr)
    det.run(pcm, fo, fs, params, mode="native", channels=ch, out=out, d=d, stages=N.STAGE_ENVELOPE)
    torch.cuda.synchronize()
    det.profile(True)
    for _ in range(steps):
        det.run(pcm, fo, fs, params, mode="native", channels=ch, out=out, d=d, stages=N.STAGE_ENVELOPE)
    torch.cuda.synchronize()
    det.profile(False)
    prof = det.profile_read()
    gb = int(fo[-1]) * ch * 2 / 1e9
    rows = {k: round(t / steps, 4) for k, (c, t) in sorted(prof.items(), key=lambda kv: -kv[1][1])}
    blk = rows.get("k_native_blocks")
    print(json.dumps({"lib": os.environ.get("BPMX_LIB", "default"), "pcm_GB": round(gb, 3),
                      "k_native_blocks_ms": blk, "TBps": round(gb / blk, 3) if blk else None, "kernels": rows}))


if __name__ == "__main__":
    main()
