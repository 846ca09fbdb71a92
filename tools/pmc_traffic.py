"""Turn two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of `bench.py` into
per-launch HBM bytes per kernel: profiles/pmc_traffic_<mode>.json.

    python tools/pmc_traffic.py --fetch gpurun_out/prof_fetch --write gpurun_out/prof_write \
        --mode native --workload "<config.workload of the bench line>"

Units and corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and
WRITE_SIZE are kilobytes; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced streaming read, so it is doubled.  Both derive from the L2's
memory-side request counters, so Infinity-Cache hits are included.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re


def short_name(kernel: str) -> str:
    k = kernel.split("(")[0]
    full = "k_rollq_wm_t<false>" in k                 # the unpruned rolling-quantile variant
    k = re.sub(r"<.*", "", k).replace("void ", "").strip() + ("[full]" if full else "")
    k = k.split("::")[-1]
    if "fft" in kernel.lower() or "bluestein" in kernel.lower():
        return "rocfft:" + k
    return k


def per_kernel(d: str, counter: str) -> dict:
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = collections.defaultdict(list)
    for fn in files:
        for r in csv.DictReader(open(fn)):
            if r["Counter_Name"] != counter:
                continue
            acc[(r["Dispatch_Id"], short_name(r["Kernel_Name"]))].append(float(r["Counter_Value"]))
    by = collections.defaultdict(list)
    for (_, k), v in acc.items():
        by[k].append(sum(v))            # sum over XCD / instance rows of one dispatch
    return {k: sum(v) / len(v) for k, v in by.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--mode", default="native")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    fetch = per_kernel(a.fetch, "FETCH_SIZE")
    write = per_kernel(a.write, "WRITE_SIZE")
    ks = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, 0.0) * 1024 * 2
        w = write.get(k, 0.0) * 1024
        ks[k] = {"fetch_bytes": round(f), "write_bytes": round(w), "hbm_bytes_per_launch": round(f + w)}
    out = {"workload": a.workload, "mode": a.mode,
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes; FETCH_SIZE(KB)*1024*2 "
                     "(gfx950 streaming-read calibration) + WRITE_SIZE(KB)*1024; mean over dispatches",
           "kernels": ks}
    path = a.out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                                 f"pmc_traffic_{a.mode}.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in ks.items():
        print(f"{k:40s} {v['hbm_bytes_per_launch'] / 1e6:12.1f} MB")


if __name__ == "__main__":
    main()
