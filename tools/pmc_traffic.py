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
    # torch's own kernels live in anonymous namespaces ("at::native::(anonymous
    # namespace)::..."): drop that before cutting at the argument list (r03's
    # summary showed the output tensors' zero fill under an empty name)
    kernel = kernel.replace("(anonymous namespace)::", "")
    k = kernel.split("(")[0]
    full = "k_rollq_wm_t<false>" in k                 # the unpruned rolling-quantile variant
    k = re.sub(r"<.*", "", k).replace("void ", "").strip() + ("[full]" if full else "")
    k = k.split("::")[-1]
    if "fft" in kernel.lower() or "bluestein" in kernel.lower():
        return "rocfft:" + k
    return k


# kernels launched more than once per step under different launch labels
# (bpmx_api.hip's LAUNCH names), in launch order within a step: their
# dispatches are labelled by their position in that cycle
LABEL_CYCLE = {"k_find_peaks_lds": ["k_find_peaks[troughs]", "k_find_peaks[peaks]"],
               "k_rollq_wm_t": ["k_rollq_wm[draft]"]}      # r05: the floor's other passes are k_floor_wm


def per_kernel(d: str, counter: str) -> dict:
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = collections.defaultdict(list)
    for fn in files:
        for r in csv.DictReader(open(fn)):
            if r["Counter_Name"] != counter:
                continue
            acc[(int(r["Dispatch_Id"]), short_name(r["Kernel_Name"]))].append(float(r["Counter_Value"]))
    by = collections.defaultdict(list)
    seen = collections.Counter()
    for (_, k), v in sorted(acc.items()):
        by[k].append(sum(v))            # sum over XCD / instance rows of one dispatch
        cyc = LABEL_CYCLE.get(k)
        if cyc:                         # also per launch label, by position in the step's cycle
            by[cyc[seen[k] % len(cyc)]].append(sum(v))
            seen[k] += 1
    return {k: sum(v) / len(v) for k, v in by.items()}


# the load width per lane of each kernel's dominant HBM stream (tools/pmc_calib.hip
# measures FETCH_SIZE against known bytes per width; 16: LDS-DMA / dwordx4)
READ_WIDTH = {"k_native_blocks_mfma": 16, "k_native_blocks_dma": 16, "k_native_blocks_i16": 16,
              "k_find_peaks_lds": 8, "k_find_peaks": 8, "k_hilbert_env": 8, "k_native_yd": 8,
              "k_quantile_reg": 8, "k_rollq_wm_t": 8, "k_floor_wm": 8, "k_draft_bounds": 8, "k_native_carry": 8}


def calibration(fetch_dir: str, write_dir: str, nbytes: int = 768 << 20) -> dict:
    """Counter bytes per true byte for each calib_read<T> / calib_write<T> of
    tools/pmc_calib.hip (FETCH_SIZE and WRITE_SIZE in KB)."""
    def by_width(d, counter, prefix):
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        acc = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for fn in files:
            for r in csv.DictReader(open(fn)):
                name = r["Kernel_Name"]
                if r["Counter_Name"] != counter or prefix not in name:
                    continue
                targ = name.split(prefix, 1)[1].split(">", 1)[0]      # the template argument
                w = 4 if "unsigned int" in targ else (8 if "double" in targ else 16)
                acc[w] += float(r["Counter_Value"])
                disp[w].add(r["Dispatch_Id"])
        return {w: acc[w] * 1024 / len(disp[w]) / nbytes for w in acc}
    return {"read": by_width(fetch_dir, "FETCH_SIZE", "calib_read"),
            "write": by_width(write_dir, "WRITE_SIZE", "calib_write")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--mode", default="native")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--out", default=None)
    ap.add_argument("--calib", default=None,
                    help="JSON with {'read': {width: counter bytes per byte}} from --make-calib")
    ap.add_argument("--make-calib", action="store_true",
                    help="--fetch / --write are tools/pmc_calib runs: write the calibration JSON to --out")
    a = ap.parse_args()
    if a.make_calib:
        cal = calibration(a.fetch, a.write)
        json.dump({"method": "tools/pmc_calib.hip: 768 MiB streamed once per kernel, counter KB * 1024 / bytes",
                   **cal}, open(a.out, "w"), indent=1)
        print(json.dumps(cal))
        return
    cal = json.load(open(a.calib))["read"] if a.calib else None
    fetch = per_kernel(a.fetch, "FETCH_SIZE")
    write = per_kernel(a.write, "WRITE_SIZE")
    ks = {}
    for k in sorted(set(fetch) | set(write)):
        if cal:
            wdt = str(READ_WIDTH.get(k.replace("[full]", ""), 16))
            f = fetch.get(k, 0.0) * 1024 / float(cal[wdt])
        else:
            f = fetch.get(k, 0.0) * 1024 * 2
        w = write.get(k, 0.0) * 1024
        ks[k] = {"fetch_bytes": round(f), "write_bytes": round(w), "hbm_bytes_per_launch": round(f + w)}
    method = ("rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes; FETCH_SIZE(KB)*1024 / the "
              "counter-per-byte factor measured by tools/pmc_calib.hip for the kernel's load width "
              "(profiles/pmc_calib.json) + WRITE_SIZE(KB)*1024; mean over dispatches") if cal else (
              "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes; FETCH_SIZE(KB)*1024*2 "
              "(gfx950 streaming-read calibration) + WRITE_SIZE(KB)*1024; mean over dispatches")
    out = {"workload": a.workload, "mode": a.mode, "method": method, "kernels": ks}
    path = a.out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                                 f"pmc_traffic_{a.mode}.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in ks.items():
        print(f"{k:40s} {v['hbm_bytes_per_launch'] / 1e6:12.1f} MB")


if __name__ == "__main__":
    main()
