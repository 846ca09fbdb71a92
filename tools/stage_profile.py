"""Per-stage GPU time from a rocprofv3 run of the library (roctx "bpmx:<stage>"
ranges, bpmx_api.hip StageRange):

    rocprofv3 --kernel-trace --marker-trace --hip-runtime-trace --output-format csv -d DIR -o run -- python3 bench.py ...
    python tools/stage_profile.py DIR [--steps K]

A kernel belongs to the innermost bpmx range whose host interval contains the
hipLaunchKernel / hipExtLaunchKernel call that enqueued it (joined on the
correlation id); its device time counts for that stage.  Prints the stages'
total device time per run (over the last K runs when given) and their kernels."""
import csv
import glob
import os
import sys
from collections import defaultdict


def rows(d, pat):
    out = []
    for p in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(p) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main():
    d = sys.argv[1]
    markers = [r for r in rows(d, "*marker_api_trace.csv") if r["Function"].startswith("bpmx:")]
    hip = {r["Correlation_Id"]: int(r["Start_Timestamp"]) for r in rows(d, "*hip_api_trace.csv")
           if "Launch" in r["Function"]}
    kern = rows(d, "*kernel_trace.csv")
    ranges = sorted(((int(m["Start_Timestamp"]), int(m["End_Timestamp"]), m["Function"]) for m in markers))
    per = defaultdict(float)
    names = defaultdict(lambda: defaultdict(float))
    runs = sum(1 for r in ranges if r[2] == "bpmx:floor") or 1
    for k in kern:
        t = hip.get(k["Correlation_Id"])
        if t is None:
            continue
        best = None
        for a, b, n in ranges:
            if a <= t < b and (best is None or a >= best[0]):
                best = (a, b, n)
        if best is None:
            continue
        dur = (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e6
        per[best[2]] += dur
        names[best[2]][k["Kernel_Name"].split("(")[0][:60]] += dur
    print(f"runs with a floor stage: {runs}")
    for st in sorted(per, key=lambda s: -per[s]):
        print(f"{st:24s} {per[st] / runs:8.3f} ms per run")
        for n, v in sorted(names[st].items(), key=lambda kv: -kv[1])[:8]:
            print(f"    {n:60s} {v / runs:8.3f}")


if __name__ == "__main__":
    main()
