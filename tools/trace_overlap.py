"""Timeline of a rocprofv3 kernel trace of tools/pipe_sweep.py (tools only).

    python tools/trace_overlap.py gpurun_out/trace_cumask/run_kernel_trace.csv [--step K] [--shape S]

Splits the trace into the sweep's shapes (each: 2 warmup + `steps` timed
runs) at the gaps between runs, and for one run prints every dispatch (queue,
stream, start, duration) plus, per shape, how long envelope kernels and
detection kernels ran at the same time."""
import argparse
import csv
import re

ENV = ("k_native_blocks", "k_native_carry", "k_native_yd", "k_hilbert_env", "k_ref_", "k_envelope_ref")


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    k = re.sub(r"<.*", "", name.split("(")[0]).replace("void ", "").strip()
    return k.split("::")[-1]


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append(dict(name=short(r["Kernel_Name"]), q=int(r["Queue_Id"]), s=int(r["Stream_Id"]),
                         t0=int(r["Start_Timestamp"]), t1=int(r["End_Timestamp"]), grid=int(r["Grid_Size_X"]),
                         wg=int(r["Workgroup_Size_X"]), lds=int(r["LDS_Block_Size"]), vgpr=int(r["VGPR_Count"])))
    return sorted(rows, key=lambda r: r["t0"])


def runs(rows):
    """runs = maximal groups of the pipeline's kernels, split at k_init_out of a
    new run on the main queue following a gap (the host waits between runs)"""
    rows = [r for r in rows if not r["name"].startswith(("k_synth", "__amd", "elementwise", "vectorized",
                                                          "unrolled", "fill"))]
    out, cur, last_end = [], [], None
    for r in rows:
        if cur and last_end is not None and r["t0"] - last_end > 20_000 and r["name"] == "k_init_out":
            out.append(cur)
            cur = []
        cur.append(r)
        last_end = max(last_end or 0, r["t1"])
    if cur:
        out.append(cur)
    return out


def overlap(run):
    env = sorted((r["t0"], r["t1"]) for r in run if r["name"].startswith(ENV))
    det = sorted((r["t0"], r["t1"]) for r in run if not r["name"].startswith(ENV))

    def union(iv):
        out = []
        for a, b in iv:
            if out and a <= out[-1][1]:
                out[-1][1] = max(out[-1][1], b)
            else:
                out.append([a, b])
        return out
    ue, ud = union(env), union(det)
    both = 0
    for a, b in ue:
        for c, d in ud:
            both += max(0, min(b, d) - max(a, c))
    return sum(b - a for a, b in ue), sum(b - a for a, b in ud), both


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--show", type=int, default=-1, help="print the dispatches of this run index")
    a = ap.parse_args()
    rs = runs(load(a.csv))
    for i, run in enumerate(rs):
        t0 = run[0]["t0"]
        span = max(r["t1"] for r in run) - t0
        e, d, b = overlap(run)
        qs = sorted({(r["q"], r["s"]) for r in run})
        print(f"run {i:2d}: {len(run):3d} dispatches, span {span / 1e6:.3f} ms, envelope busy {e / 1e6:.3f} ms, "
              f"detection busy {d / 1e6:.3f} ms, both at once {b / 1e6:.3f} ms, (queue, stream) {qs}")
        if i == a.show:
            for r in run:
                print(f"    q{r['q']} s{r['s']} {r['name']:28s} start {(r['t0'] - t0) / 1e3:9.1f} us  "
                      f"dur {(r['t1'] - r['t0']) / 1e3:8.1f} us  grid {r['grid']:8d} wg {r['wg']:5d} lds {r['lds']}")


if __name__ == "__main__":
    main()
