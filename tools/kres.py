"""Per-kernel register, spill, scratch and LDS figures of the library's HIP
sources, from the compiler's kernel-resource-usage remarks (gfx950).

    python tools/kres.py [file.hip ...] [-D...]

Defaults to every source in bpm_analysis_amd/csrc.  Prints one row per kernel:
VGPRs, AGPRs, SGPRs, SGPR spills, VGPR spills, scratch bytes per lane,
occupancy (waves per SIMD), static LDS."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "bpm_analysis_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-fno-fast-math", "--offload-device-only", "-c", "-o", "/dev/null",
         "-Rpass-analysis=kernel-resource-usage"]
KEYS = [("VGPRs", "vgpr"), ("AGPRs", "agpr"), ("TotalSGPRs", "sgpr"),
        ("SGPRs Spill", "sspill"), ("VGPRs Spill", "vspill"),
        ("ScratchSize [bytes/lane]", "scratch"), ("Occupancy [waves/SIMD]", "occ"),
        ("LDS Size [bytes/block]", "lds")]


def demangle(names):
    try:
        out = subprocess.run(["/opt/rocm/llvm/bin/llvm-cxxfilt"], input="\n".join(names),
                             capture_output=True, text=True, check=True).stdout.split("\n")
        return [o.split("(")[0] for o in out[:len(names)]]
    except Exception:
        return names


def resources(src, extra=()):
    p = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, src], cwd=CSRC,
                       capture_output=True, text=True)
    rows, cur = [], None
    for line in p.stderr.splitlines():
        m = re.search(r"remark: (.*) \[-Rpass-analysis", line)
        if not m:
            continue
        body = m.group(1).strip()
        if body.startswith("Function Name:"):
            cur = {"name": body.split(":", 1)[1].strip()}
            rows.append(cur)
            continue
        if cur is None or ":" not in body:
            continue
        k, v = body.rsplit(":", 1)
        for key, short in KEYS:
            if k.strip() == key:
                cur[short] = v.strip()
    if p.returncode != 0:
        sys.stderr.write(p.stderr[-2000:])
    return rows


def main():
    args = sys.argv[1:]
    extra = [a for a in args if a.startswith("-")]
    files = [a for a in args if not a.startswith("-")] or sorted(
        f for f in os.listdir(CSRC) if f.endswith(".hip"))
    for f in files:
        rows = resources(os.path.abspath(f) if os.path.exists(f) else f, extra)
        names = demangle([r["name"] for r in rows])
        print(f"== {os.path.basename(f)}")
        for r, n in zip(rows, names):
            print(f"  {n[:60]:60s} v{r.get('vgpr','?'):>4} a{r.get('agpr','?'):>4} "
                  f"s{r.get('sgpr','?'):>4} sspill {r.get('sspill','?'):>4} vspill {r.get('vspill','?'):>3} "
                  f"scratch {r.get('scratch','?'):>4} occ {r.get('occ','?'):>2} lds {r.get('lds','?')}")


if __name__ == "__main__":
    main()
