"""Source lines of a kernel's SGPR spill/reload instructions (v_writelane /
v_readlane with a constant lane, as the register allocator emits them).

    python tools/spill_lines.py <file.hip> <kernel-symbol-prefix> [-D...]"""
import collections
import os
import re
import subprocess
import sys

src, sym = sys.argv[1], sys.argv[2]
extra = sys.argv[3:]
csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bpm_analysis_amd", "csrc")
path = src if os.path.exists(src) else os.path.join(csrc, src)
out = "/tmp/_spill.s"
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                "-ffp-contract=off", "-fno-fast-math", "--offload-device-only", "-gline-tables-only",
                "-S", "-o", out, *extra, path], check=True, stderr=subprocess.DEVNULL)
lines = open(out).read().split("\n")
files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]+)"', l)
    if m:
        files[m.group(1)] = m.group(3).split("/")[-1]
start = next(i for i, l in enumerate(lines) if l.startswith(sym) and ":" in l)
cur = None
rd, wr = collections.Counter(), collections.Counter()
for l in lines[start:]:
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
    if re.search(r"v_readlane_b32 s\d+, v\d+, \d+\s*$", l):
        rd[cur] += 1
    if re.search(r"v_writelane_b32 v\d+, s\d+, \d+\s*$", l):
        wr[cur] += 1
    if ".end_amdhsa_kernel" in l:
        break
print(f"reloads {sum(rd.values())}, spills {sum(wr.values())}")
for k in sorted(set(rd) | set(wr), key=lambda k: (str(k[0]), k[1]) if k else ("", 0)):
    print(f"  {k[0]}:{k[1]}  reload {rd[k]}  spill {wr[k]}")
