#!/bin/bash
# r05 probes on one box: final floor and find_peaks phase timings on the bench's
# synthetic envelopes and on windows of the reference's own sample, then the GPU tests.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/probe
P=gpurun_out/probe
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$P/$name.txt" 2>&1; local rc=$?; grep -v "^   \|mismatch" "$P/$name.txt" | tail -n 12; [ $rc -eq 0 ] || { echo "STOP rc=$rc after $name"; exit $rc; }; }
run dfi_v 300 python tools/dump_floor_inputs.py 1024 vulpine /tmp/fv.bin
run rq_v 60 ./tools/rqbench_p /tmp/fv.bin
run rqq_v 60 ./tools/rqbench_q /tmp/fv.bin
run env_s 300 python tools/dump_env.py 1024 native /tmp/env_s.bin
run fp_s 120 ./tools/fpbench /tmp/env_s.bin l
run env_v 300 python tools/dump_env.py 1024 vulpine /tmp/env_v.bin
run fp_v 120 ./tools/fpbench /tmp/env_v.bin l
for f in "$@"; do bash tools/r05_measure.sh "$f" || exit 1; done
