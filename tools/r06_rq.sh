#!/bin/bash
# r06: final-floor sort variants on the bench's own curves and on the
# reference's sample (rqbench phase stamps, bit-exact check vs the library).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${R06_OUT:-rq}; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$O/$name.txt" 2>&1; local rc=$?; grep -v "^   \|mismatch" "$O/$name.txt" | tail -n 4; [ $rc -eq 0 ] || { echo "STOP rc=$rc after $name"; exit $rc; }; }
run dfi_s 300 python tools/dump_floor_inputs.py 1024 native /tmp/fs.bin
for v in "$@"; do run rq_s_$v 60 ./tools/rqbench_$v /tmp/fs.bin; done
run dfi_v 300 python tools/dump_floor_inputs.py 1024 vulpine /tmp/fv.bin
for v in "$@"; do run rq_v_$v 60 ./tools/rqbench_$v /tmp/fv.bin; done
