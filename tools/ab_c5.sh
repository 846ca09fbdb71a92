#!/bin/bash
# GPU tests (all, or those matching $1), then the C5 shard bench with the HEAD
# build (build_var/) and the working tree's library, then the metric A/B.
set -u
mkdir -p gpurun_out
sel=${1:-}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${sel:+-k "$sel"} > gpurun_out/ptq.log 2>&1; rc=$?
tail -4 gpurun_out/ptq.log
[ $rc -eq 0 ] || exit 1
for lib in build_var/libbpmx_head.so bpm_analysis_amd/libbpmx.so; do
  BPMX_LIB=$lib timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 > gpurun_out/c5.log 2>&1 || exit 1
  grep "^{" gpurun_out/c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['ms_per_step'],3), d['parity']['ok'], d['roofline']['frac'], {k:round(v['avg_ms']*v['launches']/2,3) for k,v in d['kernels'].items() if v['avg_ms']*v['launches']/2>0.2})"
done
