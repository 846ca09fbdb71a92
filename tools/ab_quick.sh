#!/bin/bash
# Quick A/B of library builds on the bench, alternating twice, with parity
# against the oracle on every run.  Usage: ab_quick.sh lib1.so lib2.so ...
set -u
mkdir -p gpurun_out
libs=("$@")
[ ${#libs[@]} -gt 0 ] || libs=(build_var/libbpmx_head.so bpm_analysis_amd/libbpmx.so)
for rep in 1 2; do
for lib in "${libs[@]}"; do
  BPMX_LIB=$lib timeout -k 10 300 python bench.py --pcie-steps 0 --contexts 0 --exact-steps 0 --host-beat-files 0 > gpurun_out/b.log 2>&1 || exit 1
  grep "^{" gpurun_out/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['ms_per_step'],4), d['parity']['ok'] if d['parity'] else None, d['roofline']['frac'], {k:v['avg_ms'] for k,v in d['kernels'].items() if v['avg_ms']>0.05})"
done
done
