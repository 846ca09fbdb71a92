#!/bin/bash
# A/B of a kernel change: phase timing (kbench, HEAD vs working tree), the GPU
# tests, and bench steps with both libraries (HEAD build in build_var/).
set -u
mkdir -p gpurun_out
if [ -x build_var/kbench_head ]; then
  timeout -k 10 120 ./build_var/kbench_head > gpurun_out/kbench_head.log 2>&1 || exit 1
  timeout -k 10 120 ./tools/kbench > gpurun_out/kbench_new.log 2>&1 || exit 1
  tail -24 gpurun_out/kbench_head.log; tail -24 gpurun_out/kbench_new.log
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?
tail -5 gpurun_out/pt.log
[ $rc -eq 0 ] || exit 1
for lib in build_var/libbpmx_head.so bpm_analysis_amd/libbpmx.so build_var/libbpmx_head.so bpm_analysis_amd/libbpmx.so; do
  BPMX_LIB=$lib timeout -k 10 300 python bench.py --pcie-steps 0 --contexts 0 --exact-steps 0 --host-beat-files 0 > gpurun_out/b.log 2>&1 || exit 1
  grep "^{" gpurun_out/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['ms_per_step'],4), d['parity']['ok'], {k:v['avg_ms'] for k,v in d['kernels'].items() if v['avg_ms']>0.05})"
done
