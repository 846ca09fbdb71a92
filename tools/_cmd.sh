set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pt_all.log 2>&1; rc=$?
tail -25 gpurun_out/pt_all.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu --pcie-steps 0 > gpurun_out/bench_o0.log 2>&1 || exit 1
grep "^{" gpurun_out/bench_o0.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
