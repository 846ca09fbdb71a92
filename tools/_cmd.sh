set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_all.log 2>&1 || { tail -40 gpurun_out/pt_all.log; exit 1; }
tail -2 gpurun_out/pt_all.log
for o in 0; do
timeout -k 10 300 python bench.py --no-cpu --pcie-steps 0 --options $o > gpurun_out/bench_o$o.log 2>&1 || exit 1
grep "^{" gpurun_out/bench_o$o.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($o, d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
done
