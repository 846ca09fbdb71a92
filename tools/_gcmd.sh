set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "draft or c5 or c2 or long_noise or sharded or synthetic_batch or c3_scale" > gpurun_out/pt.log 2>&1; rc=$?; tail -25 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload c5 --steps 5 --warmup 2 > gpurun_out/c5.log 2>&1; rc=$?; tail -3 gpurun_out/c5.log | cut -c1-600; grep -o '"k_rolling_quantile[^}]*}\|"k_draft_bounds[^}]*}' gpurun_out/c5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b.log 2>&1; rc=$?; cut -c1-400 gpurun_out/b.log | tail -2; grep -o '"k_draft_bounds[^}]*}' gpurun_out/b.log; exit $rc
