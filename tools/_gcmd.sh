set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/hbench 1024 18124 > gpurun_out/hb.log 2>&1; rc=$?; cat gpurun_out/hb.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "hilbert or native_mode_golden or c3_scale or native_ragged" > gpurun_out/pt.log 2>&1; rc=$?; tail -15 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/b.log 2>&1; rc=$?; cut -c1-300 gpurun_out/b.log | tail -2; grep -o '"k_hilbert_env[^}]*}' gpurun_out/b.log; grep -o '"parity[^}]*}' gpurun_out/b.log; exit $rc
