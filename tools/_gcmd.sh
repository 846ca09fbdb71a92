set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "reference or vulpine or synthetic_batch or ragged_batch_matches or dropin or c2 or c5_96k or stub or draft_bounds_window" > gpurun_out/pt.log 2>&1; rc=$?; tail -30 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --mode reference --no-cpu > gpurun_out/br.log 2>&1; rc=$?; cut -c1-300 gpurun_out/br.log | tail -2; grep -o '"k_envelope_ref[^}]*}\|"k_ref_env_mean[^}]*}' gpurun_out/br.log; exit $rc
