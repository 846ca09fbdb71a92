set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "dma_block or c5 or large_decimation or tile_geometries or block_kernels" > gpurun_out/pt.log 2>&1; rc=$?; tail -25 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload c5 --steps 5 --warmup 2 > gpurun_out/c5.log 2>&1; rc=$?; tail -3 gpurun_out/c5.log | cut -c1-900; grep -o '"k_native_blocks"[^}]*}' gpurun_out/c5.log; exit $rc
