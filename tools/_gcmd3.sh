set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --contexts 0 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 > gpurun_out/b1.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/b1.log; grep -o '"k_native_blocks": {[^}]*}' gpurun_out/b1.log
BPMX_LIB=tools/libbpmx_slots2.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --contexts 0 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 > gpurun_out/b2.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/b2.log; grep -o '"k_native_blocks": {[^}]*}' gpurun_out/b2.log
