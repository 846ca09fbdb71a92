#!/bin/bash
# Run GPU steps in order on the gpurun box; stop at the first crash/timeout
# (exit codes other than 0 = ok and 1 = ordinary test failure).
set -u
mkdir -p gpurun_out
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    c5) run bench_c5 900 python bench.py --workload c5 --steps 5 --warmup 2 ;;
    c5_64) run bench_c5_64 600 python bench.py --workload c5 --c5-files 64 --steps 5 --warmup 2 ;;
    gputest) run pytest_gpu_sel 600 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread -k "${GPUTEST_K:-draft}" ;;
    bench_ref) run bench_ref 600 python bench.py --steps 10 --warmup 2 --mode reference ;;
    rocprof) run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --contexts 0 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 --dropin-files 0 ;;
    rocprof_ref) run rocprof_ref 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace_ref -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --contexts 0 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 --dropin-files 0 --mode reference ;;
    rocprof_ref_mc) run rocprof_ref_mc 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_ref_mc -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --contexts 4 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 --dropin-files 0 --mode reference ;;
    pmc_fetch) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --contexts 0 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 --dropin-files 0 ;;
    pmc_write) run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --contexts 0 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 --dropin-files 0 ;;
    pmc_ref_fetch) run pmc_ref_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_ref_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --contexts 0 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 --dropin-files 0 --mode reference ;;
    pmc_ref_write) run pmc_ref_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_ref_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --contexts 0 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 --dropin-files 0 --mode reference ;;
    lanebench) run lanebench 120 ./tools/lanebench ;;
    pipesweep) run pipesweep 600 python tools/pipe_sweep.py --steps 10 ;;
    pipesweep_ref) run pipesweep_ref 600 python tools/pipe_sweep.py --steps 5 --mode reference --shapes 0,0,0 4,0,0 4,192,0 0,0,0 ;;
    fpref) run dump_env_ref 300 python tools/dump_env.py 1024 reference /tmp/env_ref.bin && run fpbench_ref 120 ./tools/fpbench /tmp/env_ref.bin l ;;
    fpnat) run dump_env_nat 300 python tools/dump_env.py 1024 native /tmp/env_nat.bin && run fpbench_nat 120 ./tools/fpbench /tmp/env_nat.bin l ;;
    pipesweep_word) BPMX_CUMASK_PER_WORD=1 run pipesweep_word 600 python tools/pipe_sweep.py --steps 10 --shapes 0,0,0 4,192,0 4,224,0 4,192,64 0,0,0 ;;
    pipesweep_grid) run pipesweep_grid 600 python tools/pipe_sweep.py --steps 10 --shapes 0,0,0,0 0,0,0,448 0,0,0,384 0,0,0,320 2,0,0,384 4,0,0,384 2,0,0,320 4,0,0,320 8,0,0,384 0,0,0,0 ;;
    kprof) run kprof 300 python tools/kprof.py ;;
    kprof_und) run kprof_und 300 python tools/kprof.py --mult 1.0 && run kprof_und_full 300 python tools/kprof.py --mult 1.0 --options 8 ;;
    kprof_ref) run kprof_ref 300 python tools/kprof.py --mode reference ;;
    nbphases) run nb_default 300 python tools/c5_env_prof.py && BPMX_LIB=build_var/libbpmx_nb_nomfma.so run nb_nomfma 300 python tools/c5_env_prof.py && BPMX_LIB=build_var/libbpmx_nb_noepi.so run nb_noepi 300 python tools/c5_env_prof.py && BPMX_LIB=build_var/libbpmx_nb_dma.so run nb_dma 300 python tools/c5_env_prof.py ;;
    c5ctx) run bench_c5_64_k1 600 python bench.py --workload c5 --c5-files 64 --steps 10 --warmup 2 --c5-contexts 1 --c5-parity-files 0 && run bench_c5_64_k3 600 python bench.py --workload c5 --c5-files 64 --steps 10 --warmup 2 --c5-contexts 3 --c5-parity-files 0 && run bench_c5_64_k2 600 python bench.py --workload c5 --c5-files 64 --steps 10 --warmup 2 --c5-contexts 2 --c5-parity-files 0 ;;
    c5conc) run c5_concurrency 600 python tools/c5_concurrency.py 3 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
