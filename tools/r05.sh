#!/bin/bash
# r05 measurement steps on one box (each step under its own time limit; the first failure stops the call).
# the C5 64-recording shard with full oracle parity, rocprofv3 kernel stats and PMC traffic.
set -u
mkdir -p gpurun_out/r05
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r05/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 3 "gpurun_out/r05/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
for s in "$@"; do
  case $s in
    bench) step bench 600 python bench.py ;;
    bench_ref) step bench_ref 600 python bench.py --mode reference --steps 10 --warmup 2 ;;
    c5) step bench_c5_64 900 python bench.py --workload c5 --c5-files 64 --steps 5 --warmup 2 ;;
    stats) step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05/prof_stats -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --contexts 0 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 --dropin-files 0 ;;
    fetch) step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r05/prof_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --contexts 0 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 --dropin-files 0 ;;
    write) step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r05/prof_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --contexts 0 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 --dropin-files 0 ;;
    pt) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    pt_tie) step pytest_tie 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "tie or vulpine" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown $s"; exit 2 ;;
  esac
done
