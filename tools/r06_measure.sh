#!/bin/bash
# r06 final measurement set on one box: bench (native, reference), the C5 64-recording
# shard, rocprofv3 kernel statistics, PMC traffic (separate FETCH_SIZE and
# WRITE_SIZE passes), the stage profile (roctx ranges), smoke.  Each step under
# its own time limit; the first failure stops the call.
set -u
O=gpurun_out/${R06_OUT:-r06m}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--no-cpu --contexts 0 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 --dropin-files 0 --real-env-steps 0"
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 2 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
for s in "$@"; do
  case $s in
    ptk) step pytest_k 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "${PTK}" ;;
    pt) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    bench) step bench 600 python bench.py ;;
    benchq) step benchq 600 python bench.py $Q ;;
    benchq_notie) step benchq_notie 600 python bench.py $Q --tie-check off ;;
    benchq_pipe) step benchq_pipe 600 python bench.py $Q --batch-pipeline on ;;
    bench_ref) step bench_ref 600 python bench.py --mode reference --steps 10 --warmup 2 --real-env-steps 0 ;;
    bench_ref_serial) step bench_ref_serial 600 python bench.py --mode reference --steps 10 --warmup 2 --real-env-steps 0 --batch-pipeline off --contexts 0 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 --dropin-files 0 --no-cpu ;;
    c5) step bench_c5_64 900 python bench.py --workload c5 --c5-files 64 --steps 5 --warmup 2 ;;
    stats) step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- python3 bench.py --steps 5 --warmup 1 $Q ;;
    stats_ref) step rocprof_stats_ref 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats_ref -o run -- python3 bench.py --mode reference --steps 5 --warmup 1 $Q ;;
    stage) step stage 600 rocprofv3 --kernel-trace --marker-trace --hip-runtime-trace --output-format csv -d $O/prof_stage -o run -- python3 bench.py --steps 3 --warmup 1 $Q ;;
    fetch) step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- python3 bench.py --steps 3 --warmup 1 $Q ;;
    write) step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- python3 bench.py --steps 3 --warmup 1 $Q ;;
    kt) step ktime 900 python tools/ktime.py ${KT:-build_var/libbpmx_head.so bpm_analysis_amd/libbpmx.so} ;;
    hb) step hbench 120 ./tools/hbench ;;
    ov) step overlap 120 ./tools/overlap_probe ;;
    rep) step realenv 900 python tools/realenv_prof.py reference ${REP:-build_var/libbpmx_head.so bpm_analysis_amd/libbpmx.so} ;;
    rpp) step refpipe 800 python tools/refpipe_probe.py reference ;;
    bench_ref_off) step bench_ref_off 600 python bench.py --mode reference --steps 10 --warmup 2 --real-env-steps 0 --batch-pipeline off --no-cpu --contexts 0 --pcie-steps 0 --exact-steps 0 --host-beat-files 0 --dropin-files 0 ;;
    c5h) step bench_c5_head 900 env BPMX_LIB=build_var/libbpmx_head.so python bench.py --workload c5 --c5-files 64 --steps 5 --warmup 2 ;;
    rqb) step rqbench 120 ./tools/rqbench /tmp/floor_in.bin ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown $s"; exit 2 ;;
  esac
done
