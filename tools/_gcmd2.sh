set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/refbench > gpurun_out/rb.log 2>&1; rc=$?; cat gpurun_out/rb.log; [ $rc -eq 0 ] || exit $rc
bash tools/_gcmd.sh
