set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 ./tools/nbbench 1024 60 146 "va<19> x8" > gpurun_out/nb_va.log 2>&1
cat gpurun_out/nb_va.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_va -o run -- $GRAFT_REPO_ROOT/tools/nbbench 1024 60 146 "va<19> x8" > $GRAFT_REPO_ROOT/gpurun_out/pmc_va.log 2>&1
