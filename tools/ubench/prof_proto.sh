set -e
mkdir -p gpurun_out
timeout -k 10 300 ./tools/ubench/crcproto > gpurun_out/crcproto2.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/ubench/crcproto 1 > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $GRAFT_REPO_ROOT/gpurun_out/pmc1 -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/ubench/crcproto 1 > $GRAFT_REPO_ROOT/gpurun_out/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/pmc2 -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/ubench/crcproto 1 > $GRAFT_REPO_ROOT/gpurun_out/pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/gpurun_out/pmc3 -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/ubench/crcproto 1 > $GRAFT_REPO_ROOT/gpurun_out/pmc3.log 2>&1
