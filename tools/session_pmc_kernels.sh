#!/bin/bash
# PMC passes over tools/pmc_kernels.py, one counter group per pass, each under its own limit.
set -u
TAG=${1:-pmck}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for grp in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
  "SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pmc_kernels.py > $OUT/p$i.out 2> $OUT/p$i.err
  rc=$?
  echo "pass $i rc=$rc" >> $OUT/status.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done >> $OUT/status.txt
