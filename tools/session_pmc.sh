#!/bin/bash
# PMC passes over the uniform kernel (one counter group per rocprofv3 run, no trace domains).
set -u
TAG=${1:-pmc}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "TA_TA_BUSY_sum TA_BUSY_avr TCP_TCC_READ_REQ_sum" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_uniform.py ${2:-1048576} 6 > $OUT/pmc$i.out 2> $OUT/pmc$i.err
  rc=$?
  echo "pmc$i ($grp) rc=$rc" >> $OUT/status.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done >> $OUT/status.txt
