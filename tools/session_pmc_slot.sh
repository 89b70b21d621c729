#!/bin/bash
# PMC passes over tools/pmc_slot.py for several library builds, one counter group per pass,
# each under its own limit.   bash tools/session_pmc_slot.sh <tag> <lib.so>...
set -u
TAG=$1; shift
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  i=0
  for grp in "SQ_WAIT_INST_ANY SQ_IFETCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" "SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
    i=$((i+1))
    SUBSPACE_CRC_PROBE_LIB=$GRAFT_REPO_ROOT/$lib timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/${n}_p$i -o run \
      --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pmc_slot.py > $OUT/${n}_p$i.out 2> $OUT/${n}_p$i.err
    rc=$?
    echo "$n pass $i rc=$rc" >> $OUT/status.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
echo done >> $OUT/status.txt
