#!/bin/bash
# tools/slot_gap.py for several library builds, interleaved round-robin in separate processes.
#   bash tools/session_slotab.sh <tag> <rounds> <lib.so>...
set -u
TAG=$1; ROUNDS=$2; shift 2
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
for i in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    n=$(basename $lib .so)
    SUBSPACE_CRC_PROBE_LIB=$lib timeout -k 10 200 python tools/slot_gap.py ${SLOT_GAP_ROUNDS:-3} > $OUT/g_${n}_$i.out 2> $OUT/g_${n}_$i.err
    rc=$?; echo "g_${n}_$i rc=$rc" >> $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
  done
done
echo done >> $OUT/status.txt
