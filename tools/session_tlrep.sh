#!/bin/bash
# Repeated wave timelines of several library builds, interleaved (probe instantiation).
#   bash tools/session_tlrep.sh <tag> <rounds> <lib.so>...
set -u
TAG=$1; ROUNDS=$2; shift 2
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
for i in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    n=$(basename $lib .so)
    SUBSPACE_CRC_PROBE_LIB=$lib timeout -k 10 200 python tools/wave_timeline.py --launches 20 > $OUT/tl_${n}_$i.out 2> $OUT/tl_${n}_$i.err
    rc=$?; echo "tl_${n}_$i rc=$rc" >> $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
  done
done
echo done >> $OUT/status.txt
