#!/bin/bash
# A/B of two library builds on tools/bench_configs.py configs, interleaved A B A B in
# separate processes on one box.
#   bash tools/session_ab_configs.sh <tag> <configs> <libA.so> <libB.so>
set -u
TAG=$1; CFG=$2; A=$3; B=$4
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
for i in $(seq 1 ${PAIRS:-2}); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    SUBSPACE_CRC_PROBE_LIB=$lib timeout -k 10 200 python tools/bench_configs.py --configs $CFG > $OUT/$v$i.out 2> $OUT/$v$i.err
    rc=$?
    echo "$v$i rc=$rc" >> $OUT/status.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
echo done >> $OUT/status.txt
