#!/bin/bash
# A/B of two library builds on the secondary configs, interleaved (A B A B), same box.
#   bash tools/session_ab.sh <tag> <libA.so> <libB.so> [configs]
set -u
TAG=$1; A=$2; B=$3; CF=${4:-C,Cu,D,E}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    SUBSPACE_CRC_PROBE_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --configs $CF > $OUT/$v$i.out 2> $OUT/$v$i.err
    rc=$?
    echo "$v$i rc=$rc" >> $OUT/status.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
echo done >> $OUT/status.txt
