#!/bin/bash
# Interleaved comparison of several library builds on the secondary configs, same box:
# PASSES (default 2) passes over the list (L1 L2 ... L1 L2 ...), one bench_configs process per run.
#   bash tools/session_libs.sh <tag> <configs> <lib.so>...
set -u
TAG=$1; CF=$2; shift 2
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for pass in $(seq 1 ${PASSES:-2}); do
  i=0
  for lib in "$@"; do
    i=$((i + 1))
    SUBSPACE_CRC_PROBE_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --configs $CF \
      > $OUT/L${i}_p$pass.out 2> $OUT/L${i}_p$pass.err
    rc=$?
    echo "L$i ($lib) pass $pass rc=$rc" >> $OUT/status.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
echo done >> $OUT/status.txt
