#!/bin/bash
# A/B of two library builds on the config-B uniform launch (sweep_uniform, 512 threads,
# order 0), interleaved A B A B ... in separate processes, after one discarded warm-up run.
#   bash tools/session_libab.sh <tag> <libA.so> <libB.so> [pairs=3]
set -u
TAG=$1; A=$2; B=$3; PAIRS=${4:-3}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
SUBSPACE_CRC_PROBE_LIB=$A timeout -k 10 200 python tools/sweep_uniform.py 65536 512 7 0 > $OUT/warm.out 2> $OUT/warm.err || exit 1
for i in $(seq 1 $PAIRS); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    SUBSPACE_CRC_PROBE_LIB=$lib timeout -k 10 200 python tools/sweep_uniform.py 65536 512 7 0 > $OUT/$v$i.out 2> $OUT/$v$i.err
    rc=$?
    echo "$v$i rc=$rc" >> $OUT/status.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
echo done >> $OUT/status.txt
