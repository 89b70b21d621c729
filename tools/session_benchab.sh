#!/bin/bash
# bench.py's headline (config B, 1,000 timed launches) for several library builds,
# interleaved round-robin in separate processes.
#   [BENCH_ARGS="--workload E --steps 50"] bash tools/session_benchab.sh <tag> <rounds> <lib.so>...
set -u
TAG=$1; ROUNDS=$2; shift 2
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
for i in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    n=$(basename $lib .so)
    SUBSPACE_CRC_PROBE_LIB=$lib timeout -k 10 200 python bench.py --configs none --no-e2e --no-cpu-baseline ${BENCH_ARGS:-} \
      > $OUT/b_${n}_$i.out 2> $OUT/b_${n}_$i.err
    rc=$?; echo "b_${n}_$i rc=$rc" >> $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
  done
done
echo done >> $OUT/status.txt
