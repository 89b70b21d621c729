#!/bin/bash
# Wave timelines (tools/wave_timeline.py) of several library builds, then their config-B
# launch times interleaved round-robin in separate processes (tools/sweep_uniform.py).
#   bash tools/session_multi.sh <tag> <rounds> <lib.so>...
set -u
TAG=$1; ROUNDS=$2; shift 2
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
run() {  # name, command...
  local name=$1; shift
  timeout -k 10 200 "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  echo "$name rc=$rc" >> $OUT/status.txt
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for lib in "$@"; do
  n=$(basename $lib .so)
  SUBSPACE_CRC_PROBE_LIB=$lib run tl_$n python tools/wave_timeline.py --launches 20
done
for i in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    n=$(basename $lib .so)
    SUBSPACE_CRC_PROBE_LIB=$lib run ab_${n}_$i python tools/sweep_uniform.py 65536 512 7 0
  done
done
echo done >> $OUT/status.txt
