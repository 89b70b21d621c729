#!/bin/bash
# Uniform-kernel probe builds (tools/ubench/build_probes.sh) timed side by side.
set -u
TAG=${1:-probes}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
for n in 0 1 3 7; do
  lib=""
  [ $n -ne 0 ] && lib=tools/ubench/probes/libprobe$n.so
  SUBSPACE_CRC_PROBE_LIB=$lib timeout -k 10 300 python tools/sweep_uniform.py 65536,1048576 512 5 0 1 1 > $OUT/probe$n.out 2> $OUT/probe$n.err
  rc=$?
  echo "probe$n rc=$rc" >> $OUT/status.txt
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 200 ./tools/ubench/streamread > $OUT/streamread.out 2>&1
echo "streamread rc=$?" >> $OUT/status.txt
