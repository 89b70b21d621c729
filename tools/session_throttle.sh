#!/bin/bash
# Uniform-kernel variants under sustained launches: parity tests of the tuned variants,
# then wall-clock phases and a kernel trace of the same script.
set -u
TAG=${1:-throttle}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  echo "$name rc=$rc" >> $OUT/status.txt
  if [ $rc -ne 0 ]; then echo "stop after $name" >> $OUT/status.txt; exit $rc; fi
}
run phases 300 python tools/throttle_trace.py --launches 400 --variants 0,1,0,1
cd /tmp
run prof 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/throttle_trace.py --launches 400 --variants 0,1,0,1
echo done >> $OUT/status.txt
