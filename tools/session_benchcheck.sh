#!/bin/bash
# Bench consistency check: launch modes, bench at two step counts, and a kernel trace of the bench.
set -u
TAG=${1:-benchcheck}
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
run modes 300 python tools/launch_modes.py
run bench200 300 python bench.py --no-cpu-baseline --no-e2e
run bench1000 300 python bench.py --no-cpu-baseline --no-e2e --steps 1000 --warmup 50
cd /tmp
run prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-e2e
echo done >> $OUT/status.txt
