#!/bin/bash
# Status session: launch modes, the WG/order sweep and the secondary configs, each step
# under its own time limit; stops at the first failure.
set -u
TAG=${1:-status}
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
run sweep 400 python tools/sweep_uniform.py 65536,1048576 256,512,1024 5 0,2
run configs 600 python tools/bench_configs.py --configs C,Cu,D,E
echo done >> $OUT/status.txt
