#!/bin/bash
# Perf-iteration session: GPU parity tests first (stop on any failure), then configs,
# the uniform-kernel sweep and the launch-mode probe. Each step has its own time limit.
set -u
TAG=${1:-perf}
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
run pytest 900 python -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 600 -rf
run configs 600 python tools/bench_configs.py --configs C,Cu,D,E
run sweep 500 python tools/sweep_uniform.py 65536,1048576 256,512,768,1024 5 0,2
run modes 300 python tools/launch_modes.py
run bench 300 python bench.py --no-cpu-baseline --no-e2e
echo done >> $OUT/status.txt
