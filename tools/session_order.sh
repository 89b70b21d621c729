#!/bin/bash
# Does a preceding heavy run (tools/bench_configs.py) lower the next bench.py? pytest -> bench x2 -> configs -> bench x2.
set -u
TAG=${1:-r01bx}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  echo "$name rc=$rc" >> $OUT/status.txt
  if [ $rc -ne 0 ]; then echo "stop after $name" >> $OUT/status.txt; exit $rc; fi
}
run pytest 600 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench1 300 python bench.py
run bench2 300 python bench.py --no-cpu-baseline --no-e2e
run configs 600 python tools/bench_configs.py --configs C,Cu,D,E
run bench3 300 python bench.py --no-cpu-baseline --no-e2e
run bench4 300 python bench.py --no-cpu-baseline --no-e2e
rocm-smi --showtemp --showpower --showclocks > $OUT/smi.txt 2>&1
echo done >> $OUT/status.txt
