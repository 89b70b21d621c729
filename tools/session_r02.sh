#!/bin/bash
# Round-2 GPU session: tests -> smoke -> bench (headline + configs) -> rocprof -> PMC -> bench E.
# Stops at the first failure (no GPU work after a fault).
set -u
TAG=${1:-r02}
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
run pytest 900 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 600 -rf
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py
cd /tmp
run prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-e2e
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_FETCH_SIZE -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 2 --settle 0 --config-iters 3 --no-cpu-baseline --no-e2e
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_WRITE_SIZE -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 2 --settle 0 --config-iters 3 --no-cpu-baseline --no-e2e
cd $GRAFT_REPO_ROOT
run bench_E 300 python bench.py --workload E --steps 100
echo done >> $OUT/status.txt
