#!/bin/bash
# Descriptor-kernel change: all GPU tests, configs C/D timing, and a kernel-trace of config C.
set -u
TAG=${1:-r01bt}
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
run pytest 600 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -rf
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run configs 600 python tools/bench_configs.py --configs C,Cu,D,S
# interleaved A/B on config C: tools/ubench/probes/lib_olddesc.so = a build of the commit before
# the descriptor change (git worktree + make; not kept)
for i in 1 2; do
  SUBSPACE_CRC_PROBE_LIB=$PWD/tools/ubench/probes/lib_olddesc.so run C_old$i 300 python tools/bench_configs.py --configs C,Cu,D
  run C_new$i 300 python tools/bench_configs.py --configs C,Cu,D
done
cd /tmp
run prof_C 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_C -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --configs C
echo done >> $OUT/status.txt
