#!/bin/bash
# slot_gap.py + per-wave timelines for the given slot-kernel variants
set -u
TAG=$1; shift
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
for v in "$@"; do
  SUBSPACE_CRC_PROBE_LIB=$PWD/tools/ubench/probes/libslot$v.so SLOT_GAP_NOCHECK=1 \
    timeout -k 10 200 python tools/slot_gap.py 3 > $OUT/v$v.jsonl 2> $OUT/v$v.err || exit $?
  SUBSPACE_CRC_PROBE_LIB=$PWD/tools/ubench/probes/libslot$v.so SLOT_GAP_NOCHECK=1 \
    timeout -k 10 200 python tools/wave_timeline.py --mode publish --launches 10 > $OUT/tl_v$v.jsonl 2> $OUT/tl_v$v.err || exit $?
done
echo done > $OUT/status.txt
