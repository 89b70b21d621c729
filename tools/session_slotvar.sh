#!/bin/bash
# slot_gap.py (config S kernels vs the plain kernel, interleaved) with the product library and
# each timing-only slot-kernel variant (tools/ubench/build_slot_variants.sh), one process each.
#   bash tools/session_slotvar.sh <tag> <variant>...
set -u
TAG=$1; shift
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 200 python tools/slot_gap.py 3 > $OUT/v0.jsonl 2> $OUT/v0.err || exit $?
for v in "$@"; do
  SUBSPACE_CRC_PROBE_LIB=$PWD/tools/ubench/probes/libslot$v.so SLOT_GAP_NOCHECK=1 \
    timeout -k 10 200 python tools/slot_gap.py 3 > $OUT/v$v.jsonl 2> $OUT/v$v.err
  rc=$?
  echo "v$v rc=$rc" >> $OUT/status.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 200 python tools/wave_timeline.py --mode publish --launches 10 > $OUT/timeline_publish.jsonl 2> $OUT/timeline.err
echo "done rc=$?" >> $OUT/status.txt
