#!/bin/bash
# per-wave timelines with HW_ID placement: config B (plain kernel), config S publish with the
# product library and slot variants 1 and 2 (tools/ubench/build_slot_variants.sh)
set -u
TAG=$1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 200 python tools/wave_timeline.py --mode uniform --launches 10 > $OUT/tl_uniform.jsonl 2> $OUT/tl_uniform.err || exit $?
timeout -k 10 200 python tools/wave_timeline.py --mode publish --launches 10 > $OUT/tl_v0.jsonl 2> $OUT/tl_v0.err || exit $?
for v in 1 2; do
  SUBSPACE_CRC_PROBE_LIB=$PWD/tools/ubench/probes/libslot$v.so SLOT_GAP_NOCHECK=1 \
    timeout -k 10 200 python tools/wave_timeline.py --mode publish --launches 10 > $OUT/tl_v$v.jsonl 2> $OUT/tl_v$v.err || exit $?
done
echo done > $OUT/status.txt
