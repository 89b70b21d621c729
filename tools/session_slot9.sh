#!/bin/bash
# Slot-kernel experiment session: slot/probe/config-S GPU tests, then tools/slot_gap.py
# interleaved over library builds.   bash tools/session_slot9.sh <tag> <lib.so>...
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_slots.py tests/test_gpu_probe.py tests/test_gpu_configs.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "slot or Slot or probe or config_S" > $OUT/pytest.log 2>&1 || { echo "pytest failed" >> $OUT/status.txt; exit 1; }
echo pytest ok >> $OUT/status.txt
SLOT_GAP_ROUNDS=3 bash tools/session_slotab.sh $TAG 3 "$@"
