#!/bin/bash
# Compute ledger of the headline kernel: kernel timing and SQ counters
# for config B (hbm), its compute-only twin (l2: every message aliasing one 4 KiB message) and
# the read probe (read), one rocprofv3 pass per counter group and mode (tools/ledger_uniform.py).
# LEDGER=small: the slot-list drain instead (tools/ledger_small.py; modes list, alias, probe0 ...).
# Passes: t (kernel trace), p1-p3 (SQ groups), f / w (TCC FETCH_SIZE / WRITE_SIZE: HBM bytes).
#   usage: [LEDGER=small] bash tools/pmc_ledger.sh <tag> [modes] [passes]
# Each step has its own time limit; the script stops at the first abort, fault or timeout.
set -u
TAG=${1:-ledger}
LEDGER=${LEDGER:-uniform}
if [ "$LEDGER" = small ]; then DEFMODES="list alias probe0"; else DEFMODES="hbm l2 read"; fi
MODES=${2:-$DEFMODES}
PASSES=${3:-"t p1 p2 p3"}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp

counters() {
  case $1 in
    p1) echo "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" ;;
    p2) echo "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM" ;;
    p3) echo "SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_IFETCH SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR" ;;
    ic1) echo "SQC_ICACHE_HITS SQC_ICACHE_MISSES" ;;
    ic2) echo "SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ" ;;
    f) echo "FETCH_SIZE" ;;
    w) echo "WRITE_SIZE" ;;
  esac
}

timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1
echo "list rc=$?" >> "$OUT/status.txt"
for m in $MODES; do
  for p in $PASSES; do
    if [ "$p" = t ]; then
      timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/${m}_t" -o run --output-format csv -- \
        python3 "$ROOT/tools/ledger_$LEDGER.py" "$m" 1000 400 > "$OUT/${m}_t.json" 2> "$OUT/${m}_t.err"
    else
      timeout -s KILL 90 rocprofv3 --pmc $(counters $p) -d "$OUT/${m}_$p" -o run --output-format csv -- \
        python3 "$ROOT/tools/ledger_$LEDGER.py" "$m" 50 100 > "$OUT/${m}_$p.json" 2> "$OUT/${m}_$p.err"
    fi
    rc=$?
    echo "$m $p rc=$rc" >> "$OUT/status.txt"
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stop" >> "$OUT/status.txt"; exit $rc; fi
  done
done
echo done >> "$OUT/status.txt"
