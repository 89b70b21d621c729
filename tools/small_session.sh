#!/bin/bash
# Slot-list drain (small-message kernel) investigation session on one GPU box (VERDICT r04
# item 1): parity of each library variant on the small-kernel tests, interleaved timing of the
# variants (tools/ledger_small.py list / ordered / list1), the read probes, then the PMC ledger
# of the product library (LEDGER=small tools/pmc_ledger.sh). Every GPU step has its own time
# limit; the script stops at the first failure, fault or timeout and never retries.
#   usage: bash tools/small_session.sh <tag> <steps> <lib>...   (lib: 0 = product, else a path)
#   steps: comma list of test,ab,probe,ledger
set -u
TAG=$1; STEPS=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
libpath() { if [ "$1" = 0 ]; then echo ""; else echo "$ROOT/$1"; fi; }
stem() { if [ "$1" = 0 ]; then echo product; else basename "${1%.so}"; fi; }
stop() {  # $1 rc, $2 step
  echo "$2 rc=$1" >> "$OUT/status.txt"
  if [ "$1" -ne 0 ]; then echo "stop" >> "$OUT/status.txt"; exit "$1"; fi
}
case ",$STEPS," in *,test,*)
  for v in "$@"; do
    SUBSPACE_CRC_PROBE_LIB=$(libpath "$v") timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider \
      --timeout 120 --timeout-method thread tests/test_gpu_small.py > "$OUT/test_$(stem "$v").log" 2>&1
    stop $? "test_$(stem "$v")"
  done ;;
esac
case ",$STEPS," in *,ab,*)
  SUBSPACE_CRC_PROBE_LIB="" timeout -k 10 200 python tools/ledger_small.py list,strided 200 400 1 > "$OUT/warm.jsonl" 2> "$OUT/warm.err"
  stop $? warm
  for r in 1 2; do
    for v in "$@"; do
      SUBSPACE_CRC_PROBE_LIB=$(libpath "$v") timeout -k 10 200 python tools/ledger_small.py list,ordered,list1 400 400 2 \
        > "$OUT/run${r}_$(stem "$v").jsonl" 2> "$OUT/run${r}_$(stem "$v").err"
      stop $? "ab_r${r}_$(stem "$v")"
    done
  done ;;
esac
case ",$STEPS," in *,probe,*)
  timeout -k 10 200 python tools/ledger_small.py probe0,probe1,probe0o,strided,alias,list 400 400 3 > "$OUT/probes.jsonl" 2> "$OUT/probes.err"
  stop $? probes ;;
esac
case ",$STEPS," in *,ledger,*)
  LEDGER=small bash "$ROOT/tools/pmc_ledger.sh" "$TAG/ledger" "list alias probe0" "t p1 p2 p3 f"
  stop $? ledger ;;
esac
echo done >> "$OUT/status.txt"
