#!/bin/bash
# Round-6 A/B session on one GPU box: parity of the working tree's library on the small-kernel
# and slot suites, then interleaved timings of each library variant on the slot-list drains
# (tools/small_sizes.py slots4k_rand / slots4k, tools/ledger_small.py list), then the product's
# small-kernel timelines. Each GPU step has its own time limit; the script stops at the first
# failure, fault or timeout and never retries.
#   usage: bash tools/ab_r06.sh <tag> <steps> <lib>...   (lib: 0 = product, else a path)
#   steps: comma list of test,sizes,uni,list,tl,bench
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
  timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    tests/test_gpu_small.py tests/test_gpu_small_fuzz.py tests/test_gpu_small_fast.py tests/test_gpu_slots.py \
    tests/test_gpu_probe.py tests/test_gpu_parity.py > "$OUT/test.log" 2>&1
  stop $? test ;;
esac
ROUNDS=${ROUNDS:-1 2}
RAND=${RAND:-4096,3000,2048,1024,256}
FIXED=${FIXED:-3000,1024,256,64}
case ",$STEPS," in *,sizes,*)
  for r in $ROUNDS; do
    for v in "$@"; do
      SUBSPACE_CRC_PROBE_LIB=$(libpath "$v") timeout -k 10 300 python tools/small_sizes.py $RAND \
        200 200 slots4k_rand > "$OUT/rand${r}_$(stem "$v").jsonl" 2> "$OUT/rand${r}_$(stem "$v").err"
      stop $? "rand_r${r}_$(stem "$v")"
      SUBSPACE_CRC_PROBE_LIB=$(libpath "$v") timeout -k 10 300 python tools/small_sizes.py $FIXED \
        200 200 slots4k > "$OUT/fixed${r}_$(stem "$v").jsonl" 2> "$OUT/fixed${r}_$(stem "$v").err"
      stop $? "fixed_r${r}_$(stem "$v")"
    done
  done ;;
esac
case ",$STEPS," in *,uni,*)
  for r in $ROUNDS; do
    for v in "$@"; do
      SUBSPACE_CRC_PROBE_LIB=$(libpath "$v") timeout -k 10 300 python tools/small_sizes.py 200,1000,1500,3000,100 \
        200 200 uniform_packed > "$OUT/upk${r}_$(stem "$v").jsonl" 2> "$OUT/upk${r}_$(stem "$v").err"
      stop $? "upk_r${r}_$(stem "$v")"
      SUBSPACE_CRC_PROBE_LIB=$(libpath "$v") timeout -k 10 300 python tools/small_sizes.py 256,1024,2000,4000 \
        200 200 uniform > "$OUT/ual${r}_$(stem "$v").jsonl" 2> "$OUT/ual${r}_$(stem "$v").err"
      stop $? "ual_r${r}_$(stem "$v")"
    done
  done ;;
esac
case ",$STEPS," in *,list,*)
  for r in $ROUNDS; do
    for v in "$@"; do
      SUBSPACE_CRC_PROBE_LIB=$(libpath "$v") timeout -k 10 200 python tools/ledger_small.py list,ordered 400 400 2 \
        > "$OUT/list${r}_$(stem "$v").jsonl" 2> "$OUT/list${r}_$(stem "$v").err"
      stop $? "list_r${r}_$(stem "$v")"
    done
  done ;;
esac
case ",$STEPS," in *,tl,*)
  for z in mixed 256; do
    timeout -k 10 300 python tools/small_timeline.py --sizes $z --launches 20 > "$OUT/smalltl_$z.json" 2> "$OUT/smalltl_$z.err"
    stop $? "smalltl_$z"
  done ;;
esac
case ",$STEPS," in *,bench,*)
  timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
  stop $? bench ;;
esac
echo done >> "$OUT/status.txt"
