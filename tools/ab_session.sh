#!/bin/bash
# Interleaved A/B of library builds on one GPU box, one process per run, after one discarded
# warm-up process (a fresh box's first GPU process runs slower: profiles/DESIGN_r01-r03.md 4.0).
#   bash tools/ab_session.sh <tag> <mode> <lib>...
#   lib:  0 = the product library; N = tools/ubench/probes/libslotN.so
#         (tools/ubench/build_variants.sh); env:VAR=VALUE = the product library with VAR set
#         (a context knob, e.g. env:SUBSPACE_CRC_UNIFORM_SHIFT2=1); anything else = a path
#         (e.g. abtmp/lib_x.so from tools/ab_lib.sh). Repeat libs for an A B A B order.
#   mode: slotgap -- tools/slot_gap.py: config S publish / verify vs the plain kernel over the
#                    same buffers (timing only: variants may compute nothing valid)
#         uniform -- tools/sweep_uniform.py: config B through the uniform kernel
#         slotlist -- tools/slot_list_order.py: config S verified strided (fused uniform) and
#                     as an ordered / shuffled slot list (small-message kernel)
# Summaries: python tools/show_ab.py gpurun_out/<tag>
set -u
TAG=$1; MODE=$2; shift 2
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p $OUT
run() {  # $1 = output stem, $2 = library path or "" (or env:VAR=VALUE)
  local envset=""
  case $2 in env:*) envset=${2#env:}; set -- "$1" "" ;; esac
  if [ -n "$envset" ]; then export "${envset?}"; fi
  if [ "$MODE" = slotgap ]; then
    SUBSPACE_CRC_PROBE_LIB=$2 SLOT_GAP_NOCHECK=1 timeout -k 10 200 python tools/slot_gap.py 3 > $OUT/$1.jsonl 2> $OUT/$1.err
  elif [ "$MODE" = slotlist ]; then
    SUBSPACE_CRC_PROBE_LIB=$2 SLOT_LIST_NOCHECK=1 timeout -k 10 200 python tools/slot_list_order.py 3 > $OUT/$1.jsonl 2> $OUT/$1.err
  else
    SUBSPACE_CRC_PROBE_LIB=$2 timeout -k 10 200 python tools/sweep_uniform.py 65536 512 7 0 > $OUT/$1.jsonl 2> $OUT/$1.err
  fi
  local rc=$?
  if [ -n "$envset" ]; then unset "${envset%%=*}"; fi
  return $rc
}
run warm "" || exit $?
i=0
for v in "$@"; do
  i=$((i + 1))
  lib=""
  if [ "$v" != 0 ]; then
    case $v in
      env:*) lib=$v ;;
      *[!0-9]*) lib=$v ;;
      *) lib=$PWD/tools/ubench/probes/libslot$v.so ;;
    esac
  fi
  stem=$(basename "${v%.so}"); stem=${stem//[:=]/_}
  run "run${i}_$stem" "$lib"
  rc=$?
  echo "run$i $v rc=$rc" >> $OUT/status.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done >> $OUT/status.txt
