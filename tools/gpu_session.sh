#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 summaries.
# Each GPU step has its own time limit; the script stops at the first fault,
# abort, segfault or timeout (exit status >= 124 or > 128) and never retries.
#   usage: bash tools/gpu_session.sh [tag] [steps...]   steps: test smoke bench prof profsel pmc configs
#   (profsel: rocprofv3 --selected-regions around bench.py --roctx-region = exactly the timed launches)
set -u
TAG=${1:-r01}
shift || true
STEPS=${*:-"test smoke bench profsel pmc"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

stop_if_fault() {  # $1 = exit status, $2 = step name
  local rc=$1
  echo "step $2 rc=$rc" >> "$OUT/status.txt"
  if [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; then
    echo "stopping after $2 (rc=$rc)" >> "$OUT/status.txt"
    exit "$rc"
  fi
}

for s in $STEPS; do
  case $s in
    test)
      timeout -k 10 1200 python -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 600 -rf \
        > "$OUT/pytest_gpu.log" 2>&1
      rc=$?
      # any failed GPU test ends the session: a fault must not be followed by more GPU work
      if [ $rc -ne 0 ]; then echo "step test rc=$rc (stop)" >> "$OUT/status.txt"; exit $rc; fi
      stop_if_fault $rc test ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      stop_if_fault $? smoke ;;
    bench)
      timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
      stop_if_fault $? bench ;;
    prof)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run \
        --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline \
        --no-e2e > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err")
      stop_if_fault $? prof ;;
    profsel)  # the timed region only: roctxProfilerResume/Pause around it (--marker-trace routes them to the tool)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --marker-trace --selected-regions -d "$GRAFT_REPO_ROOT/$OUT/profsel" -o run \
        --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-e2e --configs none \
        --roctx-region > "$GRAFT_REPO_ROOT/$OUT/profsel_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/profsel.err")
      stop_if_fault $? profsel ;;
    pmc)
      for ctr in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && timeout -k 10 600 rocprofv3 --pmc $ctr -d "$GRAFT_REPO_ROOT/$OUT/pmc_$ctr" -o run \
          --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 2 --settle 0 --no-cpu-baseline \
          --no-e2e > "$GRAFT_REPO_ROOT/$OUT/pmc_$ctr.json" 2> "$GRAFT_REPO_ROOT/$OUT/pmc_$ctr.err")
        stop_if_fault $? "pmc_$ctr"
      done ;;
    configs)
      timeout -k 10 600 python tools/bench_configs.py --configs C,Cu,D,E,S > "$OUT/configs.log" 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "step configs rc=$rc (stop)" >> "$OUT/status.txt"; exit $rc; fi ;;
    slottest)  # the slot, fault and config-S tests only (a kernel change's first check)
      timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
        tests/test_gpu_fault.py tests/test_gpu_slots.py tests/test_gpu_configs.py -k "fault or slot or Slot or S_ or stream" \
        > "$OUT/pytest_slot.log" 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "step slottest rc=$rc (stop)" >> "$OUT/status.txt"; exit $rc; fi ;;
    slotgap)  # config S kernels vs the plain uniform kernel over the same buffers, interleaved
      timeout -k 10 300 python tools/slot_gap.py 5 > "$OUT/slot_gap.jsonl" 2> "$OUT/slot_gap.err"
      stop_if_fault $? slotgap ;;
    timeline)  # per-wave timelines: config B, config S payloads, publish, verify
      for m in uniform uniform4160 publish verify; do
        timeout -k 10 300 python tools/wave_timeline.py --mode $m --launches 20 > "$OUT/timeline_$m.jsonl" 2> "$OUT/timeline_$m.err"
        stop_if_fault $? "timeline_$m"
      done ;;
    smalltl)  # small-kernel timelines (PROBE hook): S_short's and S_mixed's shuffled lists, config S's
      for z in 256 mixed 4096; do
        timeout -k 10 300 python tools/small_timeline.py --sizes $z --launches 20 > "$OUT/smalltl_$z.json" 2> "$OUT/smalltl_$z.err"
        stop_if_fault $? "smalltl_$z"
      done ;;
    *)
      echo "unknown step $s" >> "$OUT/status.txt" ;;
  esac
done
echo done >> "$OUT/status.txt"
