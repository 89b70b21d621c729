#!/bin/bash
# HBM traffic of bench.py's secondary configurations: for each configuration, two rocprofv3 PMC
# passes (FETCH_SIZE, WRITE_SIZE; separate runs, MI355X_MICROARCH.md "HBM") over
# tools/pmc_configs.py, one process per configuration and pass. Each step has its own time
# limit; the script stops at the first failure, fault or timeout and never retries.
#   usage: bash tools/pmc_configs.sh <tag> [configs]
#   then:  python tools/summarize_configs_traffic.py gpurun_out/<tag>   (-> profiles/traffic_configs.json)
set -u
TAG=$1
CONFIGS=${2:-"C Cu D Du S_publish S_verify S_meta_publish S_meta_verify S_list_publish S_list_verify Usmall S_short S_mixed S_large_verify S_large_publish"}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for c in $CONFIGS; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $ctr -d "$OUT/${c}_$ctr" -o run --output-format csv -- \
      python3 "$ROOT/tools/pmc_configs.py" "$c" 5 > "$OUT/${c}_$ctr.json" 2> "$OUT/${c}_$ctr.err"
    rc=$?
    echo "$c $ctr rc=$rc" >> "$OUT/status.txt"
    if [ $rc -ne 0 ]; then echo "stop" >> "$OUT/status.txt"; exit $rc; fi
  done
done
echo done >> "$OUT/status.txt"
