#!/bin/bash
# Kernel trace + PMC passes of any python3 command, one pass per counter group (never combined with
# another tracing domain), then tools/prof_summary.py.
#   tools/kprof.sh <outdir> "<python3 args>" "<counter group 1>" ["<counter group 2>" ...]
# e.g. tools/kprof.sh gpurun_out/cfg4 "tools/prof_driver.py --cfg 4 --calls 5" "FETCH_SIZE" "WRITE_SIZE"
# Environment (GEMMUL8_SINGLE_STREAM=1 etc.) passes through to the profiled program.
set -o pipefail
OUT=$1
ARGS=$2
shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 $ARGS > "$OUT/trace.log" 2>&1 \
  || { echo "kernel trace failed"; exit 1; }
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -f csv -d "$OUT/pmc$i" -o run -- python3 $ARGS > "$OUT/pmc$i.log" 2>&1 \
    || { echo "pmc pass $i ($grp) failed"; exit 1; }
done
python3 tools/prof_summary.py "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
