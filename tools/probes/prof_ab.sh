#!/bin/bash
# Kernel trace + PMC passes (one counter group per pass) over one probe command; summary via
# tools/prof_summary.py.  Usage: tools/probes/prof_ab.sh <tag> <probe binary> [args...]
set -e
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pab_$TAG
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- "$@" > $OUT/trace.log 2>&1
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -f csv -d $OUT/pmc$i -o run -- "$@" > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python3 tools/prof_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
