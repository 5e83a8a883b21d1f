#!/bin/bash
# Kernel trace + PMC passes (one counter group per pass, --pmc never combined with other
# tracing domains) for the cfg2 call; outputs under gpurun_out/prof_<tag>/.
set -e
TAG=${1:-r01}
shift || true
ARGS="$@"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 tools/prof_driver.py $ARGS > $OUT/trace.log 2>&1
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -f csv -d $OUT/pmc$i -o run -- python3 tools/prof_driver.py $ARGS > $OUT/pmc$i.log 2>&1 || echo "pmc pass $i failed"
done
python3 tools/prof_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
