#!/bin/bash
# Profile the bench command on the GPU box.
#   1. rocprofv3 --kernel-trace --stats on `python3 bench.py <bench args>` (the same command the
#      driver times; its JSON line goes to bench.json);
#   2. one PMC pass per counter group (--pmc never combined with another tracing domain) on a
#      short bench run;
#   3. tools/prof_summary.py -> summary.txt + summary.json (per-kernel average duration, counters,
#      HBM-side bytes with the gfx950 FETCH_SIZE x2 correction).
# Outputs under gpurun_out/prof_<tag>/.  Usage: tools/profile.sh <tag> [bench args...]
set -e
TAG=${1:-r01}
shift || true
BENCH_ARGS="$@"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
# --no-cfg3-1gpu, --no-power: the N = 1 line's extra timing of cfg3's 16384^3 shape and its one-second power loop
# (after the timed region) would mix a second shape and ~160 extra launches into the per-kernel averages
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py --no-cfg3-1gpu --no-power $BENCH_ARGS \
  > $OUT/bench.json 2> $OUT/trace.log
PMC_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-accuracy --no-dgemm --no-cfg3-1gpu --no-power $BENCH_ARGS"
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -f csv -d $OUT/pmc$i -o run -- python3 bench.py $PMC_ARGS \
    > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python3 tools/prof_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
