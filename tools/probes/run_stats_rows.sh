#!/bin/bash
# strided-stats rows-per-block sweep: GEMMUL8_STATS_ROWS in {4,8,16} at several sizes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for s in 1024 2048 4096 8192; do for r in 4 8 16; do
  GEMMUL8_STATS_ROWS=$r timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/sr_${s}_$r -o run -- python3 tools/prof_driver.py --size $s --calls 10 > /dev/null 2>&1 || exit 1
  echo "size $s rows $r"; python3 tools/probes/kstats.py gpurun_out/sr_${s}_$r/run_kernel_stats.csv stats
done; done
