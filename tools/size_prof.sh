#!/bin/bash
# Kernel traces of bench.py across sizes (DGEMM, N = 14, fast): per-kernel durations and the bench
# line per size, under gpurun_out/sizes/.  Usage: tools/size_prof.sh [sizes...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SIZES=${@:-"1024 1536 2048 3072 4096 6144"}
mkdir -p gpurun_out/sizes
for s in $SIZES; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/sizes/t$s -o run -- python3 bench.py --size $s --steps 50 --warmup 5 --no-cpu-baseline --no-accuracy > gpurun_out/sizes/b$s.json 2> gpurun_out/sizes/b$s.err || exit 1
  echo "size $s done"
done
