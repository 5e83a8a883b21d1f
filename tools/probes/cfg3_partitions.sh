#!/bin/bash
# cfg3 (16384^3, N = 14, W = 8) per-rank replay of both partitions on one box, twice each, alternating (VERDICT r05
# item 5): gemm_moduli's (modulus, column block) units and gemm_moduli_grid's 2 x 4 unit grid; each run times the
# single-GPU call of the same shape in the same process (tools/probes/shard_time.py)
set -o pipefail
OUT=${1:-gpurun_out/cfg3_partitions}
mkdir -p $OUT
for rep in 1 2; do
  timeout -k 10 240 python3 tools/probes/shard_time.py 16384 14 8 > $OUT/moduli_$rep.txt 2>&1 || exit 1
  timeout -k 10 240 env SHARD_GRID=2 python3 tools/probes/shard_time.py 16384 14 8 > $OUT/grid_$rep.txt 2>&1 || exit 1
done
grep -h 'single GPU\|W=8' $OUT/*.txt
