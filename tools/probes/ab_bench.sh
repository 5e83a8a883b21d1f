#!/bin/bash
# A/B of an environment switch on the bench, same box: ab_bench.sh VAR "v1 v2" [reps]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
VAR=$1; VALS=$2; REPS=${3:-2}
for r in $(seq $REPS); do for v in $VALS; do
  env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/ab_$v -o run -- python3 bench.py --no-cpu-baseline --no-accuracy --no-dgemm > gpurun_out/ab_$v.log 2>&1 || exit 1
  echo "$VAR=$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log)"
  python3 - gpurun_out/ab_$v/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    if any(w in n for w in ('stats', 'encode', 'crt', 'gemm_i8')):
        print('   %-58s %8.4f ms' % (n[:58], float(r['AverageNs']) / 1e6))
PY
done; done
