#!/bin/bash
# All five reference drivers' CSVs (accuracy + time, d also watt) of the current build into $1 (tools/harness.py)
set -o pipefail
OUT=${1:-gpurun_out/harness}
mkdir -p $OUT
for t in d f dfd dff fC; do
  modes="accuracy_check flops_check"
  [ $t = d ] && modes="accuracy_check flops_check watt_check"
  timeout -k 10 600 python3 tools/harness.py $t $modes --out-dir $OUT > $OUT/log_$t.txt 2>&1 || { echo "harness $t failed"; tail -5 $OUT/log_$t.txt; exit 1; }
  echo "harness $t done"
done
