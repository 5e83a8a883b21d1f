#!/bin/bash
# Same-box A/B of an environment switch on the library kernels: ab_env.sh VAR "v1 v2" "sizes" [reps]
# (prof_driver.py calls under rocprofv3 --kernel-trace --stats; prints each library kernel's mean)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
VAR=$1; VALS=$2; SIZES=${3:-8192}; REPS=${4:-1}
for r in $(seq $REPS); do for s in $SIZES; do for v in $VALS; do
  env $VAR=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/abe_${s}_$v -o run -- python3 tools/prof_driver.py --size $s --calls 10 > /dev/null 2>&1 || exit 1
  echo "size $s $VAR=$v"; python3 tools/probes/kstats.py gpurun_out/abe_${s}_$v/run_kernel_stats.csv
done; done; done
