#!/bin/bash
# Kernel traces of the other BASELINE configs (tools/prof_driver.py): cfg4 (d x s -> d 8192^3, N = 10,
# accurate) and cfg5 (complex 4096^3, N = 12, big-matrix encode type) -> gpurun_out/cfg/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cfg
for c in 4 5; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/cfg/t$c -o run -- python3 tools/prof_driver.py --cfg $c --calls 10 > gpurun_out/cfg/c$c.log 2>&1 || exit 1
  echo "cfg $c done"
done
