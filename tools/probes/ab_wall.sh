#!/bin/bash
# Same-box A/B of an environment switch on bench.py's wall time per call: ab_wall.sh VAR "v1 v2" "sizes" [reps]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
VAR=$1; VALS=$2; SIZES=${3:-8192}; REPS=${4:-1}
for r in $(seq $REPS); do for s in $SIZES; do for v in $VALS; do
  out=$(env $VAR=$v timeout -k 10 120 python3 bench.py --size $s --steps 50 --warmup 5 --no-cpu-baseline --no-accuracy --no-dgemm 2>/dev/null) || exit 1
  echo "size $s $VAR=$v $(echo "$out" | grep -o '"ms_per_step": [0-9.]*') $(echo "$out" | grep -o '"phase_ms": {[^}]*}')"
done; done; done
