#!/bin/bash
# Persistent vs one-tile product kernel across sizes (bench.py products phase, one process per run).
for s in ${@:-1024 1536 2048 2560 3072}; do
  for mode in 0 1; do
    r=$(GEMMUL8_PERSISTENT=$mode timeout -k 10 120 python3 bench.py --size $s --steps 200 --warmup 10 --no-cpu-baseline --no-accuracy --no-dgemm) || exit 1
    echo "size $s persistent=$mode $(python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step']*1e3, 'us/step', d['phase_ms'])" "$r")"
  done
done
