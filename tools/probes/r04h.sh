# CRT high-weight split: full GPU suite on the in-tree build + library A/B (base vs split)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04h; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/probes/lib_ab.py tools/probes/ab/base tools/probes/ab/split > $OUT/lib_ab.txt 2>&1; rc=$?; cat $OUT/lib_ab.txt; [ $rc -ne 0 ] && exit $rc
GEMMUL8_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --size 4096 --steps 3 --warmup 1 > $OUT/gloo2.json 2> $OUT/gloo2.err; rc=$?; python -c "
import json; d=json.load(open('$OUT/gloo2.json')); print(d['variants'], d.get('single_gpu_ms'), d.get('strong_scaling_efficiency'))"; exit $rc
