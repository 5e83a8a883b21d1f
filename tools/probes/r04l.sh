# Real / f32 / big-matrix complex CRT with the moduli outermost from N = 15 on: GPU parity on the in-tree build
# (mo15), then the CRT A/B across N (base: -DOZ2_CRT_MODOUTER_MIN_N=99, the rows innermost at every N; the
# variants are copies of gemmul8/*.py with the library linked from the in-tree objects and crt.hip rebuilt)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04l; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_phases.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/probes/crt_n_ab.py tools/probes/ab/base tools/probes/ab/mo15 > $OUT/crt_n_ab.txt 2>&1; rc=$?; cat $OUT/crt_n_ab.txt; exit $rc
