# Karatsuba CRT with the moduli outermost and the weights materialised at their use: complex GPU parity on the
# in-tree build, then library A/B (base = per-row chains, mod8 / mod4 = moduli outermost with 8 / 4 rows per lane, all = mod4 + the same order in the real CRT)
# The variants (not kept: build artefacts) were each a copy of mixed-gemmul8_amd/gemmul8/*.py under
# tools/probes/ab/<name>/gemmul8/ with libgemmul8_amd.so linked from the in-tree objects and crt.hip rebuilt as
#   hipcc -O3 -std=c++20 --offload-arch=gfx950 -fPIC -ffp-contract=off -DOCML_BASIC_ROUNDED_OPERATIONS <defines>
# base: -DOZ2_CRT_MODOUTER=0 -DOZ2_KARA_ROWS=8; mod8: -DOZ2_KARA_ROWS=8; mod4: -DOZ2_KARA_ROWS=4;
# all: -DOZ2_KARA_ROWS=4 -DOZ2_CRT_MODOUTER_ALL=1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04j; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_parity.py -m gpu -k "kara or complex or zgemm or same_inputs" -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/probes/lib_ab.py tools/probes/ab/base tools/probes/ab/mod8 tools/probes/ab/mod4 tools/probes/ab/all > $OUT/lib_ab.txt 2>&1; rc=$?; cat $OUT/lib_ab.txt; exit $rc
