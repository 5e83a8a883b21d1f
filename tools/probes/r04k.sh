# NCCL-branch tests (incl. the short soak) + a long soak through tests/dist_soak.py + cfg4 / cfg5 kernel traces
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04k; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_streams.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u tools/probes/fake_nccl_soak.py 500 12 > $OUT/soak_500_seed12.txt 2>&1; rc=$?; tail -2 $OUT/soak_500_seed12.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import sys; sys.path[:0] = ['tests', 'mixed-gemmul8_amd']; from dist_soak import soak; n, f = soak(40, 2024); print('seed 2024, 40 cases:', n, 'failures', f[:2]); sys.exit(1 if n else 0)" > $OUT/soak_40_seed2024.txt 2>&1; rc=$?; tail -1 $OUT/soak_40_seed2024.txt; [ $rc -ne 0 ] && exit $rc
bash tools/cfg_prof.sh
