# live reference sweeps on the round's last build (Karatsuba CRT and N >= 15 CRT order changed): general cases,
# and large sizes where complex products take the Karatsuba form
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04m; mkdir -p $OUT
FUZZ_AB=general FUZZ_OUT=r04m_fuzz_general.json timeout -k 10 400 python tools/probes/fuzz_ref.py 1000 501 > $OUT/fuzz_general.txt 2>&1 || { tail -5 $OUT/fuzz_general.txt; exit 1; }
tail -1 $OUT/fuzz_general.txt
FUZZ_OUT=r04m_fuzz_big.json timeout -k 10 500 python tools/probes/fuzz_ref.py 150 502 1000:3200 3072:5000 > $OUT/fuzz_big.txt 2>&1 || { tail -5 $OUT/fuzz_big.txt; exit 1; }
tail -1 $OUT/fuzz_big.txt
