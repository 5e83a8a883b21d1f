# no-exchange partition per-rank times; live reference sweeps on this round's build (accurate-mode magnitudes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04i; mkdir -p $OUT
timeout -k 10 300 python tools/probes/block_time.py > $OUT/block_time.txt 2>&1 || exit 1
cat $OUT/block_time.txt
FUZZ_EXTREME=1 FUZZ_AB=general FUZZ_OUT=r04i_fuzz_extreme.json timeout -k 10 400 python tools/probes/fuzz_ref.py 1000 401 > $OUT/fuzz_extreme.txt 2>&1 || { tail -5 $OUT/fuzz_extreme.txt; exit 1; }
tail -1 $OUT/fuzz_extreme.txt
FUZZ_LD=1 FUZZ_AB=general FUZZ_OUT=r04i_fuzz_ld.json timeout -k 10 400 python tools/probes/fuzz_ref.py 600 402 > $OUT/fuzz_ld.txt 2>&1 || { tail -5 $OUT/fuzz_ld.txt; exit 1; }
tail -1 $OUT/fuzz_ld.txt
FUZZ_OUT=r04i_fuzz_big.json timeout -k 10 500 python tools/probes/fuzz_ref.py 150 403 1000:3200 500:6000 > $OUT/fuzz_big.txt 2>&1 || { tail -5 $OUT/fuzz_big.txt; exit 1; }
tail -1 $OUT/fuzz_big.txt
