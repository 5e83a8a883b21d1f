# accurate-mode one-read magnitudes: parity (oracle + live reference), A/B on cfg4; complex CRT stream probe;
# shard replays of the two unit orders
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04d; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_parity.py tests/test_gpu_phases.py tests/test_gpu_streams.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
GEMMUL8_ONE_READ_MAGNITUDES=0 timeout -k 10 300 python bench.py --workload cfg4 --no-cpu-baseline > $OUT/cfg4_off_$i.json 2>$OUT/cfg4_off_$i.err || exit 1
timeout -k 10 300 python bench.py --workload cfg4 --no-cpu-baseline > $OUT/cfg4_on_$i.json 2>$OUT/cfg4_on_$i.err || exit 1
python -c "
import json
for t in ('off','on'):
    d=json.load(open('$OUT/cfg4_%s_$i.json'%t)); print(t, d['value'], d['ms_per_step'], d['phase_ms'], d['relerr_max'] if 'relerr_max' in d else '')"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py --workload cfg4 --no-cpu-baseline --steps 10 > $OUT/cfg4_prof.json 2> $OUT/trace.log || exit 1
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/cfg4_kernel_stats.csv
cut -c1-160 $OUT/cfg4_kernel_stats.csv | head -20
timeout -k 10 120 tools/probes/kara_stream_probe > $OUT/kara_stream.txt 2>&1 || exit 1
cat $OUT/kara_stream.txt
timeout -k 10 400 python tools/probes/shard_time.py 16384 14 8 > $OUT/shard_moduli.txt 2>&1 || exit 1
grep -v "^ " $OUT/shard_moduli.txt
SHARD_ORDER=columns timeout -k 10 400 python tools/probes/shard_time.py 16384 14 8 4 > $OUT/shard_columns.txt 2>&1 || exit 1
grep -v "^ " $OUT/shard_columns.txt
for i in 1 2; do
timeout -k 10 300 python bench.py --workload cfg5 --no-cpu-baseline > $OUT/cfg5_base_$i.json 2>$OUT/cfg5_base_$i.err || exit 1
GEMMUL8_KARA_TILE_ORDER=1 timeout -k 10 300 python bench.py --workload cfg5 --no-cpu-baseline > $OUT/cfg5_tile_$i.json 2>$OUT/cfg5_tile_$i.err || exit 1
python -c "
import json
for t in ('base','tile'):
    d=json.load(open('$OUT/cfg5_%s_$i.json'%t)); print(t, d['value'], d['ms_per_step'], d['phase_ms'])"
done
