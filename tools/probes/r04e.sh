# accurate-mode one-read magnitudes v2 (parallel fixup): parity + cfg4 A/B + kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${R04TAG:-r04e}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_parity.py tests/test_gpu_phases.py -x -q --timeout 300 --timeout-method thread -k "accurate or nonfinite or extreme or mixed or same_inputs or zero or shards or rank" > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
GEMMUL8_ONE_READ_MAGNITUDES=0 timeout -k 10 300 python bench.py --workload cfg4 --no-cpu-baseline > $OUT/cfg4_off_$i.json 2>$OUT/cfg4_off_$i.err || exit 1
timeout -k 10 300 python bench.py --workload cfg4 --no-cpu-baseline > $OUT/cfg4_on_$i.json 2>$OUT/cfg4_on_$i.err || exit 1
python -c "
import json
for t in ('off','on'):
    d=json.load(open('$OUT/cfg4_%s_$i.json'%t)); print(t, d['value'], d['ms_per_step'], d['phase_ms'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py --workload cfg4 --no-cpu-baseline --steps 10 > $OUT/cfg4_prof.json 2> $OUT/trace.log || exit 1
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/cfg4_kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/cfg4_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1))"
