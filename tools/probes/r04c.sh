set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04c; mkdir -p $OUT
timeout -k 10 120 tools/probes/kara_stream_probe > $OUT/kara_stream.txt 2>&1 || exit 1
cat $OUT/kara_stream.txt
timeout -k 10 400 python tools/probes/shard_time.py 16384 14 8 > $OUT/shard_moduli.txt 2>&1 || exit 1
grep -v "^ " $OUT/shard_moduli.txt
SHARD_ORDER=columns timeout -k 10 400 python tools/probes/shard_time.py 16384 14 8 4 > $OUT/shard_columns.txt 2>&1 || exit 1
grep -v "^ " $OUT/shard_columns.txt
