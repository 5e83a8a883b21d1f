cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/small
for s in 1024 2048 4096; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/small/t$s -o run -- python3 bench.py --size $s --steps 50 --warmup 5 --no-cpu-baseline --no-accuracy --no-dgemm > gpurun_out/small/b$s.json 2> gpurun_out/small/b$s.err || exit 1
done
