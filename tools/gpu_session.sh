#!/bin/bash
# One gpurun session of checks: usage tools/gpu_session.sh <tag> <step>...
#   steps: tests=<pytest args>   golden_cfg1   bench=<bench args>   gloo2|gloo4|gloo8=<bench args>
#          profile=<tag + bench args>   cmd=<shell command>
# Every GPU step runs under its own time limit; the first failure ends the session.
set -o pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for step in "$@"; do
  i=$((i+1))
  name=${step%%=*}
  arg=${step#*=}
  [ "$arg" = "$step" ] && arg=""
  echo "[$(date +%T)] step $i: $name $arg"
  case $name in
    tests)
      timeout -k 10 900 python -u -m pytest $arg -x -v --timeout 150 --timeout-method thread > $OUT/pytest_$i.log 2>&1
      rc=$?; tail -3 $OUT/pytest_$i.log ;;
    golden_cfg1)
      timeout -k 10 120 python tests/golden/make_golden_cfg1.py $OUT/golden_cfg1 > $OUT/golden_cfg1.log 2>&1
      rc=$?; tail -2 $OUT/golden_cfg1.log ;;
    bench)
      timeout -k 10 600 python bench.py $arg > $OUT/bench_$i.json 2> $OUT/bench_$i.err
      rc=$?; cat $OUT/bench_$i.json ;;
    gloo2)
      GEMMUL8_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 $arg > $OUT/gloo2_$i.json 2> $OUT/gloo2_$i.err
      rc=$?; cat $OUT/gloo2_$i.json ;;
    gloo4)
      GEMMUL8_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 4 $arg > $OUT/gloo4_$i.json 2> $OUT/gloo4_$i.err
      rc=$?; cat $OUT/gloo4_$i.json ;;
    gloo8)
      # the driver's 8-rank bench rehearsed on one GPU (gloo, ranks sharing the device; timing meaningless)
      GEMMUL8_BENCH_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 8 $arg > $OUT/gloo8_$i.json 2> $OUT/gloo8_$i.err
      rc=$?; cat $OUT/gloo8_$i.json ;;
    profile)
      timeout -k 10 900 bash tools/profile.sh $arg > $OUT/profile_$i.log 2>&1
      rc=$?; tail -5 $OUT/profile_$i.log ;;
    cmd)
      timeout -k 10 600 bash -c "$arg" > $OUT/cmd_$i.log 2>&1
      rc=$?; tail -20 $OUT/cmd_$i.log ;;
    *) echo "unknown step $name"; rc=2 ;;
  esac
  echo "[$(date +%T)] step $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
