#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do for o in 0 1 2; do
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES TD_TD_BUSY_sum -f csv -d gpurun_out/ord_$o -o run -- tools/probes/ord_$o 14 rand > gpurun_out/ord_$o.log 2>&1 || exit 1
  echo "order $o"; python3 tools/clock_of.py gpurun_out/ord_$o/run_counter_collection.csv | grep gemm_i8
done; done
