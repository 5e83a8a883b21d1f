#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do for i in 1 2 3 4 5; do
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES TD_TD_BUSY_sum -f csv -d gpurun_out/bits_$i -o run -- tools/probes/bits_$i 14 rand > gpurun_out/bits_$i.log 2>&1 || exit 1
  echo "bits variant $i"; python3 tools/clock_of.py gpurun_out/bits_$i/run_counter_collection.csv | grep -A1 gemm_i8
done; done
