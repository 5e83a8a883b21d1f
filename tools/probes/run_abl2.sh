#!/bin/bash
# energy split of the product kernel: full / no LDS reads in the loop / no LDS-DMA in the loop
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for a in 0 5 6 0 5 6; do
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES TD_TD_BUSY_sum -f csv -d gpurun_out/abl2_$a -o run -- tools/probes/abl_$a 14 rand > gpurun_out/abl2_$a.log 2>&1 || exit 1
  echo "ablate=$a"; python3 tools/clock_of.py gpurun_out/abl2_$a/run_counter_collection.csv | grep -A1 gemm_i8
done
