#!/bin/bash
# usage: run_var.sh "<variants>" [data] -- cycles/clock of the product kernel per variant
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in $1; do for d in ${2:-rand}; do
  OZ2_GEMM_VARIANT=$v timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES TD_TD_BUSY_sum -f csv -d gpurun_out/var_${v}_$d -o run -- tools/probes/var_probe 14 $d > gpurun_out/var_${v}_$d.log 2>&1 || exit 1
  echo "variant=$v $d"; python3 tools/clock_of.py gpurun_out/var_${v}_$d/run_counter_collection.csv | grep -A3 gemm_i8
done; done
