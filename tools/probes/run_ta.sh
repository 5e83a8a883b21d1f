#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for grp in "GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" "GRBM_GUI_ACTIVE TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum" "GRBM_GUI_ACTIVE TA_BUFFER_READ_LDS_WAVEFRONTS_sum TA_FLAT_READ_LDS_WAVEFRONTS_sum TA_TOTAL_WAVEFRONTS_sum"; do
  i=$((i+1))
  for v in 1 2; do
    OZ2_GEMM_VARIANT=$v timeout -k 10 120 rocprofv3 --pmc $grp -f csv -d gpurun_out/ta_${v}_$i -o run -- tools/probes/var_probe 14 rand > gpurun_out/ta_${v}_$i.log 2>&1 || exit 1
    echo "variant=$v pass=$i"; python3 tools/clock_of.py gpurun_out/ta_${v}_$i/run_counter_collection.csv | grep -A8 gemm_i8
  done
done
