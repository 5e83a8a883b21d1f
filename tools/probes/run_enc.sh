#!/bin/bash
# VALU / memory counters of the split kernels (bench cfg2, short run)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for grp in "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES" "GRBM_GUI_ACTIVE SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64" "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM" "GRBM_GUI_ACTIVE SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -f csv -d gpurun_out/enc$i -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-accuracy --no-dgemm > gpurun_out/enc$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/enc$i.log; continue; }
  echo "pass $i"; python3 tools/clock_of.py gpurun_out/enc$i/run_counter_collection.csv | grep -v gemm_i8 | grep -A5 "encode\|stats\|crt"
done
