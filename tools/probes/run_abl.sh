#!/bin/bash
# cycles of the plain GEMM kernel under ablations (0 full, 1 no LDS-DMA, 2 no MFMA, 3 no LDS reads)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for a in 0 1 2 3; do for d in rand const; do
  OZ2_GEMM_VARIANT=1 timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -f csv -d gpurun_out/abl_${a}_$d -o run -- tools/probes/abl_$a 14 $d > gpurun_out/abl_${a}_$d.log 2>&1 || exit 1
  echo "ablate=$a $d"; python3 tools/clock_of.py gpurun_out/abl_${a}_$d/run_counter_collection.csv | grep gemm
done; done
