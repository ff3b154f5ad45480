#!/bin/bash
# PMC pass over the lab variants on one shape: scripts/gemm_lab/pmc.sh M N K EPI
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/labpmc
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
  SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -- \
  $R/scripts/gemm_lab/lab $1 $2 $3 $4 1 > $O/p1.log 2>&1 || exit $?
python3 $R/scripts/gemm_lab/pmc_sum.py $(find $O/p1 -name "*counter_collection.csv" | head -1) > $O/pmc_$1_$2_$3_$4.txt
cat $O/pmc_$1_$2_$3_$4.txt
rm -rf $O/p1
