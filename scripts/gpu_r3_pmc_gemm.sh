#!/bin/bash
# PMC passes of the 128x128 LDS-DMA GEMM on BERT FFN1 forward (16384 x 3072 x 768)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc_gemm; rm -rf $O; mkdir -p $O
W="python3 $R/scripts/gemm_one.py 16384 3072 768 0 0 10"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace -- $W > $O/trace.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES --output-format csv -d $O/p1 -- $W > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p2 -- $W > $O/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p3 -- $W > $O/p3.log 2>&1 || exit 1
cd $R
t=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python scripts/pmc_table.py $t $(find $O/p1 $O/p2 $O/p3 -name "*counter_collection.csv") > gpurun_out/pmc_gemm_table.txt 2>&1
head -4 gpurun_out/pmc_gemm_table.txt
grep -A3 "def main" scripts/pmc_table.py > /dev/null
