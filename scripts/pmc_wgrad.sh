#!/bin/bash
# PMC passes for the BERT FFN1 weight-gradient GEMM (RC x RC, fp32 split-K atomics)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_wgrad
mkdir -p $O
W="python3 $R/scripts/bench_wgrad.py ffn1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES --output-format csv -d $O/p1 -- $W > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p2 -- $W > $O/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE \
  --output-format csv -d $O/p3 -- $W > $O/p3.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stat -- $W > $O/stat.log 2>&1 || exit $?
find $O -name "*counter_collection.csv" | head
