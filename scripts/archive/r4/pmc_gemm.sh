#!/bin/bash
# PMC passes of the GEMM kernels on the BERT shapes: 128x128 forward (FFN1), 256x256 ping-pong at 8192^3 and
# at FFN1, and the split-K weight gradient (RC x RC, fp32) of FFN1.  One pass per counter group.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4/pmc_gemm; rm -rf $O; mkdir -p $O
run() {  # name, args
  local n=$1; shift
  local W="python3 $R/scripts/gemm_one.py $*"
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/$n/trace -- $W > $O/$n.log 2>&1 || return 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES --output-format csv -d $O/$n/p1 -- $W >> $O/$n.log 2>&1 || return 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/$n/p2 -- $W >> $O/$n.log 2>&1 || return 1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/$n/p3 -- $W >> $O/$n.log 2>&1 || return 1
  (cd $R && python scripts/pmc_table.py $(find $O/$n/trace -name "*kernel_trace.csv" | head -1) $(find $O/$n/p1 $O/$n/p2 $O/$n/p3 -name "*counter_collection.csv") > $O/$n.txt 2>&1)
  head -3 $O/$n.txt
}
run ffn1_t128 16384 3072 768 0 0 5 0 bf16 && \
run sq8k_g256 8192 8192 8192 0 0 3 4 bf16 && \
run ffn1_g256 16384 3072 768 0 0 5 4 bf16 && \
run ffn1_wgrad 3072 768 16384 1 1 5 auto f32
