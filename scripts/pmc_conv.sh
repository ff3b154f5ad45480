#!/bin/bash
# PMC counters + kernel stats for the 3x3 convolution kernels (counter runs separate from traces).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/cstat -- python3 $R/scripts/bench_conv3x3.py > $R/gpurun_out/cstat.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  --output-format csv -d $R/gpurun_out/cpmc1 -- python3 $R/scripts/bench_conv3x3.py > $R/gpurun_out/cpmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM \
  --output-format csv -d $R/gpurun_out/cpmc2 -- python3 $R/scripts/bench_conv3x3.py > $R/gpurun_out/cpmc2.log 2>&1 || exit $?
find $R/gpurun_out/cstat $R/gpurun_out/cpmc1 $R/gpurun_out/cpmc2 -name "*.csv" | head -20
