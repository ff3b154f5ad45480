#!/bin/bash
# PMC counters for the attention kernels (two passes, counters only; no traces combined).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  --output-format csv -d $R/gpurun_out/pmc1 -- python3 $R/scripts/bench_attention.py > $R/gpurun_out/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE \
  --output-format csv -d $R/gpurun_out/pmc2 -- python3 $R/scripts/bench_attention.py > $R/gpurun_out/pmc2.log 2>&1 || exit $?
find $R/gpurun_out/pmc1 $R/gpurun_out/pmc2 -name "*counter_collection*" | head
