#!/bin/bash
# GEMM evidence at HEAD: microbenchmark (BERT / ResNet / square shapes), PMC counters of the BERT
# FFN1-forward and 8192^3 GEMMs (one rocprofv3 pass per counter group), ResNet-50 per-layer roofline.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5gemm
mkdir -p $O
cd $R
timeout -k 10 300 python3 scripts/bench_gemm.py > $O/gemm.jsonl 2> $O/gemm.err || exit $?
timeout -k 10 300 python3 scripts/bench_resnet_layers.py > $O/resnet50_layer_roofline.json 2> $O/roof.err || exit $?
cd /tmp
W="python3 $R/scripts/bench_gemm.py bert_ffn1_fwd,bert_ffn2_fwd,square_8192"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/stat -- $W > $O/stat.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES --output-format csv -d $O/p1 -- $W > $O/p1.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p2 -- $W > $O/p2.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU \
  --output-format csv -d $O/p3 -- $W > $O/p3.log 2>&1 || exit $?
cd $R
T=$(find $O/stat -name "*kernel_trace.csv" | head -1)
P1=$(find $O/p1 -name "*counter_collection.csv" | head -1)
P2=$(find $O/p2 -name "*counter_collection.csv" | head -1)
P3=$(find $O/p3 -name "*counter_collection.csv" | head -1)
python3 scripts/pmc_table.py $T $P1 $P2 $P3 > $O/pmc_table.txt 2>&1 || exit $?
rm -rf $O/stat $O/p1 $O/p2 $O/p3
