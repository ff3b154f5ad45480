#!/bin/bash
# round-5 call A: rnn kernel tests, NYISO timings, GEMM K sweep, hipBLASLt solution names, baselines
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rnn.py > $O/rnn_tests.log 2>&1 || { tail -20 $O/rnn_tests.log; exit 1; }
tail -2 $O/rnn_tests.log
timeout -k 10 300 python bench.py --model nyiso_gru > $O/nyiso_gru.log 2>&1 || { tail -20 $O/nyiso_gru.log; exit 1; }
tail -1 $O/nyiso_gru.log
timeout -k 10 300 python bench.py --model nyiso_lstm > $O/nyiso_lstm.log 2>&1 || { tail -20 $O/nyiso_lstm.log; exit 1; }
tail -1 $O/nyiso_lstm.log
DDL_BENCH_W4=0 timeout -k 10 300 python scripts/bench_gemm.py bert_ffn1_fwd,16384x3072x1536,16384x3072x3072,16384x3072x6144,bert_ffn2_fwd,16384x768x6144,bert_qkv_fwd,16384x768x768 > $O/ksweep.jsonl 2>&1 || { tail -20 $O/ksweep.jsonl; exit 1; }
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/hipblaslt -- python3 $GRAFT_REPO_ROOT/scripts/r5/hipblaslt_names.py > $GRAFT_REPO_ROOT/$O/hipblaslt.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/hipblaslt.log; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench0.log 2>&1 || { tail -20 $O/bench0.log; exit 1; }
tail -1 $O/bench0.log
timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > $O/bert0.log 2>&1 || { tail -20 $O/bert0.log; exit 1; }
tail -1 $O/bert0.log
