#!/bin/bash
# gemm256 correctness then microbenchmark; stop on crash/timeout.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_gemm256.py tests/test_gpu_rnn.py -x -q > gpurun_out/g256_tests.log 2>&1
rc=$?
tail -3 gpurun_out/g256_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1
brc=$?
cat gpurun_out/bench_gemm.log | grep shape
exit $brc
