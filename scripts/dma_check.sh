#!/bin/bash
# LDS-DMA GEMM kernel check: kernel tests under each DDL_GEMM_DMA mode, then the 3x3 conv
# microbench kernel stats and the ResNet-50 bench per mode.  Stops at the first crash.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
for m in 1 2; do
  DDL_GEMM_DMA=$m timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_gemm256.py tests/test_gpu_transformer.py -x -q > gpurun_out/dma_tests_$m.log 2>&1
  rc=$?; echo "mode $m tests rc=$rc: $(tail -1 gpurun_out/dma_tests_$m.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for m in 0 1 2; do
  (cd /tmp && DDL_GEMM_DMA=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/dstat$m -- python3 $R/scripts/bench_conv3x3.py > $R/gpurun_out/dstat$m.log 2>&1) || exit $?
  DDL_GEMM_DMA=$m timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/dbench$m.log 2>&1 || exit $?
  echo "mode $m: $(tail -1 gpurun_out/dbench$m.log | cut -c1-150)"
done
