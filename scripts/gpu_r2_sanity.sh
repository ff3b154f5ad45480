#!/bin/bash
# Fresh-box sanity of the restored tree: GPU tests, headline bench, per-layer conv table with the
# single-stage (default) and the two-stage LDS-DMA GEMM.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/sanity; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/layers_dma1.json 2> $O/layers_dma1.err || { tail $O/layers_dma1.err; exit 1; }
DDL_GEMM_DMA=2 timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/layers_dma2.json 2> $O/layers_dma2.err || { tail $O/layers_dma2.err; exit 1; }
exit 0
