#!/bin/bash
# wgrad halo kernel with two-tap-deep B prefetch: tests + microbench + ResNet bench; then the GEMM PMC passes
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "wgrad_halo or resnet50_step" > gpurun_out/wg3c_tests.log 2>&1
rc=$?; tail -1 gpurun_out/wg3c_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/wg3c_tests.log | head; exit $rc; }
timeout -k 10 300 python scripts/bench_wgrad3.py > gpurun_out/wg3c_micro.jsonl 2>&1 || { tail gpurun_out/wg3c_micro.jsonl; exit 1; }
grep '^{' gpurun_out/wg3c_micro.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['H'], {k: d[k]['ms'] for k in ('pp_slab','slab','gemm')})"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/ab_tmp.log 2>&1 || { tail gpurun_out/ab_tmp.log; exit 1; }
  grep '^{' gpurun_out/ab_tmp.log | python -c 'import json,sys; d=json.load(sys.stdin); print("resnet50", d["value"], d["ms_per_step"])'
done
bash scripts/gpu_r3_pmc_gemm.sh
