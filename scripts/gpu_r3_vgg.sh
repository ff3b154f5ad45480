#!/bin/bash
# Fused conv+BN(+ReLU) node for Sequential models: tests + interleaved VGG-16 A/B (+ host overhead probe)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_layers.py tests/test_gpu_ddp.py > gpurun_out/vgg_tests.log 2>&1
rc=$?; tail -1 gpurun_out/vgg_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/vgg_tests.log | head; exit $rc; }
OUT=gpurun_out/ab_fuse_convbn.jsonl; : > $OUT
for r in 1 2 3; do
  for v in 1 0; do
    DDL_FUSE_CONVBN=$v timeout -k 10 300 python bench.py --model vgg16 --steps 30 --warmup 5 > gpurun_out/ab_tmp.log 2>&1 || { tail gpurun_out/ab_tmp.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_tmp.log | tail -1)
    echo "{\"round\": $r, \"DDL_FUSE_CONVBN\": \"$v\", \"bench\": $line}" >> $OUT
    echo "r$r fuse=$v $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
if [ -f scripts/cpu_overhead.py ]; then
  for v in 1 0; do DDL_FUSE_CONVBN=$v timeout -k 10 200 python scripts/cpu_overhead.py --model vgg16 > gpurun_out/vgg_host_$v.txt 2>&1; head -3 gpurun_out/vgg_host_$v.txt | grep -i "host\|wall" ; done
fi
