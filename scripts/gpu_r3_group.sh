#!/bin/bash
# Grouped tile raster of the LDS-DMA GEMM (DDL_GEMM_GROUP_M): GEMM microbench + BERT / ResNet A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "gemm_layouts or splitk or conv_fwd_bwd" > gpurun_out/grp_tests.log 2>&1
rc=$?; tail -1 gpurun_out/grp_tests.log; [ $rc -ne 0 ] && exit $rc
DDL_GEMM_GROUP_M=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "gemm_layouts or splitk or conv_fwd_bwd" > gpurun_out/grp_tests8.log 2>&1
rc=$?; tail -1 gpurun_out/grp_tests8.log; [ $rc -ne 0 ] && exit $rc
for g in 0 8 16 4; do
  DDL_GEMM_GROUP_M=$g timeout -k 10 200 python scripts/bench_gemm.py > gpurun_out/grp_gemm_$g.jsonl 2>&1 || { tail gpurun_out/grp_gemm_$g.jsonl; exit 1; }
  echo "G=$g $(grep '^{' gpurun_out/grp_gemm_$g.jsonl | python -c '
import json,sys
print(" ".join(f"{d[\"shape\"][:14]}:{d[\"t128\"][\"tflops\"]}" for d in map(json.loads, sys.stdin) if "bert" in d["shape"] or "rn50_l3" in d["shape"]))')"
done
OUT=gpurun_out/ab_group.jsonl; : > $OUT
for r in 1 2; do
  for g in 8 0; do
    for m in bert resnet50; do
      DDL_GEMM_GROUP_M=$g timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 3 > gpurun_out/ab_tmp.log 2>&1 || { tail gpurun_out/ab_tmp.log; exit 1; }
      line=$(grep '^{' gpurun_out/ab_tmp.log | tail -1)
      echo "{\"round\": $r, \"model\": \"$m\", \"DDL_GEMM_GROUP_M\": $g, \"bench\": $line}" >> $OUT
      echo "r$r $m G=$g $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
    done
  done
done
