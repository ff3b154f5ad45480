#!/bin/bash
# Re-test the gathered-GEMM ring depth now that the tap tables live in LDS (DDL_GATHER_STAGES
# 1 / 3, interleaved), and list the ATen ops left in the VGG-16 / ResNet-50 steps.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/knobs; mkdir -p $O
for r in 1 2; do
  for st in 0 3; do
    for m in resnet50 vgg16; do
      DDL_GATHER_STAGES=$st timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > $O/${m}_st${st}_$r.log 2>&1 || { tail $O/${m}_st${st}_$r.log; exit 1; }
      echo "$m st=$st r=$r $(tail -1 $O/${m}_st${st}_$r.log | grep -o '"value": [0-9.]*')"
    done
  done
done
timeout -k 10 300 python scripts/aten_sites.py --model vgg16 > $O/aten_vgg16.txt 2>&1 || { tail $O/aten_vgg16.txt; exit 1; }
timeout -k 10 300 python scripts/aten_sites.py --model resnet50 > $O/aten_resnet50.txt 2>&1 || { tail $O/aten_resnet50.txt; exit 1; }
head -30 $O/aten_vgg16.txt
head -30 $O/aten_resnet50.txt
SHAPES=vgg16 timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/vgg_layers.json 2> $O/vgg_layers.err || { tail $O/vgg_layers.err; exit 1; }
cat $O/vgg_layers.err | cut -c1-400
