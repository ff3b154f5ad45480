#!/bin/bash
# Launches and ATen call sites per training step at HEAD: ResNet-50 and VGG-16 (bench.py configs).
# Kernel traces of 5 steps (2 warmup + 3 timed) summarised by trace_busy.py, then deleted.
export TMPDIR=/tmp
O=gpurun_out/r5/launches
mkdir -p $O
timeout -k 10 200 python scripts/r5/resnet_ops.py > $O/resnet50_aten_sites.txt 2>&1 || exit 1
MODEL=vgg16 timeout -k 10 200 python scripts/r5/resnet_ops.py > $O/vgg16_aten_sites.txt 2>&1 || exit 1
for m in resnet50 vgg16; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o $m -- \
    python bench.py --model $m --steps 3 --warmup 2 > $O/prof_$m.log 2>&1 || exit 1
  python scripts/r5/trace_busy.py $(find $O/prof_$m -name '*kernel_trace.csv') 80 > $O/${m}_busy.txt || exit 1
  find $O/prof_$m -type f ! -name '*kernel_stats.csv' -delete
done
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --model vgg16 > $O/vgg16_bench_$i.log 2>&1 || exit 1
  tail -1 $O/vgg16_bench_$i.log | cut -c1-120
done
