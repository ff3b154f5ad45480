#!/bin/bash
# End-of-round 2/2: BERT-base x2, VGG-16 x5, NYISO GRU / LSTM, MNIST 8 co-located workers.
export TMPDIR=/tmp
O=gpurun_out/r5/final
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > $O/bench_bert_$i.log 2>&1 || { tail -20 $O/bench_bert_$i.log; exit 1; }
  tail -1 $O/bench_bert_$i.log | cut -c1-130
done
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --model vgg16 > $O/bench_vgg16_$i.log 2>&1 || { tail -20 $O/bench_vgg16_$i.log; exit 1; }
  tail -1 $O/bench_vgg16_$i.log | cut -c1-130
done
for c in gru lstm; do
  timeout -k 10 300 python bench.py --model nyiso_$c > $O/bench_nyiso_$c.log 2>&1 || { tail -20 $O/bench_nyiso_$c.log; exit 1; }
  tail -1 $O/bench_nyiso_$c.log | cut -c1-200
done
cd examples && timeout -k 10 240 python -u ddl_mnist.py --executors 4 --processes 2 --epochs 5 --train-rows 60000 --test-rows 10000 --workers-per-gpu 8 > ../$O/mnist.log 2>&1 || { tail -20 ../$O/mnist.log; exit 1; }
grep "Training time\|Accuracy\|updates" ../$O/mnist.log
