#!/bin/bash
# Final evidence at HEAD on one box: BERT-base x3, VGG-16 x3 (the ResNet-50 x3 runs are in suite.sh).
set -o pipefail
O=gpurun_out/r6/final
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --model bert > $O/bert_$i.json 2> $O/bert_$i.err || exit 1
  timeout -k 10 200 python -u bench.py --model vgg16 --steps 50 --warmup 10 > $O/vgg_$i.json 2> $O/vgg_$i.err || exit 1
done
for f in $O/bert_*.json $O/vgg_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'])"; done
