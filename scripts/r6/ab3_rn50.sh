#!/bin/bash
# Interleaved ResNet-50: abx/base, abx/varA, head.
O=gpurun_out/r6/ab3
mkdir -p $O
for r in 1 2 3; do
  for arm in base varA head; do
    if [ $arm = head ]; then B=bench.py; else B=abx/$arm/bench.py; fi
    timeout -k 10 300 python $B --steps 20 --warmup 5 > $O/${arm}_$r.log 2>&1 || { tail -5 $O/${arm}_$r.log; exit 1; }
    echo "round $r $arm $(tail -1 $O/${arm}_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a $O/summary.txt
  done
done
