#!/bin/bash
# Same-box interleaved A/B of bench.py: arm "base" = abx/base (a prebuilt older tree), arm "head" = this tree.
#   ROUNDS=3 ARGS="--steps 20 --warmup 5" TAG=name bash scripts/r6/ab_tree.sh
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/${TAG:-ab}
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-3}); do
  for arm in base head; do
    if [ $arm = base ]; then B=abx/base/bench.py; else B=bench.py; fi
    timeout -k 10 300 python $B ${ARGS:---steps 20 --warmup 5} > $O/${arm}_$r.log 2>&1 || { tail -20 $O/${arm}_$r.log; exit 1; }
    v=$(tail -1 $O/${arm}_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
    echo "round $r $arm $v" | tee -a $O/summary.txt
  done
done
