#!/bin/bash
# Interleaved ResNet-50 runs with a module constant patched before bench.py starts:
#   MOD=distributeddeeplearningspark_amd.ops.gemm NAME=_TILE_FILL VALUES="1.0 2.0 3.0" bash scripts/r6/knob_sweep.sh
O=gpurun_out/r6/knob_${NAME}
mkdir -p $O
for r in 1 2 3; do
  for v in $VALUES; do
    timeout -k 10 300 python -c "import sys, runpy, importlib; sys.argv = ['bench.py'] + '${ARGS}'.split(); m = importlib.import_module('$MOD'); setattr(m, '$NAME', $v); runpy.run_path('bench.py', run_name='__main__')" > $O/run.json 2> $O/run.err || { tail -5 $O/run.err; exit 1; }
    echo "round $r $NAME=$v $(python3 -c "import json; d=json.load(open('$O/run.json')); print(d['value'], d['ms_per_step'])")" | tee -a $O/summary.txt
  done
done
