#!/bin/bash
# halo conv variants on the ResNet-50 3x3 layers (per-layer table), one process per variant
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/exp3; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "conv3x3_halo or conv_fwd" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in "def|" "bn64|DDL_CONV3X3_BN=64" "c64|DDL_CONV3X3_C64=1" "off|DDL_CONV3X3=0"; do
  tag=${v%%|*}; envs=${v#*|}
  env $envs timeout -k 10 300 python scripts/bench_resnet_layers.py > $O/layers_$tag.json 2>$O/layers_$tag.err || exit 1
  python - $O/layers_$tag.json $tag <<'PY'
import json, sys
d=json.load(open(sys.argv[1])); print(sys.argv[2], d['total_ms_per_step'])
for r in d['layers']:
    if r['k']==3 and r['stride']==1: print('  ', r['H'], r['Ci'], {k: r[k]['ms'] for k in ('fwd','dgrad')})
PY
done
