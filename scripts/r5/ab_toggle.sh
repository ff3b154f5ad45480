#!/bin/bash
# Same-box interleaved A/B of bench.py against a module-level switch of this tree:
#   SWITCH="distributeddeeplearningspark_amd.ops.conv:_CLASS_BATCH=False" ROUNDS=3 TAG=name bash scripts/r5/ab_toggle.sh
# arm "off" runs bench.py with the switch applied before it starts, arm "on" runs it unchanged.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5/${TAG:-ab_toggle}
mkdir -p $O
MOD=${SWITCH%%:*}
ASSIGN=${SWITCH#*:}
for r in $(seq 1 ${ROUNDS:-3}); do
  for arm in off on; do
    if [ $arm = off ]; then
      timeout -k 10 300 python -c "import sys, runpy, importlib; sys.argv = ['bench.py'] + '${ARGS:---steps 20 --warmup 5}'.split(); m = importlib.import_module('$MOD'); setattr(m, '${ASSIGN%%=*}', ${ASSIGN#*=}); runpy.run_path('bench.py', run_name='__main__')" > $O/${arm}_$r.log 2>&1 || { tail -20 $O/${arm}_$r.log; exit 1; }
    else
      timeout -k 10 300 python bench.py ${ARGS:---steps 20 --warmup 5} > $O/${arm}_$r.log 2>&1 || { tail -20 $O/${arm}_$r.log; exit 1; }
    fi
    v=$(tail -1 $O/${arm}_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
    echo "round $r $arm $v" | tee -a $O/summary.txt
  done
done
