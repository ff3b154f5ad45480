#!/bin/bash
# Round 3: interleaved A/B of env knobs on the headline benches in ONE box session.
#   AB_VAR=DDL_WGRAD_STREAM AB_VALUES="1 0" MODELS="resnet50 vgg16 bert" ROUNDS=2 bash scripts/gpu_r3_ab.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
VAR=${AB_VAR:-DDL_WGRAD_STREAM}
VALUES=${AB_VALUES:-"1 0"}
MODELS=${MODELS:-resnet50}
ROUNDS=${ROUNDS:-2}
OUT=gpurun_out/ab_${VAR}.jsonl
: > $OUT
for r in $(seq 1 $ROUNDS); do
  for m in $MODELS; do
    for v in $VALUES; do
      steps=20; [ "$m" = "bert" ] && steps=10
      env $VAR=$v timeout -k 10 300 python bench.py --model $m --steps $steps --warmup 3 > gpurun_out/ab_tmp.log 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "bench $m $VAR=$v failed rc=$rc"; tail -20 gpurun_out/ab_tmp.log; exit $rc; fi
      line=$(grep '^{' gpurun_out/ab_tmp.log | tail -1)
      echo "{\"round\": $r, \"model\": \"$m\", \"$VAR\": \"$v\", \"bench\": $line}" >> $OUT
      echo "r$r $m $VAR=$v $(echo $line | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
    done
  done
done
