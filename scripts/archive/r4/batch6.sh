#!/bin/bash
# Deterministic-mode cost (ResNet-50 / BERT-base, flag on vs off, interleaved), VGG-16 five-run spread,
# split-K slabs A/B on VGG-16 / ResNet-50.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "[batch6] fatal rc=$1 in $2"; exit $1;; esac; }
run() { local tag=$1; shift; env "$@" timeout -k 10 240 python bench.py $BARGS 2>/dev/null | grep '^{' | sed "s/^/$tag /" >> gpurun_out/r4/b6.txt; }
: > gpurun_out/r4/b6.txt
for i in 1 2; do
  BARGS="--steps 15 --warmup 4" run "rn50 det=0" DDL_DETERMINISTIC=0; fatal $? det
  BARGS="--steps 15 --warmup 4" run "rn50 det=1" DDL_DETERMINISTIC=1; fatal $? det
  BARGS="--model bert --steps 10 --warmup 3" run "bert det=0" DDL_DETERMINISTIC=0; fatal $? det
  BARGS="--model bert --steps 10 --warmup 3" run "bert det=1" DDL_DETERMINISTIC=1; fatal $? det
done
for i in 1 2 3 4 5; do
  BARGS="--model vgg16 --steps 30 --warmup 5" run "vgg slabs=0" DDL_SPLITK_SLABS=0; fatal $? vgg
  BARGS="--model vgg16 --steps 30 --warmup 5" run "vgg slabs=1" DDL_SPLITK_SLABS=1; fatal $? vgg
done
for i in 1 2; do
  BARGS="--steps 15 --warmup 4" run "rn50 slabs=auto" DDL_X=0; fatal $? rn50
  BARGS="--steps 15 --warmup 4" run "rn50 slabs=1" DDL_SPLITK_SLABS=1; fatal $? rn50
done
python - <<'PY'
import json
for line in open("gpurun_out/r4/b6.txt"):
    a, b, js = line.split(" ", 2); d = json.loads(js); print(a, b, round(d["value"]), d["ms_per_step"])
PY
exit 0
