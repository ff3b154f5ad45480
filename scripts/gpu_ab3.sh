#!/bin/bash
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/ab3; mkdir -p $O
run() { # name env... -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py $BARGS > $O/$name.log 2>&1 || { tail -3 $O/$name.log; return 1; }
  echo "$name $(tail -1 $O/$name.log | grep -o '"value": [0-9.]*')"
}
BARGS="--model bert --steps 10 --warmup 3"
run bert_def DDL_X=1 && run bert_st1 DDL_WGRAD_STAGES=1 && run bert_def2 DDL_X=1 || exit 1
BARGS="--model vgg16 --steps 30 --warmup 5"
run vgg_def DDL_X=1 && run vgg_nosplit DDL_CONV_SPLITK=0 && run vgg_def2 DDL_X=1 || exit 1
BARGS="--steps 20 --warmup 5"
run rn_def DDL_X=1 && run rn_st1 DDL_WGRAD_STAGES=1 || exit 1
