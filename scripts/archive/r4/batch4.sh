#!/bin/bash
# Big weight gradients on 128x128 tiles + split-K slabs (DDL_SPLITK_SLABS=auto, default) vs the previous
# atomics route: GEMM tests, the production wgrad micro, interleaved BERT A/B.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "[batch4] fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -k "wgrad or splitk or slabs or linear" --timeout 120 --timeout-method thread > gpurun_out/r4/b4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4/b4_tests.log; fatal $rc tests
for v in auto 0; do
  DDL_SPLITK_SLABS=$v timeout -k 10 300 python scripts/bench_gemm.py bert_qkv_wgrad,bert_ffn1_wgrad,bert_ffn2_wgrad,rn50_wgrad_1x1_1024to256 > gpurun_out/r4/b4_wgrad_$v.jsonl 2>&1; fatal $? micro
  python - $v <<'PY'
import json, sys
for l in open(f"gpurun_out/r4/b4_wgrad_{sys.argv[1]}.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print("slabs", sys.argv[1], d["shape"], {k: d[k]["tflops"] for k in d if isinstance(d[k], dict)})
PY
done
: > gpurun_out/r4/b4_bert_ab.txt
for i in 1 2; do
  for v in auto 0; do
    DDL_SPLITK_SLABS=$v timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 2>/dev/null | grep '^{' | sed "s/^/slabs=$v /" >> gpurun_out/r4/b4_bert_ab.txt; fatal $? bert
  done
done
python - <<'PY'
import json
for line in open("gpurun_out/r4/b4_bert_ab.txt"):
    tag, js = line.split(" ", 1); d = json.loads(js); print(tag, round(d["value"]), d["ms_per_step"])
PY
exit 0
