#!/bin/bash
# Register cap of the bf16-output LDS-DMA GEMM (DDL_DMA_BF16_MIN_BLOCKS = 4 default / 3 / 2, built as
# _C.so / _C_mb3.so / _C_mb2.so): GEMM micro on the BERT shapes and interleaved BERT-base / ResNet-50 steps.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4/mb
P=distributeddeeplearningspark_amd
cp $P/_C.so $P/_C_mb4.so
fatal() { case $1 in 124|134|137|139) echo "[mb_ab] fatal rc=$1 in $2"; cp $P/_C_mb4.so $P/_C.so; exit $1;; esac; }
: > gpurun_out/r4/mb/steps.txt
for v in 4 3 2; do
  cp $P/_C_mb$v.so $P/_C.so
  DDL_GEMM_FULL_EPI=1 timeout -k 10 300 python scripts/bench_gemm.py bert_qkv_fwd,bert_ffn1_fwd,bert_ffn2_fwd,bert_ffn1_dgrad,bert_ffn2_dgrad > gpurun_out/r4/mb/gemm_$v.jsonl 2>&1; fatal $? gemm
  python - $v <<'PY'
import json, sys
for l in open(f"gpurun_out/r4/mb/gemm_{sys.argv[1]}.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print("minblocks", sys.argv[1], d["shape"], {k: d[k]["tflops"] for k in ("t128", "g256") if k in d})
PY
done
for i in 1 2; do
  for v in 4 3 2; do
    cp $P/_C_mb$v.so $P/_C.so
    timeout -k 10 240 python bench.py --model bert --steps 10 --warmup 3 2>/dev/null | grep '^{' | sed "s/^/bert mb=$v /" >> gpurun_out/r4/mb/steps.txt; fatal $? bert
  done
done
for v in 4 3; do
  cp $P/_C_mb$v.so $P/_C.so
  timeout -k 10 240 python bench.py --steps 15 --warmup 4 2>/dev/null | grep '^{' | sed "s/^/rn50 mb=$v /" >> gpurun_out/r4/mb/steps.txt; fatal $? rn50
done
cp $P/_C_mb4.so $P/_C.so
python - <<'PY'
import json
for line in open("gpurun_out/r4/mb/steps.txt"):
    a, b, js = line.split(" ", 2); d = json.loads(js); print(a, b, round(d["value"]), d["ms_per_step"])
PY
