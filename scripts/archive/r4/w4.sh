#!/bin/bash
# Four-wave 256-row GEMM (ddl_gemm_w4.h): correctness on every layout / epilogue, then the BERT /
# ResNet shape micro-benchmark against the 128x128 kernel, the 256x256 ping-pong and hipBLASLt.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm256.py -q --timeout 120 --timeout-method thread > gpurun_out/r4/w4_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4/w4_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
S=bert_qkv_fwd,bert_ffn1_fwd,bert_ffn2_fwd,bert_ffn1_dgrad,bert_ffn2_dgrad,square_8192,square_4096,rn50_l3_1x1_1024to256,rn50_l3_1x1_256to1024,bert_qkv_wgrad,bert_ffn1_wgrad
timeout -k 10 400 python scripts/bench_gemm.py $S > gpurun_out/r4/w4_micro.jsonl 2>&1 || { tail -20 gpurun_out/r4/w4_micro.jsonl; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r4/w4_micro.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["shape"], {k: d[k]["tflops"] for k in d if isinstance(d[k], dict)})
PY
