#!/bin/bash
# Four-wave 256-row GEMM (ddl_gemm_w4.h): correctness on every layout / epilogue, then the BERT /
# ResNet shape micro-benchmark against the 128x128 kernel, the 256x256 ping-pong and hipBLASLt.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm256.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/w4_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4/w4_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAIL" gpurun_out/r4/w4_tests.log | head -20; exit $rc; fi
S=bert_qkv_fwd,bert_ffn1_fwd,bert_ffn2_fwd,bert_ffn1_dgrad,bert_ffn2_dgrad,square_8192,square_4096,rn50_l3_1x1_1024to256,rn50_l3_1x1_256to1024,bert_qkv_wgrad,bert_ffn1_wgrad
timeout -k 10 400 python scripts/bench_gemm.py $S > gpurun_out/r4/w4_micro.jsonl 2>&1 || { tail -20 gpurun_out/r4/w4_micro.jsonl; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r4/w4_micro.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["shape"], {k: d[k]["tflops"] for k in d if isinstance(d[k], dict)})
PY
# weight gradients (fp32, split-K) routed to the four-wave kernels: atomics vs partial slabs
W=bert_qkv_wgrad,bert_ffn1_wgrad,bert_ffn2_wgrad,rn50_wgrad_1x1_1024to256
for v in "0 0" "128 0" "256 0" "128 1" "256 1"; do
  set -- $v
  DDL_GEMM_W4_WGRAD=$1 DDL_SPLITK_SLABS=$2 timeout -k 10 300 python scripts/bench_gemm.py $W > gpurun_out/r4/w4_wgrad_$1_$2.jsonl 2>&1 || { tail -5 gpurun_out/r4/w4_wgrad_$1_$2.jsonl; exit 1; }
  python - "$1" "$2" <<'PY'
import json, sys
for l in open(f"gpurun_out/r4/w4_wgrad_{sys.argv[1]}_{sys.argv[2]}.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print("w4_wgrad", sys.argv[1], "slabs", sys.argv[2], d["shape"], {k: d[k]["tflops"] for k in d if isinstance(d[k], dict)})
PY
done
