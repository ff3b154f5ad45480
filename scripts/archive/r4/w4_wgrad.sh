#!/bin/bash
# Four-wave kernels for the fp32 weight gradients (split-K over tokens): atomics vs partial slabs.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
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
