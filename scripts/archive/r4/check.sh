#!/bin/bash
# Round 4 GPU checks: determinism + replica groups + the tests touched by the BN pre-reduce guard,
# then the reference workloads through the replica groups.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_colocated.py \
  "tests/test_gpu_kernels.py::test_resnet_per_layer_gradients_match_fp32_cpu" \
  "tests/test_gpu_kernels.py::test_resnet50_step_matches_reference" "tests/test_gpu_kernels.py::test_prob_xent_matches_fp32" -v -s --timeout 300 --timeout-method thread > gpurun_out/r4/check_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|cosine|passed|failed" gpurun_out/r4/check_tests.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for m in nyiso_gru nyiso_lstm; do
  timeout -k 10 300 python bench.py --model $m > gpurun_out/r4/bench_${m}_groups.json 2> gpurun_out/r4/bench_${m}_groups.err || { tail -30 gpurun_out/r4/bench_${m}_groups.err; exit 1; }
  cat gpurun_out/r4/bench_${m}_groups.json
done
timeout -k 10 400 python examples/ddl_mnist.py --executors 4 --processes 2 --epochs 5 --train-rows 60000 --test-rows 10000 --workers-per-gpu 8 > gpurun_out/r4/mnist_8workers_groups.log 2>&1 || { tail -30 gpurun_out/r4/mnist_8workers_groups.log; exit 1; }
grep -E "Training time|Accuracy|updates|Workers" gpurun_out/r4/mnist_8workers_groups.log

# GEMM: 256x256 kernel with the slim (LITE) epilogue vs the full-epilogue instantiation (code size A/B)
timeout -k 10 300 python scripts/bench_gemm.py bert_qkv_fwd,bert_ffn1_fwd,bert_ffn2_fwd,bert_ffn1_dgrad,square_8192 > gpurun_out/r4/gemm_lite.jsonl 2>&1 || exit 1
DDL_GEMM_FULL_EPI=1 timeout -k 10 300 python scripts/bench_gemm.py bert_qkv_fwd,bert_ffn1_fwd,bert_ffn2_fwd,bert_ffn1_dgrad,square_8192 > gpurun_out/r4/gemm_full.jsonl 2>&1 || exit 1
cat gpurun_out/r4/gemm_lite.jsonl gpurun_out/r4/gemm_full.jsonl | grep shape
exit $rc
