#!/bin/bash
# Deterministic-mode kernels (two-pass bias / word-embedding gradients), the ResNet-50 convergence test at
# lr 0.01, and the deterministic-mode cost on BERT-base after the fix.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
( while true; do sleep 50; echo "[hb] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
fatal() { case $1 in 124|134|137|139) echo "[batch8] fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_transformer.py tests/test_gpu_determinism.py \
  tests/test_gpu_convergence.py::test_resnet50_learns_synthetic_task_like_torch_path \
  -q -s --timeout 400 --timeout-method thread > gpurun_out/r4/b8_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|loss windows" gpurun_out/r4/b8_tests.log | tail -20; fatal $rc tests
: > gpurun_out/r4/b8.txt
for i in 1 2; do
  for v in 0 1; do
    DDL_DETERMINISTIC=$v timeout -k 10 240 python bench.py --model bert --steps 10 --warmup 3 2>/dev/null | grep '^{' | sed "s/^/bert det=$v /" >> gpurun_out/r4/b8.txt; fatal $? bert
  done
done
python - <<'PY'
import json
for line in open("gpurun_out/r4/b8.txt"):
    a, b, js = line.split(" ", 2); d = json.loads(js); print(a, b, round(d["value"]), d["ms_per_step"])
PY
exit 0
