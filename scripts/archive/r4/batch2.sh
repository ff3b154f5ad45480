#!/bin/bash
# Second GPU call: round-4 GPU tests (determinism, co-located replica groups, convergence, row epilogue),
# then the split-K slab A/B on the whole VGG-16 / ResNet-50 step.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "[batch2] fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "splitk or slabs" --timeout 120 --timeout-method thread > gpurun_out/r4/b2_splitk.log 2>&1
rc=$?; tail -2 gpurun_out/r4/b2_splitk.log; fatal $rc splitk
timeout -k 10 900 python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_colocated.py tests/test_gpu_convergence.py \
  -v -s --timeout 400 --timeout-method thread > gpurun_out/r4/b2_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|cosine|passed|failed|MAPE|accuracy" gpurun_out/r4/b2_tests.log | tail -40; fatal $rc tests
: > gpurun_out/r4/b2_slabs_ab.txt
for i in 1 2; do
  for v in 0 1; do
    DDL_SPLITK_SLABS=$v timeout -k 10 200 python bench.py --model vgg16 --steps 30 --warmup 5 2>/dev/null | grep '^{' | sed "s/^/vgg slabs=$v /" >> gpurun_out/r4/b2_slabs_ab.txt; fatal $? vgg
    DDL_SPLITK_SLABS=$v timeout -k 10 200 python bench.py --steps 15 --warmup 4 2>/dev/null | grep '^{' | sed "s/^/rn50 slabs=$v /" >> gpurun_out/r4/b2_slabs_ab.txt; fatal $? rn50
  done
done
python - <<'PY'
import json
for line in open("gpurun_out/r4/b2_slabs_ab.txt"):
    m, tag, js = line.split(" ", 2)
    d = json.loads(js)
    print(m, tag, round(d["value"]), d["ms_per_step"])
PY
exit 0
