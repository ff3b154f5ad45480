#!/bin/bash
# Convergence-parity tests (NYISO GPU vs CPU fp32, MNIST 8 co-located workers, ResNet-50 vs the torch path)
# with a heartbeat (the CPU NYISO leg is silent for minutes), then a kernel profile of the NYISO GRU bench.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
( while true; do sleep 50; echo "[hb] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
fatal() { case $1 in 124|134|137|139) echo "[batch5] fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_determinism.py::test_resnet50_full_depth_gradient_direction_per_stage \
  tests/test_gpu_convergence.py::test_mnist_8_colocated_workers_accuracy \
  tests/test_gpu_convergence.py::test_resnet50_learns_synthetic_task_like_torch_path \
  tests/test_gpu_convergence.py::test_nyiso_gpu_mape_matches_cpu_fp32 \
  -v -s --timeout 480 --timeout-method thread > gpurun_out/r4/b5_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|cosine|MAPE|accuracy|loss windows|passed|failed" gpurun_out/r4/b5_tests.log | tail -30; fatal $rc tests
R=$PWD
mkdir -p gpurun_out/r4/prof
( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4/prof/nyiso -- python3 $R/bench.py --model nyiso_gru > $R/gpurun_out/r4/prof/nyiso.log 2>&1 )
rc=$?; echo "[batch5] nyiso prof rc=$rc"; grep '^{' gpurun_out/r4/prof/nyiso.log | cut -c1-400; fatal $rc prof
for f in $(find gpurun_out/r4/prof/nyiso -name "*kernel_stats.csv"); do python3 scripts/prof_summary.py "$f" 1 gpurun_out/r4/prof/nyiso_$(basename $(dirname $f))_stats.csv | head -14; done
exit 0
