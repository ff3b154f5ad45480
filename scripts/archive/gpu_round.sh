#!/bin/bash
# One gpurun call: kernel tests -> bench -> rocprofv3 kernel stats.  Stops at the first
# crash/abort/timeout (exit codes other than pytest's 0/1) so nothing runs on a sick GPU.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-10}
TESTS=${TESTS:-tests/test_gpu_kernels.py}
rc=0
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest $TESTS -x -q -m gpu ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -5 gpurun_out/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
fi
if [ "${SMOKE:-1}" = "1" ]; then
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
  src=$?
  tail -2 gpurun_out/smoke.log
  if [ $src -ne 0 ]; then echo "smoke failed rc=$src"; exit $src; fi
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py --steps $STEPS --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  brc=$?
  tail -3 gpurun_out/bench.log
  if [ $brc -ne 0 ]; then echo "bench failed rc=$brc"; exit $brc; fi
fi
if [ "${VGG:-0}" = "1" ]; then
  timeout -k 10 600 python bench.py --model vgg16 --steps $STEPS --warmup 3 > gpurun_out/bench_vgg.log 2>&1
  vrc=$?
  tail -2 gpurun_out/bench_vgg.log
  if [ $vrc -ne 0 ]; then echo "vgg bench failed rc=$vrc"; exit $vrc; fi
fi
if [ "${BERT:-0}" = "1" ]; then
  timeout -k 10 600 python bench.py --model bert --steps ${BERT_STEPS:-5} --warmup 2 ${BERT_ARGS:-} > gpurun_out/bench_bert.log 2>&1
  berc=$?
  tail -2 gpurun_out/bench_bert.log
  if [ $berc -ne 0 ]; then echo "bert bench failed rc=$berc"; exit $berc; fi
fi
if [ "${PROFILE:-0}" = "1" ]; then
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 ${BENCH_ARGS:-} > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
  prc=$?
  cd - >/dev/null
  echo "rocprof rc=$prc"
  find gpurun_out/prof -name "*stats*" | head
fi
exit $rc
