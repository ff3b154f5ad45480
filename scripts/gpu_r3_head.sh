#!/bin/bash
# HEAD evidence: selected GPU tests -> ResNet-50 bench -> rocprofv3 kernel stats of the bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu $TESTS > gpurun_out/head_tests.log 2>&1
  rc=$?; tail -4 gpurun_out/head_tests.log
  [ $rc -ne 0 ] && { echo "tests rc=$rc"; exit $rc; }
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/head_bench.log 2>&1 || { tail -20 gpurun_out/head_bench.log; exit 1; }
grep '^{' gpurun_out/head_bench.log
if [ "${PROFILE:-1}" = "1" ]; then
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/head_prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 ${BENCH_ARGS:-} > $GRAFT_REPO_ROOT/gpurun_out/head_prof.log 2>&1 ) || { echo "rocprof failed"; tail -20 gpurun_out/head_prof.log; exit 1; }
  f=$(find gpurun_out/head_prof -name "*kernel_stats.csv" | head -1)
  python scripts/prof_summary.py $f 7 gpurun_out/head_kstats.csv | head -25
fi
