#!/bin/bash
# DataFrame-fed ResNet-50 on one MI355X: GPU tests of the ingest paths, the plain bench, the
# --via-dataframe bench with the shard resident and streamed, and a kernel + memory-copy trace of
# the streamed run (H2D copies on the side stream under the compute kernels).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/df; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_dataframe.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_plain.log 2>&1 || { tail $O/bench_plain.log; exit 1; }
tail -1 $O/bench_plain.log
for ing in resident stream; do
  timeout -k 10 400 python bench.py --via-dataframe --ingest $ing --steps 20 --warmup 5 > $O/bench_df_$ing.log 2>&1 || { tail $O/bench_df_$ing.log; exit 1; }
  tail -1 $O/bench_df_$ing.log
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_stream -- python3 $GRAFT_REPO_ROOT/bench.py --via-dataframe --ingest stream --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof_stream.log 2>&1
echo "rocprof rc=$?"
