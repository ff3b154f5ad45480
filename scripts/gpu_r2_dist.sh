#!/bin/bash
# Round-2 distributed-path check on the 1-GPU box: forced-RCCL tests, benches with and
# without the world-1 RCCL group / bf16 reduce / hipGraph step, all-reduce sweep, and a
# kernel trace of the forced-RCCL step.  Stops at the first crash/abort/timeout.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r2
export TMPDIR=/tmp
O=gpurun_out/r2
ok() { local rc=$1 what=$2; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$what crashed rc=$rc"; exit $rc; fi; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_ddp.py tests/test_gpu_graphs.py} > $O/tests.log 2>&1; ok $? tests; tail -3 $O/tests.log
for cfg in "A|" "B|--graph 0" "C|--reduce-dtype fp32" "D|--reduce-dtype bf16"; do
  tag=${cfg%%|*}; a=${cfg#*|}
  if [ $tag = C ] || [ $tag = D ]; then export DDL_FORCE_DIST=1; else unset DDL_FORCE_DIST; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $a > $O/bench_$tag.log 2>&1; ok $? bench_$tag; tail -1 $O/bench_$tag.log
done
unset DDL_FORCE_DIST
timeout -k 10 300 python bench.py --model vgg16 --steps 30 --warmup 5 > $O/vgg_graph.log 2>&1; ok $? vgg; tail -1 $O/vgg_graph.log
timeout -k 10 300 python bench.py --model vgg16 --steps 30 --warmup 5 --graph 0 > $O/vgg_eager.log 2>&1; ok $? vgg0; tail -1 $O/vgg_eager.log
timeout -k 10 300 python scripts/bench_allreduce.py --out $O/allreduce_n1.json > $O/allreduce.log 2>&1; ok $? allreduce; tail -2 $O/allreduce.log
cd /tmp
DDL_FORCE_DIST=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_forced -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof_forced.log 2>&1
echo "rocprof rc=$?"
