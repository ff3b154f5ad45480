#!/bin/bash
# Generic round-5 GPU call: optional pytest selection, GEMM sweep, benches.  Every GPU step runs under its own
# time limit and the script stops at the first failure.
#   TESTS="tests/a.py tests/b.py" KTEST="expr" GEMM="shape,list" BENCH=1 BERT=1 VGG=1 NYISO=1 TAG=name
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5/${TAG:-run}
mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS ${KTEST:+-k "$KTEST"} > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log
  [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
fi
if [ -n "${GEMM:-}" ]; then
  timeout -k 10 300 python scripts/bench_gemm.py $GEMM > $O/gemm.jsonl 2>&1 || { tail -20 $O/gemm.jsonl; exit 1; }
  grep -v amdgpu.ids $O/gemm.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['shape'], ' '.join('%s=%s'%(k,v['tflops']) for k,v in d.items() if isinstance(v,dict)))"
fi
for i in $(seq 1 ${BENCH:-0}); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | cut -c1-200
done
for i in $(seq 1 ${BERT:-0}); do
  timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 > $O/bert_$i.log 2>&1 || { tail -20 $O/bert_$i.log; exit 1; }
  tail -1 $O/bert_$i.log | cut -c1-200
done
for i in $(seq 1 ${VGG:-0}); do
  timeout -k 10 300 python bench.py --model vgg16 --steps 50 --warmup 10 > $O/vgg_$i.log 2>&1 || { tail -20 $O/vgg_$i.log; exit 1; }
  tail -1 $O/vgg_$i.log | cut -c1-200
done
if [ "${NYISO:-0}" = "1" ]; then
  for c in gru lstm; do
    timeout -k 10 300 python bench.py --model nyiso_$c > $O/nyiso_$c.log 2>&1 || { tail -20 $O/nyiso_$c.log; exit 1; }
    tail -1 $O/nyiso_$c.log | cut -c1-160
  done
fi
if [ -n "${PROF:-}" ]; then  # PROF="bench.py args" -> kernel stats
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -- python3 $GRAFT_REPO_ROOT/bench.py $PROF > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
  prc=$?; cd $GRAFT_REPO_ROOT; echo "rocprof rc=$prc"; [ $prc -eq 0 ] || exit $prc
fi
exit 0
