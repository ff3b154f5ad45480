#!/bin/bash
# Same-box kernel-level A/B: rocprofv3 kernel stats of bench.py for ab/base and this tree, plus the GEMM
# microbenchmark on both.  ARGS="bench args" GEMM="shapes" TAG=name
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5/${TAG:-abprof}
mkdir -p $O
if [ -n "${GEMM:-}" ]; then
  for r in 1 2; do
    timeout -k 10 300 python ab/base/bench_gemm.py $GEMM > $O/gemm_base_$r.jsonl 2>&1 || { tail -5 $O/gemm_base_$r.jsonl; exit 1; }
    timeout -k 10 300 python scripts/bench_gemm.py $GEMM > $O/gemm_head_$r.jsonl 2>&1 || { tail -5 $O/gemm_head_$r.jsonl; exit 1; }
  done
fi
if [ -n "${ARGS:-}" ]; then
  cd /tmp
  for arm in base head; do
    if [ $arm = base ]; then B=$GRAFT_REPO_ROOT/ab/base/bench.py; else B=$GRAFT_REPO_ROOT/bench.py; fi
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$arm -- python3 $B $ARGS > $O/prof_$arm.log 2>&1 || { tail -5 $O/prof_$arm.log; exit 1; }
  done
fi
echo done
