# attention / transformer numerics at each dK-dV occupancy, then the attention microbenchmark
# and BERT at each (one GPU call)
set -u
mkdir -p gpurun_out
for o in 2 3; do
  DDL_ATTN_DKDV_OCC=$o timeout -k 10 300 python -u -m pytest tests/test_gpu_transformer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tr_occ$o.log 2>&1 || { tail -20 gpurun_out/tr_occ$o.log; exit 1; }
  tail -1 gpurun_out/tr_occ$o.log
done
for o in 2 3 2 3; do
  DDL_ATTN_DKDV_OCC=$o timeout -k 10 200 python scripts/bench_attention.py > gpurun_out/attn_occ$o.log 2>&1 || exit $?
  tail -3 gpurun_out/attn_occ$o.log | cut -c1-300
  DDL_ATTN_DKDV_OCC=$o timeout -k 10 200 python bench.py --model bert --steps 10 --warmup 3 > gpurun_out/bert_occ$o.log 2>&1 || exit $?
  echo "dkdv_occ=$o $(tail -1 gpurun_out/bert_occ$o.log | cut -c1-120)"
done
