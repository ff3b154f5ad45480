# attention / transformer numerics at both dK-dV occupancies, then BERT at each (one GPU call)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_transformer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tr_occ1.log 2>&1 || { tail -20 gpurun_out/tr_occ1.log; exit 1; }
tail -1 gpurun_out/tr_occ1.log
DDL_ATTN_DKDV_OCC=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_transformer.py -x -q -k attention --timeout 120 --timeout-method thread > gpurun_out/tr_occ2.log 2>&1 || { tail -20 gpurun_out/tr_occ2.log; exit 1; }
tail -1 gpurun_out/tr_occ2.log
for o in 1 2; do
  DDL_ATTN_DKDV_OCC=$o timeout -k 10 200 python scripts/bench_attention.py > gpurun_out/attn_occ$o.log 2>&1 || exit $?
  tail -3 gpurun_out/attn_occ$o.log | cut -c1-300
  DDL_ATTN_DKDV_OCC=$o timeout -k 10 200 python bench.py --model bert --steps 10 --warmup 2 > gpurun_out/bert_occ$o.log 2>&1 || exit $?
  tail -1 gpurun_out/bert_occ$o.log | cut -c1-200
done
