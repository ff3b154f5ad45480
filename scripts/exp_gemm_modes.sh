set -u
mkdir -p gpurun_out
for m in 0 2; do
  DDL_GEMM_DMA=$m timeout -k 10 200 python bench.py --model bert --steps 10 --warmup 2 > gpurun_out/bert_dma$m.log 2>&1 || exit $?
  tail -1 gpurun_out/bert_dma$m.log | cut -c1-200
done
DDL_GEMM_DMA=2 timeout -k 10 200 python scripts/bench_gemm.py > gpurun_out/gemm_dma2.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_bert -- python3 $GRAFT_REPO_ROOT/bench.py --model bert --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_bert.log 2>&1
echo prof rc=$?
