#!/bin/bash
# HEAD evidence: full GPU test suite, smoke, ResNet-50 bench + kernel profile, BERT / VGG benches;
# optional PMC pass of the 64-channel resident-filter kernel (C64PMC=1)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
if [ "${C64PMC:-0}" = "1" ]; then
  O=$R/gpurun_out/pmc_c64; rm -rf $O; mkdir -p $O
  export DDL_CONV3X3_C64PP=1
  ( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -- python3 $R/scripts/bench_c64.py > $O/trace.log 2>&1 ) || { echo trace failed; exit 1; }
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES --output-format csv -d $O/p1 -- python3 $R/scripts/bench_c64.py > $O/p1.log 2>&1 ) || { echo p1 failed; exit 1; }
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p2 -- python3 $R/scripts/bench_c64.py > $O/p2.log 2>&1 ) || { echo p2 failed; exit 1; }
  unset DDL_CONV3X3_C64PP
  t=$(find $O/trace -name "*kernel_trace.csv" | head -1); a=$(find $O/p1 -name "*counter_collection.csv" | head -1); b=$(find $O/p2 -name "*counter_collection.csv" | head -1)
  python scripts/pmc_table.py $t $a $b > gpurun_out/pmc_c64_table.txt 2>&1; head -3 gpurun_out/pmc_c64_table.txt; grep -E "c64" gpurun_out/pmc_c64_table.txt | head -4
fi
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/ev_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ev_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/ev_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ev_smoke.log 2>&1 || { tail gpurun_out/ev_smoke.log; exit 1; }
tail -1 gpurun_out/ev_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/ev_bench_default.log 2>&1 || { tail gpurun_out/ev_bench_default.log; exit 1; }
grep '^{' gpurun_out/ev_bench_default.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ev_bench.log 2>&1 || { tail gpurun_out/ev_bench.log; exit 1; }
grep '^{' gpurun_out/ev_bench.log
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ev_prof -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/ev_prof.log 2>&1 ) || { echo "rocprof failed"; exit 1; }
f=$(find gpurun_out/ev_prof -name "*kernel_stats.csv" | head -1)
python scripts/prof_summary.py $f 7 gpurun_out/ev_kstats.csv > gpurun_out/ev_ksum.txt; head -12 gpurun_out/ev_ksum.txt
for m in bert vgg16; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/ev_bench_$m.log 2>&1 || { tail gpurun_out/ev_bench_$m.log; exit 1; }
  grep '^{' gpurun_out/ev_bench_$m.log
done
