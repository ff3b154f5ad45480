#!/bin/bash
# rocprofv3 kernel statistics of the BERT-base and ResNet-50 benches at HEAD -> gpurun_out/r4/prof/*.csv
# (per-step tables via scripts/prof_summary.py; 5 timed + 2 warmup steps each).
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4/prof
cd /tmp && export TMPDIR=/tmp
for m in bert resnet50 vgg16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4/prof/$m -- python3 $R/bench.py --model $m --steps 5 --warmup 2 > $R/gpurun_out/r4/prof/$m.log 2>&1
  rc=$?; echo "[prof] $m rc=$rc"; grep '^{' $R/gpurun_out/r4/prof/$m.log | cut -c1-160
  case $rc in 0) ;; *) exit $rc;; esac
  f=$(find $R/gpurun_out/r4/prof/$m -name "*kernel_stats.csv" | head -1)
  python3 $R/scripts/prof_summary.py "$f" 7 $R/gpurun_out/r4/prof/${m}_kernel_stats.csv | head -12
  find $R/gpurun_out/r4/prof/$m -name "*kernel_trace.csv" -delete
done
