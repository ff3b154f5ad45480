#!/bin/bash
# Rows-per-workgroup sweep of the register-resident GRU/LSTM kernels (kernel times via rocprofv3).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for bb in 1 2 4; do
  DDL_RNN_BB=$bb timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bb$bb -- python3 $R/scripts/bench_rnn_step.py 200 > $R/gpurun_out/bb$bb.log 2>&1 || exit $?
  echo "BB=$bb"; grep step $R/gpurun_out/bb$bb.log
  grep -h "rnn_" $R/gpurun_out/bb$bb/*/*kernel_stats.csv | awk -F'","' '{print $2, $4}' | cut -c1-120
done
