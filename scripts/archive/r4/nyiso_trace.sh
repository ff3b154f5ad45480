#!/bin/bash
# NYISO GRU / LSTM through the replica group: plain bench runs, then a kernel trace and its concurrency.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4/nyiso
R=$PWD
for m in nyiso_gru nyiso_lstm; do
  timeout -k 10 200 python bench.py --model $m 2>/dev/null | grep '^{' | cut -c1-330
done
( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4/nyiso/trace -- python3 $R/bench.py --model nyiso_gru > $R/gpurun_out/r4/nyiso/trace.log 2>&1 )
echo "trace rc=$?"
for f in $(find gpurun_out/r4/nyiso/trace -name "*kernel_trace.csv"); do python3 scripts/r4/overlap.py $f; done
