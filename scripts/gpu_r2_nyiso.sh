#!/bin/bash
# The reference's own published workloads on one MI355X (4 co-located ADAG workers), plus the
# MNIST CNN workflow at the reference's AZTK configuration (8 workers, batch 16, window 5, 5 epochs)
# and a kernel trace of the GRU run.  Logs land in gpurun_out/nyiso (copied to profiles/ after).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/nyiso; mkdir -p $O
export TMPDIR=/tmp
for m in nyiso_gru nyiso_lstm; do
  timeout -k 10 300 python bench.py --model $m > $O/$m.json 2> $O/$m.log || { tail -20 $O/$m.log; exit 1; }
  tail -1 $O/$m.json
done
timeout -k 10 400 python examples/ddl_mnist.py --executors 4 --processes 2 --epochs 5 --train-rows 60000 --test-rows 10000 --workers-per-gpu 8 > $O/mnist8.log 2>&1 || { tail -20 $O/mnist8.log; exit 1; }
tail -4 $O/mnist8.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_gru -- python3 $GRAFT_REPO_ROOT/bench.py --model nyiso_gru > $GRAFT_REPO_ROOT/$O/prof_gru.log 2>&1
echo "rocprof rc=$?"
