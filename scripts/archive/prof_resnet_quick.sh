#!/bin/bash
# kernel-trace + stats of a short ResNet-50 bench run (bs 256) -> gpurun_out/profq
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profq -- python3 $R/bench.py --steps 5 --warmup 2 ${BENCH_ARGS:-} > $R/gpurun_out/profq.log 2>&1
echo "rocprof rc=$?"; tail -1 $R/gpurun_out/profq.log | cut -c1-200
