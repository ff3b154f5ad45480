#!/bin/bash
# rocprofv3 kernel statistics of the ResNet-50 headline step (3 timed + 2 warmup steps).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG:-x} -- python3 $R/bench.py --steps 3 --warmup 2 ${BENCH_ARGS:-} > $R/gpurun_out/prof_${TAG:-x}.log 2>&1
rc=$?
tail -n 1 $R/gpurun_out/prof_${TAG:-x}.log
exit $rc
