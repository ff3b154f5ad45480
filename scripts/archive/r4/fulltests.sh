#!/bin/bash
# The whole GPU test suite at HEAD (as the round driver runs it), with a heartbeat, then smoke().
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
( while true; do sleep 50; echo "[hb] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1080 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4/full_gpu_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r4/full_gpu_tests.log | grep -v "^\s*$"; echo "[fulltests] rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2
