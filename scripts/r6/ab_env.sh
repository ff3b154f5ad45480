#!/bin/bash
# Interleaved A/B of an environment toggle: VAR=<name> A=<value> B=<value> R=<rounds> CMD=<command> (JSON lines).
set -o pipefail
mkdir -p gpurun_out/r6
out=gpurun_out/r6/ab_${VAR}${TAG}.txt
: > $out
for r in $(seq 1 ${R:-2}); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 ${T:-200} $CMD 2>/dev/null | sed "s/^/$VAR=$v /" >> $out || exit 1
  done
done
cat $out
