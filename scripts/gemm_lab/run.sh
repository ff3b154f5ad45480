#!/bin/bash
# GEMM lab sweep on one MI355X: scripts/gemm_lab/run.sh [outfile]
cd "$(dirname "$0")"
out=${1:-../../gpurun_out/gemm_lab.jsonl}
mkdir -p "$(dirname "$out")"
: > "$out"
while read -r M N K E; do
  [ -z "$M" ] && continue
  timeout -k 5 60 ./lab "$M" "$N" "$K" "$E" 5 >> "$out" 2>&1 || { echo "FAIL $M $N $K $E rc=$?" >> "$out"; exit 1; }
done <<SHAPES
${SHAPES:-8192 8192 8192 lite
4096 4096 4096 lite
16384 2304 768 lite
16384 3072 768 lite
16384 768 3072 lite
16384 768 768 lite
16384 768 2304 lite
16384 3072 768 gelu
16384 768 3072 resid
16384 768 768 resid}
SHAPES
cat "$out"
