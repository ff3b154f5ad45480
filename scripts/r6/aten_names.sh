#!/bin/bash
# Steady-state kernels per training step by name (bench.py traced at --steps 3 and 8, same warmup): the at::native
# and runtime-copy kernels that remain per step, and the launch totals.  Usage: MODELS="bert resnet50" bash ...
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/aten
mkdir -p $O
for m in ${MODELS:-bert}; do
  for s in 3 8; do
    timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/t_${m}_$s -o t -- \
      python3 $R/bench.py --model $m --steps $s --warmup 2 > $O/${m}_$s.log 2>&1 || exit 1
  done
  python3 - "$m" "$O" <<'PY' >> $O/summary.txt || exit 1
import csv, glob, sys
from collections import Counter
m, o = sys.argv[1], sys.argv[2]
cnt = {}
for s in (3, 8):
    rows = list(csv.DictReader(open(glob.glob(f"{o}/t_{m}_{s}/**/*kernel_trace.csv", recursive=True)[0])))
    cnt[s] = Counter(r["Kernel_Name"] for r in rows)
per = {k: (cnt[8][k] - cnt[3][k]) / 5 for k in set(cnt[8]) | set(cnt[3])}
tot = sum(per.values())
aten = {k: v for k, v in per.items() if "at::" in k and v}
print(f"{m}: {tot:.1f} launches/step, at::native {sum(aten.values()):.1f}/step")
for k, v in sorted(aten.items(), key=lambda kv: -kv[1]):
    print(f"   {v:5.1f}  {k[:150]}")
PY
  rm -rf $O/t_${m}_3 $O/t_${m}_8
done
cat $O/summary.txt
