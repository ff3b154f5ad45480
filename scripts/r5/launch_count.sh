#!/bin/bash
# Steady-state kernel launches per training step: bench.py traced at --steps 3 and --steps 8 (same warmup);
# launches per step = (dispatches(8) - dispatches(3)) / 5, so one-time setup and warmup work cancels out.
# Usage: MODELS="resnet50 vgg16 bert" bash scripts/r5/launch_count.sh
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5/launch_count
mkdir -p $O
for m in ${MODELS:-resnet50 vgg16}; do
  for s in 3 8; do
    timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/t_${m}_$s -o t -- \
      python3 $R/bench.py --model $m --steps $s --warmup 2 > $O/${m}_$s.log 2>&1 || exit 1
  done
  python3 - "$m" "$O" <<'EOF' >> $O/summary.txt || exit 1
import csv, glob, sys
from collections import Counter
m, o = sys.argv[1], sys.argv[2]
cnt = {}
for s in (3, 8):
    rows = list(csv.DictReader(open(glob.glob(f"{o}/t_{m}_{s}/**/*kernel_trace.csv", recursive=True)[0])))
    cnt[s] = Counter("aten" if "at::" in r["Kernel_Name"] else "copy" if "rocclr" in r["Kernel_Name"] else "ddl"
                     for r in rows)
d = {k: (cnt[8][k] - cnt[3][k]) / 5 for k in ("ddl", "aten", "copy")}
print(f"{m}: {sum(d.values()):.1f} launches/step (ddl {d['ddl']:.1f}, at::native {d['aten']:.1f}, "
      f"runtime copies {d['copy']:.1f}); totals 3-step {sum(cnt[3].values())}, 8-step {sum(cnt[8].values())}")
EOF
  rm -rf $O/t_${m}_3 $O/t_${m}_8
done
cat $O/summary.txt
