"""Summarise a rocprofv3 kernel trace: dispatch count, summed kernel time, GPU-busy union, and the
top kernels by total time, restricted to the window [t0 + skip, t0 + skip + span] seconds.
Usage: python scripts/r5/trace_busy.py <kernel_trace.csv> [top=25] [min_gap_s=0.5]
The window is the longest run of dispatches whose gaps stay under min_gap_s (the training loop)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
gap = float(sys.argv[3]) if len(sys.argv) > 3 else 0.5
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# split into segments at gaps > gap seconds; take the segment with the most summed kernel time
segs, cur = [], [ev[0]]
for e in ev[1:]:
    if e[0] - max(c[1] for c in cur[-64:]) > gap * 1e9:
        segs.append(cur)
        cur = []
    cur.append(e)
segs.append(cur)
for s in segs:
    print(f"segment: {len(s)} dispatches, span {(max(e[1] for e in s) - s[0][0]) / 1e9:.3f} s, "
          f"kernel sum {sum(e[1] - e[0] for e in s) / 1e9:.3f} s")
seg = max(segs, key=lambda s: sum(e[1] - e[0] for e in s))
span = (max(e[1] for e in seg) - seg[0][0]) / 1e9
busy, end = 0, 0
for a, b, _ in seg:
    if b > end:
        busy += b - max(a, end)
        end = b
agg = defaultdict(lambda: [0, 0])
for a, b, n in seg:
    agg[n][0] += 1
    agg[n][1] += b - a
print(f"\nmain segment: {len(seg)} dispatches, span {span:.3f} s, busy union {busy / 1e9:.3f} s, "
      f"kernel sum {sum(v[1] for v in agg.values()) / 1e9:.3f} s")
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{t / 1e6:9.2f} ms {c:8d} x {t / c / 1e3:7.2f} us  {n[:110]}")
