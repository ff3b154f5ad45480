"""Idle time inside whole training steps of a rocprofv3 kernel trace.  Steps are delimited by a marker
kernel that runs once per step (default: the step-start `zero_ranges_kernel`); for the last N complete
steps prints the step span, the busy union of its kernels, the idle remainder and the largest gaps with
the kernels on either side.
Usage: python scripts/r6/trace_gaps.py <kernel_trace.csv> [N=5] [marker=zero_ranges_kernel] [top=12]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
N = int(sys.argv[2]) if len(sys.argv) > 2 else 5
marker = sys.argv[3] if len(sys.argv) > 3 else "zero_ranges_kernel"
top = int(sys.argv[4]) if len(sys.argv) > 4 else 12
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
starts = [i for i, e in enumerate(ev) if marker in e[2]]
if len(starts) < N + 1:
    sys.exit(f"only {len(starts)} marker dispatches")
gaps_all = []
tot_span = tot_busy = 0
for s, e in zip(starts[-N - 1:-1], starts[-N:]):
    win = ev[s:e]
    t0, t1 = win[0][0], ev[e][0]
    busy, end = 0, t0
    prev = None
    for a, b, n in win:
        if a > end and prev is not None:
            gaps_all.append((a - end, prev, n))
        if b > end:
            busy += b - max(a, end)
            end = b
            prev = n
    tot_span += t1 - t0
    tot_busy += busy
print(f"{N} steps: span {tot_span / N / 1e6:.3f} ms/step, busy {tot_busy / N / 1e6:.3f} ms/step, "
      f"idle {(tot_span - tot_busy) / N / 1e6:.3f} ms/step, dispatches/step {(starts[-1] - starts[-N - 1]) / N:.0f}")
gaps_all.sort(reverse=True)
print(f"gaps > 5 us: {sum(1 for g in gaps_all if g[0] > 5000) / N:.1f}/step totalling "
      f"{sum(g[0] for g in gaps_all if g[0] > 5000) / N / 1e3:.1f} us/step; "
      f"gaps <= 5 us: {sum(1 for g in gaps_all if g[0] <= 5000) / N:.0f}/step totalling "
      f"{sum(g[0] for g in gaps_all if g[0] <= 5000) / N / 1e3:.1f} us/step")
for g, a, b in gaps_all[:top]:
    print(f"{g / 1e3:8.1f} us  after {a[:70]}  before {b[:70]}")
