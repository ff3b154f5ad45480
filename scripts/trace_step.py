"""Print the dispatches of the last training step of a rocprofv3 kernel trace (>= a threshold in us).
Usage: python scripts/trace_step.py <kernel_trace.csv> <steps in the trace> [min_us]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2])
thr = float(sys.argv[3]) if len(sys.argv) > 3 else 8.0
ks = [(r["Kernel_Name"][:70], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000,
       int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), r["Grid_Size_Y"]) for r in rows]
n = len(ks) // steps
tot = 0.0
for k in ks[-n:]:
    tot += k[1]
    if k[1] >= thr:
        print(f"{k[1]:7.1f} {k[2]:6d}x{k[3]:<3} {k[0]}")
print(f"step kernel total {tot:.1f} us over {n} dispatches")
