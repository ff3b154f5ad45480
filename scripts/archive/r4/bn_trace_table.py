"""Per-call BN sweep durations from a rocprofv3 kernel trace, grouped by (kernel, grid): calls per step,
mean microseconds — the grid identifies the layer shape (stream_grid / col_grid of bn.hip)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
g = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"]
    if not any(s in k for s in ("bn_apply", "bn_bwd_dx", "bn_finalize", "bn_bwd_finalize", "pool3s2")):
        continue
    key = (k.split("(")[0][-40:], r.get("Grid_Size_X", r.get("Grid_Size", "?")), r.get("Grid_Size_Y", ""))
    g[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
steps = 5
tot = 0.0
for key, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v) / steps
    print(f"{key[0]:42s} grid {key[1]:>8s} x {key[2]:>3s}  calls/step {len(v) / steps:5.1f}  mean {sum(v) / len(v):7.1f} us  "
          f"ms/step {sum(v) / steps / 1e3:6.3f}")
print(f"total {tot / 1e3:.3f} ms/step")
