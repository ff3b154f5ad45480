"""Compare per-layer conv tables (scripts/bench_resnet_layers.py outputs) side by side."""
import json
import sys

ds = [json.load(open(f)) for f in sys.argv[1:]]
for f, d in zip(sys.argv[1:], ds):
    print(f, {k: round(v, 3) for k, v in d["total_ms_per_step"].items()})
for i, r in enumerate(ds[0]["layers"]):
    cells = []
    for pas in ("fwd", "dgrad", "wgrad"):
        cells.append(pas[0] + " " + " ".join(f"{d['layers'][i][pas]['ms']:.4f}" for d in ds))
    print(f"{r['H']:3d} {r['Ci']:4d}->{r['Co']:4d} k{r['k']} s{r['stride']} x{r['count']} | " + " | ".join(cells))
