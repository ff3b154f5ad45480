"""Write profiles/isa_summary.csv: per-kernel MFMA / LDS-transpose / LDS-DMA / scratch
instruction counts of the gfx950 code in the built extension (static, no GPU)."""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributeddeeplearningspark_amd.utils.isa import summary  # noqa: E402

rows = summary(os.path.join(ROOT, "distributeddeeplearningspark_amd", "_C.so"))
out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "isa_summary.csv")
with open(out, "w", newline="") as f:
    w = csv.DictWriter(f, fieldnames=["kernel", "instructions", "mfma", "ds_read_tr", "lds_dma", "scratch", "loop_scratch"])
    w.writeheader()
    w.writerows(rows)
print(f"{len(rows)} kernels -> {out}; with MFMA: {sum(r['mfma'] > 0 for r in rows)}; "
      f"spilling: {[r['kernel'][:60] for r in rows if r['scratch']]}")
