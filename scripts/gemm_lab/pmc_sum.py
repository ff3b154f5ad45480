"""Sum rocprofv3 counter_collection.csv rows per kernel name; print per-kernel ratios."""
import csv
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(float))
n = defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0][-60:]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[k].add(r["Dispatch_Id"])
print(f"{'kernel':60s} {'disp':>4s} {'mfma%':>6s} {'wait%':>6s} {'ldsconf%':>8s} {'ldsbusy%':>8s} {'insts_lds':>10s}")
for k, c in agg.items():
    gui = c["GRBM_GUI_ACTIVE"] or 1
    mf = 100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * 1024)
    wt = 100 * c["SQ_WAIT_INST_ANY"] / max(1, c["SQ_WAVE_CYCLES"])
    lc = 100 * c["SQ_LDS_BANK_CONFLICT"] / max(1, c["SQ_LDS_IDX_ACTIVE"])
    lb = 100 * c["SQ_LDS_IDX_ACTIVE"] / (gui * 256)
    print(f"{k:60s} {len(n[k]):4d} {mf:6.1f} {wt:6.1f} {lc:8.2f} {lb:8.1f} {c['SQ_INSTS_LDS']:10.0f}")
