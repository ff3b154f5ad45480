"""Join rocprofv3 --pmc passes (one CSV per pass) by the order of the ddl:: dispatches and print
one row per dispatch: kernel, grid, VGPRs, duration and the derived counter ratios.

    python scripts/pmc_table.py <trace kernel_trace.csv> <pass1 counter_collection.csv> [...]
"""
import csv
import sys
from collections import OrderedDict, defaultdict


def load_pass(path):
    d = OrderedDict()
    for r in csv.DictReader(open(path)):
        if "ddl::" not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        e = d.setdefault(k, {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]), "vgpr": r["VGPR_Count"],
                             "agpr": r["Accum_VGPR_Count"], "lds": r["LDS_Block_Size"]})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(d.values())


def main():
    trace = [r for r in csv.DictReader(open(sys.argv[1])) if "ddl::" in r["Kernel_Name"]]
    passes = [load_pass(p) for p in sys.argv[2:]]
    rows = []
    for i, t in enumerate(trace):
        row = {"name": t["Kernel_Name"].split("(")[0].replace("void ddl::", "").replace("ddl::", ""),
               "grid": int(t["Grid_Size_X"]) * int(t["Grid_Size_Y"]) // int(t["Workgroup_Size_X"]),
               "us": (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3, "vgpr": t["VGPR_Count"],
               "agpr": t["Accum_VGPR_Count"]}
        for p in passes:
            if i < len(p):
                row.update({k: v for k, v in p[i].items() if k not in ("name", "grid", "vgpr", "agpr", "lds")})
        rows.append(row)
    agg = defaultdict(list)
    for r in rows:
        agg[(r["name"], r["grid"])].append(r)
    print(f"{'kernel':44s} {'grid':>6s} {'us':>7s} {'vg':>4s} {'mfma%':>6s} {'wait%':>6s} {'winst%':>6s} {'FETCH_MB':>9s} {'L2hit':>6s} {'ldsconf':>8s}")
    for (name, grid), rs in agg.items():
        n = len(rs)
        f = lambda k: sum(r.get(k, 0.0) for r in rs) / n
        us = f("us")
        gui = f("GRBM_GUI_ACTIVE")
        busy = f("SQ_BUSY_CYCLES")
        mfma = f("SQ_VALU_MFMA_BUSY_CYCLES")
        wave = f("SQ_WAVE_CYCLES")
        # MFMA busy (cycles, summed over SIMDs) / (GUI cycles per XCD * 8 XCDs * 32 CUs * 4 SIMDs)
        mf = 100 * mfma / (gui / 8 * 1024) if gui else float("nan")
        wait = 100 * f("SQ_WAIT_ANY") / wave if wave else float("nan")
        winst = 100 * f("SQ_WAIT_INST_ANY") / wave if wave else float("nan")
        hit = f("TCC_HIT_sum")
        miss = f("TCC_MISS_sum")
        l2 = 100 * hit / (hit + miss) if hit + miss else float("nan")
        print(f"{name[:44]:44s} {grid:6d} {us:7.1f} {rs[0]['vgpr']:>4s} {mf:6.1f} {wait:6.1f} {winst:6.1f} "
              f"{2 * f('FETCH_SIZE') / 1024:9.1f} {l2:6.1f} {f('SQ_LDS_BANK_CONFLICT'):8.0f}")


if __name__ == "__main__":
    main()
