"""Summarise a rocprofv3 --stats kernel_stats.csv into profiles/: per-kernel calls, average
microseconds and milliseconds per training step.  Usage:
    python scripts/prof_summary.py <kernel_stats.csv> <timed+warmup steps> <out.csv>"""
import csv
import sys


def main():
    src, steps, dst = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    rows = list(csv.DictReader(open(src)))
    out = []
    for r in rows:
        tot = float(r["TotalDurationNs"])
        calls = int(r["Calls"])
        out.append({"ms_per_step": round(tot / 1e6 / steps, 3), "calls": calls,
                    "avg_us": round(tot / calls / 1e3, 1), "kernel": r["Name"][:200]})
    out.sort(key=lambda d: -d["ms_per_step"])
    with open(dst, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["ms_per_step", "calls", "avg_us", "kernel"])
        w.writeheader()
        w.writerows(out)
    print(f"total {sum(d['ms_per_step'] for d in out):.2f} ms/step over {len(out)} kernels")
    for d in out[:25]:
        print(f"{d['ms_per_step']:8.3f} {d['calls']:6d} {d['avg_us']:8.1f}  {d['kernel'][:90]}")


if __name__ == "__main__":
    main()
