"""Concurrency of a rocprofv3 kernel trace: sum of kernel durations / union of their intervals (1.0 = fully
serial), and the same per time window.  Usage: python scripts/r4/overlap.py <kernel_trace.csv>"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    ksum = sum(e - s for s, e in iv)
    union, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                union += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union += ce - cs
    span = iv[-1][1] - iv[0][0]
    print(f"kernels {len(iv)}  span {span / 1e6:.1f} ms  busy(union) {union / 1e6:.1f} ms  kernel-sum {ksum / 1e6:.1f} ms"
          f"  concurrency {ksum / union:.2f}  idle {(span - union) / 1e6:.1f} ms")


if __name__ == "__main__":
    main()
