"""Per-step GPU busy time vs idle gaps from a rocprofv3 kernel trace.

Steps are delimited by the optimizer kernel (the last launch of every training step).  For each step:
wall = end of this step's optimizer kernel - end of the previous one, busy = union of kernel
intervals inside it, gaps = wall - busy (GPU idle: host launch overhead, synchronisation).
Usage: python scripts/r4/trace_gaps.py <kernel_trace.csv> [step_kernel_substring]"""
import csv
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    marker = sys.argv[2] if len(sys.argv) > 2 else "sgd_kernel"
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    ends = [e for s, e, n in ks if marker in n]
    out = []
    for a, b in zip(ends, ends[1:]):
        inside = [(max(s, a), min(e, b)) for s, e, n in ks if e > a and s < b]
        busy, cur_s, cur_e = 0, None, None
        for s, e in sorted(inside):
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        ksum = sum(e - s for s, e in inside)
        out.append(((b - a) / 1e6, busy / 1e6, ksum / 1e6, len(inside)))
    if not out:
        print("no steps found (marker %r)" % marker)
        return
    for i, (w, bu, ksum, n) in enumerate(out):
        print(f"step {i:3d}: wall {w:7.3f} ms  busy {bu:7.3f} ms  idle {w - bu:6.3f} ms  kernel-sum {ksum:7.3f} ms  kernels {n}")
    med = lambda j: statistics.median(o[j] for o in out)
    print(f"median: wall {med(0):.3f} busy {med(1):.3f} idle {med(0) - med(1):.3f} kernel-sum {med(2):.3f} ms")


if __name__ == "__main__":
    main()
