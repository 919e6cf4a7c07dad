"""Per-stage timeline summary from a rocprofv3 ``--marker-trace --kernel-trace`` run with ``DXA_TRACE=1``.

For every roctx range name (parse, project, windows, sql:<view>, output_stage, …): how many times it ran, its mean
host duration, and how much of that wall time the GPU spent executing kernels (any stream) — a stage whose GPU-busy
share is low is host-bound.  Only ranges after the first ``--skip`` occurrences of each name are counted (warm-up).
    python tools/marker_summary.py <rocprofv3 output dir> [--skip N]"""
import bisect
import csv
import glob
import os
import sys
from collections import defaultdict


def _find(root, pat):
    g = glob.glob(os.path.join(root, "**", pat), recursive=True)
    return g[0] if g else None


def _col(row, *names):
    for n in names:
        if n in row and row[n] != "":
            return row[n]
    raise KeyError(names)


def main():
    root = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 5
    mk = _find(root, "*marker_api_trace.csv")
    kt = _find(root, "*kernel_trace.csv")
    if not mk or not kt:
        print("missing marker or kernel trace under", root)
        return 1
    kern = sorted((int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp"))) for r in csv.DictReader(open(kt)))
    # merge kernel intervals (streams overlap) into busy intervals
    busy = []
    for s, e in kern:
        if busy and s <= busy[-1][1]:
            busy[-1][1] = max(busy[-1][1], e)
        else:
            busy.append([s, e])
    starts = [b[0] for b in busy]
    cum = [0]
    for s, e in busy:
        cum.append(cum[-1] + (e - s))

    def busy_in(a, b):
        """GPU-busy ns within [a, b)."""
        i = bisect.bisect_right(starts, a) - 1
        tot = 0
        i = max(i, 0)
        while i < len(busy) and busy[i][0] < b:
            s, e = busy[i]
            tot += max(0, min(e, b) - max(s, a))
            i += 1
        return tot

    seen = defaultdict(int)
    agg = defaultdict(lambda: [0, 0, 0])
    for r in csv.DictReader(open(mk)):
        name = _col(r, "Message", "Marker_Message", "Function", "Operation", "Name")
        s, e = int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp"))
        if e <= s:
            continue
        seen[name] += 1
        if seen[name] <= skip:
            continue
        a = agg[name]
        a[0] += 1
        a[1] += e - s
        a[2] += busy_in(s, e)
    print(f"{'range':34s} {'n':>5s} {'host ms':>9s} {'gpu busy':>9s}")
    for name, (n, d, b) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"{name[:34]:34s} {n:5d} {d / n / 1e6:9.3f} {100.0 * b / d:8.1f}%")
    return 0


if __name__ == "__main__":
    sys.exit(main())
