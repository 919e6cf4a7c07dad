"""Where the GPU sits idle: from a rocprofv3 kernel (+ memory-copy) trace, the union of busy intervals over every
queue in the last N ms, and each idle gap attributed to the (last work that ended before it, first work that
started after it) pair.  A gap is host time the device waited through: a host sync followed by planning, or a
launch-bound stretch.  Summed per pair, the top rows name the syncs worth removing.

usage: python tools/gap_summary.py TRACE_DIR [--last-ms 300] [--min-gap-us 5] [--top 25]"""
import argparse
import collections
import csv
import glob
import os


def _name(r):
    return r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last-ms", type=float, default=300)
    ap.add_argument("--min-gap-us", type=float, default=5)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    ev = []
    for p in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), _name(r)))
    for p in glob.glob(os.path.join(a.dir, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       "copy:" + r["Direction"].replace("MEMORY_COPY_", "")))
    if not ev:
        raise SystemExit("no trace rows")
    ev.sort()
    end = max(e[1] for e in ev)
    t0 = end - a.last_ms * 1e6
    ev = [e for e in ev if e[0] >= t0]
    busy = 0
    gaps = collections.Counter()
    ngaps = collections.Counter()
    cur_end, last_name = ev[0][1], ev[0][2]
    seg_start = ev[0][0]
    for s, e, name in ev[1:]:
        if s > cur_end:
            busy += cur_end - seg_start
            gap = s - cur_end
            if gap >= a.min_gap_us * 1e3:
                gaps[(last_name, name)] += gap
                ngaps[(last_name, name)] += 1
            seg_start = s
        if e > cur_end:
            cur_end, last_name = e, name
    busy += cur_end - seg_start
    span = cur_end - ev[0][0]
    print(f"window {span / 1e6:.1f} ms: busy {busy / 1e6:.1f} ms ({100 * busy / span:.1f} %), "
          f"idle {(span - busy) / 1e6:.1f} ms in {sum(ngaps.values())} gaps >= {a.min_gap_us:g} us")
    print(f"\n{'idle ms':>8} {'gaps':>5} {'avg us':>7}  ended before -> started after")
    for (x, y), g in gaps.most_common(a.top):
        print(f"{g / 1e6:8.2f} {ngaps[(x, y)]:5d} {g / ngaps[(x, y)] / 1e3:7.1f}  {x} -> {y}")


if __name__ == "__main__":
    main()
