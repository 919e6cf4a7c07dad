"""Summarise a rocprofv3 kernel + memory-copy trace as a timeline of the last N ms: per stream/queue, the busy
intervals of large kernels and copies (ms relative to the window start).

usage: python tools/timeline.py TRACE_DIR [--last-ms 60] [--min-us 200]"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last-ms", type=float, default=60)
    ap.add_argument("--min-us", type=float, default=200)
    a = ap.parse_args()
    ev = []
    for p in glob.glob(os.path.join(a.dir, "*kernel_trace.csv")):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"q{r['Queue_Id']}/s{r['Stream_Id']}",
                       r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:40]))
    for p in glob.glob(os.path.join(a.dir, "*memory_copy_trace.csv")):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"copy/s{r['Stream_Id']}",
                       r["Direction"].replace("MEMORY_COPY_", "")))
    ev.sort()
    end = max(e[1] for e in ev)
    t0 = end - a.last_ms * 1e6
    for s, e, lane, name in ev:
        if e < t0 or (e - s) < a.min_us * 1e3:
            continue
        print(f"{(s - t0) / 1e6:8.2f} {(e - t0) / 1e6:8.2f} {(e - s) / 1e6:7.2f}  {lane:10s} {name}")


if __name__ == "__main__":
    main()
