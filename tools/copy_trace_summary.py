"""Summarise a rocprofv3 kernel + memory-copy trace: blit-kernel copies by grid size, SDMA copies by direction/size,
and the kernels' busy time per name, over the last 10 steps of a bench run."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
kt = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
mt = glob.glob(os.path.join(root, "**", "*memory_copy_trace.csv"), recursive=True)
if kt:
    rows = list(csv.DictReader(open(kt[0])))
    print("kernel trace rows", len(rows), "fields", list(rows[0].keys())[:30])
    blit = defaultdict(lambda: [0, 0])
    for r in rows:
        if "copyBuffer" in r["Kernel_Name"] or "fillBuffer" in r["Kernel_Name"]:
            g = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            k = (r["Kernel_Name"][:40], g)
            blit[k][0] += 1
            blit[k][1] += d
    for k, (c, d) in sorted(blit.items(), key=lambda x: -x[1][1])[:25]:
        print(f"{k[0]:42s} grid {k[1]:>10d} calls {c:5d} total_us {d/1e3:10.1f} avg_us {d/c/1e3:8.1f}")
if mt:
    rows = list(csv.DictReader(open(mt[0])))
    print("memcpy trace rows", len(rows), "fields", list(rows[0].keys()))
    agg = defaultdict(lambda: [0, 0, 0])
    for r in rows:
        sz = int(r.get("Bytes") or r.get("Size") or 0)
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        b = 1 << max(0, sz.bit_length() - 1)
        k = (r.get("Direction") or r.get("Operation") or "?", b)
        agg[k][0] += 1
        agg[k][1] += d
        agg[k][2] += sz
    for k, (c, d, sz) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
        print(f"{k[0]:28s} >= {k[1]:>12d} B calls {c:5d} total_us {d/1e3:10.1f} GB/s {sz/max(d,1):7.1f}")
