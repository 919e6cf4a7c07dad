"""Summarise rocprofv3 ``--pmc`` CSVs: counters summed per kernel over all dispatches, plus derived ratios.

usage: python tools/pmc_summary.py OUT.md DIR [DIR...]   (each DIR holds *counter_collection.csv files)
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(dirs):
    per = defaultdict(lambda: defaultdict(float))
    meta = {}
    disp = defaultdict(set)
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    k = row.get("Kernel_Name", "?")
                    k = k.replace("(anonymous namespace)::", "").split("(")[0][:70]
                    per[k][row["Counter_Name"]] += float(row["Counter_Value"])
                    disp[k].add((path, row.get("Dispatch_Id")))
                    meta.setdefault(k, {c: row.get(c) for c in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count",
                                                               "LDS_Block_Size", "Workgroup_Size", "Grid_Size")})
    return per, meta, disp


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    per, meta, disp = load(dirs)
    counters = sorted({c for v in per.values() for c in v})
    rows = sorted(per.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", kv[1].get("GRBM_GUI_ACTIVE", 0)))
    with open(out, "w") as f:
        f.write("| kernel | dispatches | VGPR | LDS | " + " | ".join(counters) +
                " | VALU/wave | VMEM_RD/wave | active% | wait% |\n")
        f.write("|---" * (len(counters) + 8) + "|\n")
        for k, v in rows:
            m = meta.get(k, {})
            waves = v.get("SQ_WAVES") or 0
            cyc = v.get("SQ_WAVE_CYCLES") or 0
            d = [f"{v[c]:.4g}" for c in counters]
            valu = f"{v.get('SQ_INSTS_VALU', 0) / waves:.0f}" if waves else ""
            vm = f"{v.get('SQ_INSTS_VMEM_RD', 0) / waves:.0f}" if waves else ""
            act = f"{100 * v.get('SQ_ACTIVE_INST_ANY', 0) / cyc:.0f}" if cyc and "SQ_ACTIVE_INST_ANY" in v else ""
            wt = f"{100 * v.get('SQ_WAIT_ANY', 0) / cyc:.0f}" if cyc and "SQ_WAIT_ANY" in v else ""
            f.write(f"| {k} | {len(disp[k])} | {m.get('VGPR_Count', '')} | {m.get('LDS_Block_Size', '')} | " +
                    " | ".join(d) + f" | {valu} | {vm} | {act} | {wt} |\n")
    print(open(out).read()[:6000])


if __name__ == "__main__":
    main()
