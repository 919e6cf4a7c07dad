"""Per-kernel roofline table from rocprofv3 ``--pmc`` passes (``tools/gpu/gpu_pmc.sh``).

usage: python tools/pmc_roofline.py OUT.md TITLE PASS_DIR [PASS_DIR...]

Every counter is averaged over the dispatches of the pass that collected it (a pass holds only some counters, so
summing over all passes' dispatches would dilute them).  HBM bytes per dispatch are FETCH_SIZE + WRITE_SIZE (both
in KiB, rocprofv3's derived-counter definitions); the duration of a dispatch is End − Start of the same record, so
the achieved bandwidth pairs bytes and time of the same launches (counter collection serialises dispatches: this is
the kernel alone on the chip).  MI355X HBM3E peak ≈ 8 TB/s.
"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

PEAK_TBS = 8.0


def _short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    base = name.split("(")[0]
    return base[:64]


def load(dirs):
    vals = defaultdict(lambda: defaultdict(list))         # kernel -> counter -> per-dispatch values
    durs = defaultdict(lambda: defaultdict(list))         # kernel -> counter -> durations of the same dispatches
    meta = {}
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    k = _short(row.get("Kernel_Name", "?"))
                    c = row["Counter_Name"]
                    vals[k][c].append(float(row["Counter_Value"]))
                    durs[k][c].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
                    meta.setdefault(k, (row.get("VGPR_Count"), row.get("LDS_Block_Size"), row.get("Grid_Size"),
                                        row.get("Workgroup_Size")))
    return vals, durs, meta


def mean(v):
    return sum(v) / len(v) if v else 0.0


def table(vals, durs, meta, top=24):
    rows = []
    for k, cs in vals.items():
        g = lambda c: mean(cs.get(c, []))                  # noqa: E731
        nd = max(len(v) for v in cs.values())
        dur_ns = statistics.median(durs[k].get("FETCH_SIZE") or durs[k].get("SQ_WAVES") or [0])
        rd, wr = g("FETCH_SIZE") * 1024, g("WRITE_SIZE") * 1024
        tbs = (rd + wr) / dur_ns / 1e3 if dur_ns else 0.0
        waves = g("SQ_WAVES") or 1.0
        wc = g("SQ_WAVE_CYCLES") or 1.0
        hit, miss = g("TCC_HIT_sum"), g("TCC_MISS_sum")
        lds = g("SQ_ACTIVE_INST_LDS")
        rows.append({
            "kernel": k, "n": nd, "us": dur_ns / 1e3, "rd": rd / 1e6, "wr": wr / 1e6, "tbs": tbs,
            "pct": 100 * tbs / PEAK_TBS, "valu": g("SQ_INSTS_VALU") / waves, "salu": g("SQ_INSTS_SALU") / waves,
            "vmem": g("SQ_INSTS_VMEM_RD") / waves, "active": 100 * g("SQ_ACTIVE_INST_ANY") / wc,
            "wait": 100 * g("SQ_WAIT_ANY") / wc, "l2": 100 * hit / (hit + miss) if hit + miss else 0.0,
            "ldsc": 100 * g("SQ_LDS_BANK_CONFLICT") / lds if lds else 0.0, "vgpr": meta[k][0],
            "total_us": dur_ns / 1e3 * nd,
        })
    rows.sort(key=lambda r: -r["total_us"])
    out = ["| kernel | dispatches/pass | median µs | HBM read MB | HBM write MB | achieved TB/s | % of 8 TB/s | "
           "VALU / wave | SALU / wave | VMEM rd / wave | active % | wait % | L2 hit % | LDS conflict % | VGPR |",
           "|---" * 15 + "|"]
    for r in rows[:top]:
        out.append(f"| {r['kernel']} | {r['n']} | {r['us']:.1f} | {r['rd']:.2f} | {r['wr']:.2f} | {r['tbs']:.2f} | "
                   f"{r['pct']:.0f} | {r['valu']:.0f} | {r['salu']:.0f} | {r['vmem']:.0f} | {r['active']:.0f} | "
                   f"{r['wait']:.0f} | {r['l2']:.0f} | {r['ldsc']:.1f} | {r['vgpr']} |")
    return "\n".join(out) + "\n", rows


def main():
    out, title, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    vals, durs, meta = load(dirs)
    text, _ = table(vals, durs, meta)
    with open(out, "w") as f:
        f.write(f"# {title}\n\n")
        f.write(__doc__.split("\n\n", 2)[2].strip() + "\n\n")
        f.write(text)


if __name__ == "__main__":
    main()
