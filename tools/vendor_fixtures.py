#!/usr/bin/env python3
"""Copy the reference's golden test DATA (JSON / text / conf / CSV / XML templates — no source code) that the CPU
suite checks against into ``tests/fixtures/ref/<same relative path>``, so the suite runs in any checkout without
the read-only reference mount.  Re-run after the reference changes:

    python tools/vendor_fixtures.py [/root/reference]
"""
import glob
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEST = os.path.join(ROOT, "tests", "fixtures", "ref")

PATTERNS = [
    # rules codegen goldens (CodegenTests.cs cases; the .cs file itself is not needed)
    "Services/DataX.Flow/DataX.Flow.CodegenRules.Tests/*.txt",
    "Services/DataX.Flow/DataX.Flow.CodegenRules.Tests/*.json",
    "Services/DataX.Flow/DataX.Flow.CodegenRules.Tests/*.xml",
    # config generation / flattener goldens
    "Services/DataX.Config/DataX.Config.Test/Resource/*.json",
    "Services/DataX.Config/DataX.Config.Test/Resource/*.conf",
    "Services/DataX.Config/DataX.Config.Test/Resource/*.txt",
    "Services/DataX.Config/DataX.Config.Test/Resource/Flattener/*",
    # onebox sample flows + reference data
    "DeploymentLocal/sample/*.json",
    "DeploymentCloud/Deployment.DataX/Samples/usercontent/devices.csv",
    # SimulatedData seeded-RNG goldens
    "Services/DataX.SimulatedData/DataX.SimulatedData.DataGenServiceTest/*.json",
]


def main(ref="/root/reference"):
    n = 0
    for pat in PATTERNS:
        for src in sorted(glob.glob(os.path.join(ref, pat))):
            if not os.path.isfile(src):
                continue
            rel = os.path.relpath(src, ref)
            dst = os.path.join(DEST, rel)
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            shutil.copyfile(src, dst)
            n += 1
    print(f"vendored {n} fixture files into {os.path.relpath(DEST, ROOT)}")


if __name__ == "__main__":
    main(*sys.argv[1:])
