"""Build the gfx950 kernel library ``libdxa_kernels.so`` in-tree with hipcc (no JIT cache, so the built object
travels to the GPU box with the repository snapshot).

    python -m dxa.ops.build            # incremental
    python -m dxa.ops.build --force
"""
from __future__ import annotations

import argparse
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
OUT_DIR = HERE / "_native"
LIB = OUT_DIR / "libdxa_kernels.so"
HOST_LIB = OUT_DIR / "libdxa_host.so"
ARCH = os.environ.get("DXA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-Wno-unused-result", "-Wno-unused-command-line-argument"]
LINK_LIBS = ["-lhiprtc", "-lhsa-runtime64"]      # hipRTC (fused expressions, HIP UDFs), ROCr (SDMA copies)
HOST_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-pthread", "-Wall", "-Wno-unused-function"]


def _digest(paths) -> str:
    h = hashlib.sha256()
    for p in sorted(paths):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    h.update(" ".join(HIP_FLAGS + HOST_FLAGS + LINK_LIBS).encode())
    return h.hexdigest()


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build_variant(name: str, defines, csrc: Path = CSRC) -> Path:
    """A/B builds: ``tools/_cmp/libdxa_kernels_<name>.so`` from ``csrc`` with extra ``-D`` defines (loaded by runs
    with ``DXA_NATIVE_LIB``; tools/gpu/gpu_variants.sh)."""
    out = HERE.parent.parent / "tools" / "_cmp"
    out.mkdir(parents=True, exist_ok=True)
    lib = out / f"libdxa_kernels_{name}.so"
    flags = [*HIP_FLAGS, *[f"-D{d}" for d in defines]]

    def compile_one(src: Path):
        obj = out / f"{name}_{src.stem}.o"
        _run([HIPCC, *flags, "-c", str(src), "-o", str(obj), "-I", str(csrc)])
        return obj

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(compile_one, sorted(csrc.glob("*.hip"))))
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), *LINK_LIBS, "-o", str(lib)])
    for o in objs:
        o.unlink(missing_ok=True)
    print(f"[dxa.build] built variant {lib}", file=sys.stderr)
    return lib


def build(force: bool = False, verbose: bool = True) -> Path:
    OUT_DIR.mkdir(exist_ok=True)
    hip_srcs = sorted(CSRC.glob("*.hip"))
    host_srcs = sorted(CSRC.glob("host_*.cpp"))
    headers = sorted(CSRC.glob("*.h"))
    stamp = OUT_DIR / "build.stamp"
    digest = _digest(hip_srcs + host_srcs + headers)
    if not force and LIB.exists() and (HOST_LIB.exists() or not host_srcs) and stamp.exists() and \
            stamp.read_text() == digest:
        return LIB
    objs = []

    def compile_one(src: Path):
        obj = OUT_DIR / (src.stem + ".o")
        _run([HIPCC, *HIP_FLAGS, "-c", str(src), "-o", str(obj), "-I", str(CSRC)])
        return obj

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(compile_one, hip_srcs))
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), *LINK_LIBS, "-o", str(LIB)])
    if host_srcs:
        _run(["g++", *HOST_FLAGS, "-shared", *map(str, host_srcs), "-I", str(CSRC), "-lz", "-ldl", "-o", str(HOST_LIB)])
    for o in objs:
        o.unlink(missing_ok=True)
    stamp.write_text(digest)
    if verbose:
        print(f"[dxa.build] built {LIB.name} ({len(hip_srcs)} HIP sources, arch {ARCH})"
              + (f" and {HOST_LIB.name}" if host_srcs else ""), file=sys.stderr)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--variant", help="build tools/_cmp/libdxa_kernels_<VARIANT>.so instead")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra define for --variant")
    ap.add_argument("--csrc", default=str(CSRC), help="source folder for --variant")
    args = ap.parse_args()
    if args.variant:
        build_variant(args.variant, args.defines, Path(args.csrc))
        sys.exit(0)
    build(force=args.force)
