"""Runtime compilation of generated HIP kernels (hipRTC → gfx950 code object → module launch on torch's stream).

The engine's analogue of Spark's whole-stage codegen (the reference's expressions run through JVM codegen inside
``spark.sql``, DataProcessing/datax-host/src/main/scala/datax/processor/CommonProcessorFactory.scala:253-289): a
fused expression (``dxa.engine.jit``) becomes one HIP kernel, compiled once per expression shape and cached —
in memory per process and on disk by source hash (``$DXA_JIT_CACHE``, default ``~/.cache/dxa/jit``), so a restarted
job does not pay the compile again.

``host_compile`` builds the same generated row body as a CPU shared object with g++, so the code generator's
semantics are testable on machines without a GPU.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess
import tempfile
import threading
from pathlib import Path
from typing import Dict, List, Optional, Tuple

from . import native as N

ARCH = os.environ.get("DXA_OFFLOAD_ARCH", "gfx950")
_LOCK = threading.Lock()
_FUNCS: Dict[Tuple[str, str], ctypes.c_void_p] = {}
_HOST: Dict[str, ctypes.CDLL] = {}
_BOUND = False
STATS = {"compiles": 0, "disk_hits": 0, "launches": 0}


class RtcError(RuntimeError):
    pass


def _bind():
    global _BOUND
    if _BOUND:
        return N.lib()
    L = N.lib()
    p, i64, u32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint32
    L.dxa_rtc_compile.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                  ctypes.POINTER(p), ctypes.POINTER(i64), ctypes.c_char_p, i64]
    L.dxa_rtc_compile.restype = ctypes.c_int
    L.dxa_rtc_free.argtypes = [p]
    L.dxa_rtc_free.restype = None
    L.dxa_rtc_version.argtypes = []
    L.dxa_rtc_version.restype = ctypes.c_int
    L.dxa_rtc_options.argtypes = []
    L.dxa_rtc_options.restype = ctypes.c_char_p
    L.dxa_module_load.argtypes = [p, ctypes.POINTER(p)]
    L.dxa_module_load.restype = ctypes.c_int
    L.dxa_module_function.argtypes = [p, ctypes.c_char_p, ctypes.POINTER(p)]
    L.dxa_module_function.restype = ctypes.c_int
    L.dxa_module_launch.argtypes = [p, u32, u32, p, p]
    L.dxa_module_launch.restype = ctypes.c_int
    _BOUND = True
    return L


def cache_dir() -> Path:
    d = Path(os.environ.get("DXA_JIT_CACHE", os.path.join(os.path.expanduser("~"), ".cache", "dxa", "jit")))
    d.mkdir(parents=True, exist_ok=True)
    return d


_TOOLCHAIN: Optional[str] = None
# bump when the generated-code ABI (kernel argument layout of dxa/engine/jit.py) changes
CODEGEN_ABI = 2


def toolchain_id() -> str:
    """hipRTC version + fixed compile options of ``dxa_rtc_compile``: a toolchain upgrade invalidates the cache."""
    global _TOOLCHAIN
    if _TOOLCHAIN is None:
        L = _bind()
        _TOOLCHAIN = f"hiprtc{L.dxa_rtc_version()}|{L.dxa_rtc_options().decode()}|abi{CODEGEN_ABI}"
    return _TOOLCHAIN


def source_digest(src: str, name: str = "", extra_opts: str = "") -> str:
    key = f"{ARCH}\0{toolchain_id()}\0{extra_opts}\0{name}\0{src}"
    return hashlib.sha256(key.encode()).hexdigest()[:32]


def compile_code_object(src: str, name: str) -> bytes:
    """hipRTC-compile ``src`` → gfx950 code object bytes (disk-cached by source hash).  Works without a GPU."""
    path = None
    try:
        path = cache_dir() / f"{source_digest(src, name)}.co"
        if path.exists():
            STATS["disk_hits"] += 1
            return path.read_bytes()
    except OSError:
        path = None
    L = _bind()
    code, size = ctypes.c_void_p(), ctypes.c_int64()
    log = ctypes.create_string_buffer(16384)
    rc = L.dxa_rtc_compile(src.encode(), name.encode(), ARCH.encode(), b"", ctypes.byref(code), ctypes.byref(size),
                           log, len(log))
    if rc != 0:
        raise RtcError(f"hipRTC compile of {name} failed ({rc}):\n{log.value.decode(errors='replace')}\n{src}")
    try:
        data = ctypes.string_at(code, size.value)
    finally:
        L.dxa_rtc_free(code)
    STATS["compiles"] += 1
    if path is not None:
        try:
            tmp = path.with_suffix(f".{os.getpid()}.tmp")
            tmp.write_bytes(data)
            os.replace(tmp, path)
        except OSError:
            pass
    return data


def function(src: str, name: str) -> ctypes.c_void_p:
    """Loaded kernel handle for (``src``, ``name``) — compiled and module-loaded once per process."""
    key = (hashlib.sha256(src.encode()).hexdigest(), name)      # in-process: the toolchain cannot change
    fn = _FUNCS.get(key)
    if fn is not None:
        return fn
    with _LOCK:
        fn = _FUNCS.get(key)
        if fn is not None:
            return fn
        image = compile_code_object(src, name)
        L = _bind()
        buf = ctypes.create_string_buffer(image, len(image))
        mod, f = ctypes.c_void_p(), ctypes.c_void_p()
        rc = L.dxa_module_load(buf, ctypes.byref(mod))
        if rc != 0:
            raise RtcError(f"hipModuleLoadData failed ({rc}) for {name}")
        rc = L.dxa_module_function(mod, name.encode(), ctypes.byref(f))
        if rc != 0:
            raise RtcError(f"hipModuleGetFunction failed ({rc}) for {name}")
        _FUNCS[key] = f
        return f


def launch(fn: ctypes.c_void_p, grid: int, block: int, stream: int, args: List[ctypes._SimpleCData]):
    """Launch with kernel arguments given as ctypes scalars (c_int64 / c_void_p), in declaration order."""
    params = (ctypes.c_void_p * len(args))(*[ctypes.cast(ctypes.pointer(a), ctypes.c_void_p) for a in args])
    rc = _bind().dxa_module_launch(fn, grid, block, ctypes.c_void_p(stream), params)
    STATS["launches"] += 1
    if rc != 0:
        raise RtcError(f"hipModuleLaunchKernel failed ({rc})")


def host_compile(src: str) -> ctypes.CDLL:
    """Compile a plain C++ translation unit into a CPU shared object (tests of generated code without a GPU)."""
    key = hashlib.sha256(("host\0" + src).encode()).hexdigest()[:32]
    lib = _HOST.get(key)
    if lib is not None:
        return lib
    d = Path(tempfile.mkdtemp(prefix="dxa_jit_host_"))
    cpp, so = d / "k.cpp", d / "k.so"
    cpp.write_text(src)
    r = subprocess.run(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", str(cpp), "-o", str(so)],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RtcError(f"host compile failed:\n{r.stderr}\n{src}")
    lib = ctypes.CDLL(str(so))
    _HOST[key] = lib
    return lib
