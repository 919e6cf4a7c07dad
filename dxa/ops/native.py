"""ctypes binding to the in-tree gfx950 kernel library (``dxa/ops/_native/libdxa_kernels.so``).

The library is a plain C ABI over HIP kernels; it is loaded *after* ``import torch`` so its ``libamdhip64.so.7``
dependency resolves (by SONAME) to the HIP runtime torch already mapped — one runtime, one set of streams, and our
kernels run on torch's current stream with torch-allocated HBM buffers.

GPU tensors always take the native path; if the library is missing on a GPU box we raise instead of silently
falling back to slower PyTorch code (``DXA_ALLOW_FALLBACK=1`` is for debugging only).
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import torch

_LIB = None
_LOCK = threading.Lock()
_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("DXA_NATIVE_LIB") or (_HERE / "_native" / "libdxa_kernels.so"))  # override: A/B runs

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_p = ctypes.c_void_p

_SIGS = {
    "dxa_byte_map": [c_p, c_p, c_i64, c_p, c_p],
    "dxa_lz4_block_sizes": [c_p, c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_p],
    "dxa_lz4_decode": [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_p],
    "dxa_memcpy_h2d_async": [c_p, c_p, c_i64, c_p],
    "dxa_copy_sdma": [c_p, c_p, c_i64],
    "dxa_lz4_decode_into": [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_p, c_p],
    "dxa_inflate_into": [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_p, c_p],
    "dxa_snappy_decode_into": [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_p, c_p],
    "dxa_zstd_decode_into": [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_p, c_p],
    "dxa_zstd_decode_prof": [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_p],
    "dxa_kafka_records": [c_p, c_i64] + [c_p] * 14,
    "dxa_kafka_crc": [c_p, c_i64, c_p, c_p, c_p, c_p, c_p],
    "dxa_csv_tokenize": [c_p, c_p, c_i64, c_i32, c_i32, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p],
    "dxa_spark_hash_fixed": [c_p, c_i32, c_p, c_i64, c_p, c_p],
    "dxa_spark_hash_str": [c_p, c_p, c_p, c_p, c_i64, c_p, c_p],
    "dxa_serialize_rows": [c_i32, c_p, c_i32, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p],
    "dxa_java_double_dev": [c_p, c_i64, c_p, c_p, c_p],
    "dxa_java_double_hostcheck": [c_p, c_i64, c_p, c_p],
    "dxa_json_parse": [c_p, c_p, c_i64, c_p, c_p, c_i32, c_p, c_p, c_p, c_i32, c_p, c_p, c_p, c_p,
                       c_p, c_p, c_p, c_p, c_p, c_i32, c_p, c_p, c_p, c_p, c_i32, c_i32, c_i32, c_p, c_i32,
                       c_p],
    "dxa_count_newlines": [c_p, c_i64, c_i64, c_p, c_p, c_p],
    "dxa_write_newlines_bits": [c_p, c_i64, c_i64, c_p, c_p, c_i64, c_i64, c_p],
    "dxa_null_counts": [c_p, c_i64, c_i32, c_p, c_p],
    "dxa_hash_i64": [c_p, c_p, c_i64, c_p, ctypes.c_int, c_p],
    "dxa_hash_f64": [c_p, c_p, c_i64, c_p, ctypes.c_int, c_p],
    "dxa_hash_str": [c_p, c_p, c_p, c_p, c_i64, c_p, ctypes.c_int, c_p],
    "dxa_table_insert": [c_p, c_i64, c_p, c_i64, c_p, c_p],
    "dxa_group_ids": [c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_p],
    "dxa_verify_i64": [c_p, c_p, c_p, c_p, c_i64, c_p, c_p],
    "dxa_verify_str": [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_p],
    "dxa_aggregate": [c_p, c_p, c_p, c_i64, c_i32, c_i32, c_i32, c_p, c_p],
    "dxa_aggregate_multi": [c_p, c_i64, c_i32, c_i32, c_p, c_i32, c_p, c_p, c_p],
    "dxa_aggregate_finish": [c_p, c_i32, c_i32, c_i32, c_p, c_p, c_p, c_p],
    "dxa_partial_finish_size": [],
    "dxa_partial_finish": [c_p, c_p],
    "dxa_group_renumber": [c_p, c_i64, c_p, c_i32, c_p, c_p, c_p],
    "dxa_group_build": [c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_p],
    "dxa_group_build_init": [c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_p],
    "dxa_slot_count": [c_p, c_i64, c_p, c_p],
    "dxa_slot_scatter": [c_p, c_i64, c_p, c_p, c_p, c_p],
    "dxa_probe_count": [c_p, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, ctypes.c_int, c_p],
    "dxa_probe_write": [c_p, c_i64, c_p, c_p, c_p, c_p, c_p, c_p, ctypes.c_int, c_p],
    "dxa_str_cmp_lit": [c_p, c_p, c_p, c_i64, c_p, c_i32, c_i32, c_p, c_p],
    "dxa_str_eq_col": [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_p],
    "dxa_str_cmp_col": [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i32, c_p, c_p],
    "dxa_str_gather": [c_p, c_p, c_p, c_i64, c_p, c_p, c_p],
    "dxa_str_gather_parts": [c_p, c_i32, c_p],
    "dxa_str_split_count": [c_p, c_p, c_p, c_i64, c_p, c_i32, c_p, c_p],
    "dxa_ts_format": [c_p, c_i64, c_p, c_i32, c_p, c_i32, c_p, c_p],
    "dxa_str_like": [c_p, c_p, c_p, c_i64, c_p, c_i32, c_p, c_p],
    "dxa_str_rlike": [c_p, c_p, c_p, c_i64, c_p, c_i32, c_i32, c_i32, c_p, c_p],
    "dxa_str_regex": [c_p, c_p, c_p, c_i64, c_p, c_i32, c_p, c_i32, c_i32, c_i32, c_p, c_i32, c_p, c_p, c_p, c_p, c_p,
                      c_p, c_p],
    "dxa_gzip_chunks": [c_p, c_i64, c_i32, c_p, c_p, c_i32, c_p, c_p],
    "dxa_gzip_pack": [c_p, c_i32, c_p, c_p, c_i64, c_p, c_p],
    "dxa_str_digest": [c_p, c_p, c_p, c_i64, c_i32, c_p, c_p],
    "dxa_str_crc32": [c_p, c_p, c_p, c_i64, c_p, c_p],
    "dxa_str_encode": [c_p, c_p, c_p, c_i64, c_i32, c_p, c_p, c_p],
    "dxa_f64_str_len": [c_p, c_p, c_i64, c_p, c_p],
    "dxa_f64_str_write": [c_p, c_p, c_i64, c_p, c_p, c_p],
    "dxa_str_to_num": [c_p, c_p, c_p, c_p, c_i64, c_i32, c_p, c_p, c_p],
    "dxa_concat_ws_len": [c_p, c_i32, c_i64, c_i32, c_p, c_p],
    "dxa_concat_ws_write": [c_p, c_i32, c_i64, c_p, c_i32, c_p, c_p, c_p],
    "dxa_str_substr": [c_p, c_p, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p],
    "dxa_str_trim": [c_p, c_p, c_p, c_i64, c_i32, c_p, c_p, c_p],
    "dxa_str_numchars": [c_p, c_p, c_p, c_i64, c_p, c_p],
    "dxa_str_locate": [c_p, c_p, c_p, c_i64, c_p, c_i32, c_i64, c_p, c_p],
    "dxa_str_replace_len": [c_p, c_p, c_p, c_i64, c_p, c_i32, c_i32, c_p, c_p],
    "dxa_str_replace_write": [c_p, c_p, c_p, c_i64, c_p, c_i32, c_p, c_i32, c_p, c_p, c_p],
    "dxa_str_split_write": [c_p, c_p, c_p, c_i64, c_p, c_i32, c_i32, c_p, c_p, c_p],
    "dxa_str_part_size": [],
    "dxa_concat_len": [c_p, c_i32, c_i64, c_p, c_p, c_p],
    "dxa_concat_write": [c_p, c_i32, c_i64, c_p, c_p, c_p, c_p],
    "dxa_concat_part_size": [],
    "dxa_i64_to_str_len": [c_p, c_i64, c_p, c_p],
    "dxa_i64_to_str_write": [c_p, c_i64, c_p, c_p, c_p],
    "dxa_i64_to_str_slots": [c_p, c_i64, c_p, c_p, c_p, c_p],
    "dxa_case_map": [c_p, c_p, c_p, c_i64, c_p, c_p, ctypes.c_int, c_p],
    "dxa_str_to_ts": [c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_p],
    "dxa_datagen_op_size": [],
    "dxa_datagen_lengths": [c_p, c_i32, c_p, c_i32, c_p, c_i32, ctypes.c_uint64, c_i64, c_i64, c_i64, c_i64, c_p,
                            c_p],
    "dxa_datagen_write": [c_p, c_i32, c_p, c_i32, c_p, c_i32, ctypes.c_uint64, c_i64, c_i64, c_i64, c_i64, c_p,
                          c_p, c_p],
}

# optional symbols (added by later kernels); bound if present
_OPTIONAL_SIGS = {}


class NativeError(RuntimeError):
    pass


def register_sigs(sigs: dict):
    """Declare argument types for extra symbols; applied immediately if the library is already loaded (an unbound
    ctypes function would silently pass 64-bit arguments as C ints)."""
    _OPTIONAL_SIGS.update(sigs)
    if _LIB is not None:
        for name, args in sigs.items():
            fn = getattr(_LIB, name, None)
            if fn is not None:
                fn.argtypes = args
                fn.restype = ctypes.c_int


def lib():
    """Load (building first if needed and hipcc is present) the kernel library."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        if not LIB_PATH.exists() or os.environ.get("DXA_REBUILD") == "1":
            from .build import build
            build()
        L = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
        for name, args in {**_SIGS, **_OPTIONAL_SIGS}.items():
            fn = getattr(L, name, None)
            if fn is None:
                if name in _SIGS:
                    raise NativeError(f"symbol {name} missing from {LIB_PATH}")
                continue
            fn.argtypes = args
            fn.restype = ctypes.c_int
        _LIB = L
        return L


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def ptr(t) -> int:
    if t is None:
        return 0
    return t.data_ptr()


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_handle(device=None) -> int:
    """The current HIP stream of ``device`` as an integer handle (the raw-stream query skips building a Stream
    object; a few hundred kernel launches per batch go through here)."""
    if _RAW_STREAM is not None:
        idx = getattr(device, "index", None)
        if idx is None:
            idx = torch.device(device).index if isinstance(device, (str, int)) and not isinstance(device, bool) \
                else None
        if idx is None:
            idx = torch.cuda.current_device()
        return _RAW_STREAM(idx)
    return torch.cuda.current_stream(device).cuda_stream


def call(name: str, *args):
    fn = getattr(lib(), name)
    rc = fn(*args)
    if rc != 0:
        raise NativeError(f"{name} failed with HIP error {rc}")
    return rc


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` lives on the GPU (the native HIP path is mandatory there)."""
    if t.is_cuda:
        if os.environ.get("DXA_ALLOW_FALLBACK") == "1" and not available():
            return False
        return True
    return False


def u8(mask):
    """bool mask → uint8 view for kernels (bool and uint8 share the 1-byte layout)."""
    if mask is None:
        return None
    return mask.view(torch.uint8) if mask.dtype == torch.bool else mask


def h2d(data, dtype=None, device="cpu") -> torch.Tensor:
    """Host data (list, bytes or CPU tensor) as a tensor on ``device`` WITHOUT stalling the host.

    On ROCm a blocking host→device copy from pageable memory — ``tensor.to(cuda)``, ``torch.tensor(list,
    device=cuda)`` — returns only after the stream has drained (``tools/gpu/h2d_sync_probe.py``: a 64-byte upload
    behind a 20 ms kernel blocks the host 20 ms), which serialises host planning with device work.  Here the bytes go
    through a pinned staging block from torch's caching host allocator (reused only after the copy ran) and a
    non-blocking copy on the current stream."""
    dev = torch.device(device)
    if isinstance(data, torch.Tensor):
        h = data
    elif isinstance(data, (bytes, bytearray, memoryview)):
        h = torch.frombuffer(bytearray(data), dtype=torch.uint8) if len(data) else torch.empty(0, dtype=torch.uint8)
        if dtype is not None and dtype != torch.uint8:
            h = h.view(dtype)
    else:
        h = torch.tensor(data, dtype=dtype)
    if dev.type != "cuda":
        return h.to(dev)
    if h.numel() == 0:
        return torch.empty(h.shape, dtype=h.dtype, device=dev)
    return h.pin_memory().to(dev, non_blocking=True)
