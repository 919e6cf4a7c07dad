"""Filesystem helpers (the reference's HadoopClient, DataProcessing/datax-host/src/main/scala/datax/fs/
HadoopClient.scala:33-815): read (gzip-aware), atomic write via temp-then-rename, write with timeout, list.

``wasbs://container@account.blob.<suffix>/path`` URLs whose account key is known (``io/azure.storage_key_for``) go to
Azure Blob storage over its REST API. Every other ``wasbs://``/``hdfs://``/… URI is mapped under ``DXA_FS_ROOT``
(default ``./.dxa_fs``), so reference job configs run unchanged on a single node. Local paths (optional ``file://``
prefix) are used as they are.
"""
from __future__ import annotations

import gzip
import os
import re
import threading
from concurrent.futures import ThreadPoolExecutor, TimeoutError as _Timeout
from pathlib import Path
from typing import List, Optional

_REMOTE = re.compile(r"^(wasbs?|abfss?|hdfs|adl|dbfs|s3a?)://(.*)$", re.I)
_pool = ThreadPoolExecutor(max_workers=5, thread_name_prefix="dxa-fs")


def local_path(path: str) -> Path:
    if path.startswith("file://"):
        return Path(path[7:])
    m = _REMOTE.match(path)
    if m:
        root = Path(os.environ.get("DXA_FS_ROOT", ".dxa_fs"))
        rest = m.group(2).replace("@", "/")
        return root / m.group(1).lower() / rest
    return Path(path)


def _remote(path: str):
    if not _REMOTE.match(path):
        return None
    from .azure import blob_client_for_url
    return blob_client_for_url(path)


def read_bytes(path: str) -> bytes:
    r = _remote(path)
    if r is not None:
        client, container, blob = r
        data = client.get_blob(container, blob)
    else:
        data = local_path(path).read_bytes()
    if path.endswith(".gz") or data[:2] == b"\x1f\x8b":
        data = gzip.decompress(data)
    return data


def read_text(path: str) -> str:
    return read_bytes(path).decode("utf-8-sig")


def read_lines(path: str) -> List[str]:
    return read_text(path).splitlines()


_GZ_CHUNK = 4 << 20
_gz_pool: Optional[ThreadPoolExecutor] = None
_gz_lock = threading.Lock()


def _gz_member(chunk, level: int) -> bytes:
    return gzip.compress(chunk, compresslevel=level, mtime=0)


def gzip_parallel(data, level: int = 6, chunk: int = _GZ_CHUNK) -> bytes:
    """gzip ``data`` as concatenated members compressed in parallel (zlib releases the GIL).  A multi-member gzip
    file is one valid gzip stream to every reader (RFC 1952 §2.2; ``gzip -d``, Java ``GZIPInputStream``, Hadoop's
    codec).  Level 6 is ``java.util.zip.GZIPOutputStream``'s default — what the reference's BlobSinker writes."""
    global _gz_pool
    mv = memoryview(data) if not isinstance(data, memoryview) else data
    n = len(mv)
    if n <= chunk:
        return _gz_member(mv, level)
    with _gz_lock:
        if _gz_pool is None:
            _gz_pool = ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4), thread_name_prefix="dxa-gz")
    parts = list(_gz_pool.map(lambda i: _gz_member(mv[i:i + chunk], level), range(0, n, chunk)))
    return b"".join(parts)


_DIRS_MADE: set = set()


def write_atomic(path: str, data: bytes | str, gzip_it: bool = False, gzipped: bool = False) -> Path:
    """Write to a temp file in the destination folder, then rename (never leaves a partial file).  A blob PUT is
    atomic on the service side, so remote paths are written in one request.  ``gzipped``: ``data`` is already a
    gzip stream (e.g. compressed on the GPU by ops/deflate.py)."""
    if isinstance(data, str):
        data = data.encode("utf-8")
    if gzip_it and not gzipped:
        data = gzip_parallel(data)
    gzip_it = gzip_it or gzipped
    r = _remote(path)
    if r is not None:
        client, container, blob = r
        client.put_blob(container, blob, data, "application/json" if ".json" in path else "application/octet-stream",
                        "gzip" if gzip_it else None)
        return Path(path)
    p = local_path(path)
    parent = str(p.parent)
    if parent not in _DIRS_MADE:
        p.parent.mkdir(parents=True, exist_ok=True)
        _DIRS_MADE.add(parent)
    # a temp name unique per process and thread (no random-name search): every batch's state flip writes one
    tmp = os.path.join(parent, f".{p.name}.{os.getpid()}.{threading.get_ident()}.tmp")
    try:
        fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    except FileNotFoundError:                    # the directory went away since it was made: make it again
        p.parent.mkdir(parents=True, exist_ok=True)
        fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    with os.fdopen(fd, "wb") as f:
        f.write(data)
    os.replace(tmp, p)
    return p


def write_with_timeout(path: str, data: bytes | str, timeout_s: float, gzip_it: bool = False,
                       gzipped: bool = False) -> Path:
    fut = _pool.submit(write_atomic, path, data, gzip_it, gzipped)
    return fut.result(timeout=timeout_s)


def exists(path: str) -> bool:
    r = _remote(path)
    if r is not None:
        client, container, blob = r
        return bool([n for n in client.list_blobs(container, blob) if n == blob or n.startswith(blob.rstrip("/") + "/")])
    return local_path(path).exists()


def list_files(path: str, recursive: bool = False) -> List[str]:
    r = _remote(path)
    if r is not None:
        client, container, blob = r
        prefix = blob.rstrip("/") + "/" if blob else ""
        base = path[: len(path) - len(blob)] if blob else path.rstrip("/") + "/"
        names = client.list_blobs(container, prefix)
        if not recursive:
            names = [n for n in names if "/" not in n[len(prefix):]]
        return sorted(base + n for n in names)
    p = local_path(path)
    if not p.exists():
        return []
    it = p.rglob("*") if recursive else p.iterdir()
    return sorted(str(x) for x in it if x.is_file())


_GLOB = re.compile(r"[*?\[]")


def list_matching(path: str) -> List[str]:
    """Files under ``path`` (HadoopClient.listFiles: a folder is listed recursively, HadoopClient.scala:470-479), or
    matching it when it holds glob characters (``*``, ``?``, ``[…]``; ``**`` crosses folders) — local and remote
    (``wasbs://``) alike, through ``list_files``."""
    m = _GLOB.search(path)
    if m is None:
        r = _remote(path)
        if r is None and local_path(path).is_file():
            return [str(local_path(path))]
        return list_files(path, recursive=True)
    base = path[: path.rfind("/", 0, m.start()) + 1]
    names = list_files(base, recursive=True) if base else []
    rx = glob_regex(str(local_path(path)) if _remote(path) is None else path)
    return sorted(n for n in names if rx.fullmatch(n))


def glob_regex(pattern: str):
    """``*`` / ``?`` stay inside one folder, ``**`` (and ``**/``) crosses folders, ``[…]`` is a character class."""
    out, i = [], 0
    while i < len(pattern):
        ch = pattern[i]
        if pattern.startswith("**/", i):
            out.append("(?:.*/)?")
            i += 3
        elif pattern.startswith("**", i):
            out.append(".*")
            i += 2
        elif ch == "*":
            out.append("[^/]*")
            i += 1
        elif ch == "?":
            out.append("[^/]")
            i += 1
        elif ch == "[" and "]" in pattern[i + 1:]:
            j = pattern.index("]", i + 1)
            body = pattern[i + 1:j]
            out.append("[" + ("^" + body[1:] if body.startswith("!") else body) + "]")
            i = j + 1
        else:
            out.append(re.escape(ch))
            i += 1
    return re.compile("".join(out))


def owned_by_rank(items: List[str], rank: int, world: int) -> List[str]:
    """The share of ``items`` (file paths, partition names) one rank reads: a stable hash of the name modulo the
    world size, so every rank agrees without communicating and a file is read by exactly one rank (SURVEY §2.G X11:
    source partition → rank)."""
    if world <= 1:
        return list(items)
    import zlib
    return [x for x in items if zlib.crc32(x.encode("utf-8")) % world == rank]


def delete(path: str):
    r = _remote(path)
    if r is not None:
        client, container, blob = r
        for n in client.list_blobs(container, blob):
            if n == blob or n.startswith(blob.rstrip("/") + "/"):
                client.delete_blob(container, n)
        return
    p = local_path(path)
    if p.is_dir():
        import shutil
        shutil.rmtree(p)
    elif p.exists():
        p.unlink()
