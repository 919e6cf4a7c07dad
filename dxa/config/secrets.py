"""Secret references ``keyvault://<vault>/<secret>`` and ``secretscope://<scope>/<key>`` (reference:
DataProcessing/datax-host/src/main/scala/datax/securedsetting/KeyVaultClient.scala:19-133).

Resolution order, cached per process: environment variable ``DXA_SECRET_<VAULT>_<SECRET>`` (non-alphanumerics →
``_``, upper-case), then the JSON file ``$DXA_SECRETS_FILE`` (``{"vault/secret": "value"}``), then the local
secret directory ``$DXA_SECRETS_DIR/<vault>/<secret>``, then — for ``keyvault://`` when ``DXA_KEYVAULT_URL`` is
set — Azure Key Vault over REST (``keyvault.py``: MSI or client-credentials token).  Unresolvable references raise.
"""
from __future__ import annotations

import json
import os
import re
import threading
from pathlib import Path
from typing import Dict, Optional

_REF = re.compile(r"^(keyvault|secretscope)://([^/]+)/(.+)$")
_cache: Dict[str, str] = {}
_lock = threading.Lock()


class SecretError(KeyError):
    pass


def is_secret_ref(v: Optional[str]) -> bool:
    return bool(v) and _REF.match(v) is not None


def _env_name(vault: str, name: str) -> str:
    return "DXA_SECRET_" + re.sub(r"[^A-Za-z0-9]", "_", f"{vault}_{name}").upper()


def resolve(value: Optional[str]) -> Optional[str]:
    if not is_secret_ref(value):
        return value
    with _lock:
        if value in _cache:
            return _cache[value]
    _, vault, name = _REF.match(value).groups()
    out = os.environ.get(_env_name(vault, name))
    if out is None and os.environ.get("DXA_SECRETS_FILE"):
        try:
            out = json.loads(Path(os.environ["DXA_SECRETS_FILE"]).read_text()).get(f"{vault}/{name}")
        except (OSError, ValueError):
            out = None
    if out is None:
        p = Path(os.environ.get("DXA_SECRETS_DIR", ".dxa_secrets")) / vault / name
        if p.exists():
            out = p.read_text().strip()
    if out is None and value.startswith("keyvault://"):
        from .keyvault import KeyVaultError, default_client
        kv = default_client()
        if kv is not None:
            try:
                out = kv.get_secret(vault, name)
            except KeyVaultError as e:
                raise SecretError(f"cannot resolve secret {value}: {e}") from None
    if out is None:
        raise SecretError(f"cannot resolve secret {value}")
    with _lock:
        _cache[value] = out
    return out


def store(vault: str, name: str, value: str) -> str:
    """Write a secret to the local secret directory and return its reference (used by config generation)."""
    p = Path(os.environ.get("DXA_SECRETS_DIR", ".dxa_secrets")) / vault / name
    p.parent.mkdir(parents=True, exist_ok=True)
    p.write_text(value)
    ref = f"keyvault://{vault}/{name}"
    with _lock:
        _cache[ref] = value
    return ref


def delete_prefix(vault: str, prefix: str) -> int:
    """Remove every secret of ``vault`` whose name starts with ``prefix`` (flow deletion; DataX.Flow.DeleteHelper)."""
    d = Path(os.environ.get("DXA_SECRETS_DIR", ".dxa_secrets")) / vault
    n = 0
    if d.is_dir():
        for p in d.iterdir():
            if p.name.startswith(prefix):
                p.unlink()
                n += 1
                with _lock:
                    _cache.pop(f"keyvault://{vault}/{p.name}", None)
    return n
