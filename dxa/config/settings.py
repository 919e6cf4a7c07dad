"""Flat ``datax.job.*`` settings with typed getters and namespace grouping.

Behavioural parity with the reference's config contracts:
* ``SettingDictionary`` (DataProcessing/datax-core/src/main/scala/datax/config/SettingDictionary.scala:20-150):
  typed getters, ``;``-separated lists, ``group_by_sub_namespace`` / ``sub_dictionary`` stripping prefixes;
* ``SettingNamespace`` (…/SettingNamespace.scala:9-48): ``datax.job.`` root, ``input.default``, ``process``, ``output``;
* ``ConfigManager`` (DataProcessing/datax-host/src/main/scala/datax/config/ConfigManager.scala:61-135):
  ``conf=… driverLogLevel=… executorLogLevel=… checkpointEnabled=…`` arguments, ``DATAX_*`` environment variables,
  ``.conf`` files of ``k=v`` lines with ``#`` comments and ``${TOKEN}`` substitution.
The name prefix (``DataX``) is overridable with ``DATAX_NAMEPREFIX`` (NamePrefix.scala:7-11).
"""
from __future__ import annotations

import os
import re
import threading
from pathlib import Path
from typing import Callable, Dict, Iterable, List, Optional

from ..sql.parser import parse_duration_micros

NAME_PREFIX = os.environ.get("DATAX_NAMEPREFIX", "DataX")
SEP = "."
VALUE_SEP = ";"
ROOT = NAME_PREFIX.lower()
JOB_PREFIX = f"{ROOT}.job."
JOB_NAME = JOB_PREFIX + "name"
INPUT_PREFIX = JOB_PREFIX + "input.default."
PROCESS_PREFIX = JOB_PREFIX + "process."
OUTPUT_PREFIX = JOB_PREFIX + "output."
OUTPUT_DEFAULT_PREFIX = OUTPUT_PREFIX + "default."

ENV_PREFIX = f"{NAME_PREFIX}_".upper()
ARG_APPCONF = ENV_PREFIX + "APPCONF"
ARG_APPNAME = ENV_PREFIX + "APPNAME"
ARG_LOGLEVEL = ENV_PREFIX + "LOGLEVEL"
ARG_DRIVERLOGLEVEL = ENV_PREFIX + "DRIVERLOGLEVEL"
ARG_CHECKPOINT = ENV_PREFIX + "CHECKPOINTENABLED"
ARG_APPINSIGHTKEYREF = ENV_PREFIX + "APPINSIGHTKEYREF"

METRIC_APP_PREFIX = f"{NAME_PREFIX}-".upper()
DEFAULT_APP_NAME = f"{NAME_PREFIX}_Unknown_App"


class SettingError(KeyError):
    pass


def sub_namespace(prop: str, start: int = 0) -> Optional[str]:
    if len(prop) <= start:
        return None
    pos = prop.find(SEP, start)
    return prop[start:pos] if pos >= 0 else prop[start:]


class SettingDictionary:
    def __init__(self, elems: Optional[Dict[str, str]] = None, parent_prefix: str = ""):
        self.dict: Dict[str, str] = dict(elems or {})
        self.parent_prefix = parent_prefix

    # -- getters -------------------------------------------------------------------------------------------------
    def __len__(self):
        return len(self.dict)

    def __contains__(self, key):
        return key in self.dict

    def items(self):
        return self.dict.items()

    def get(self, key: str, default=None):
        return self.dict.get(key, default)

    def get_default(self):
        return self.dict.get("")

    def get_string(self, key: str) -> str:
        if key not in self.dict:
            raise SettingError(f"config setting '{self.parent_prefix + key}' is not found")
        return self.dict[key]

    def get_or_else(self, key: str, default: str) -> str:
        return self.dict.get(key, default)

    def get_int(self, key: str, default: Optional[int] = None) -> Optional[int]:
        v = self.dict.get(key)
        if v is None:
            if default is None and key not in self.dict:
                return None
            return default
        return int(v)

    def get_long(self, key: str) -> int:
        return int(self.get_string(key))

    def get_double(self, key: str, default: Optional[float] = None) -> Optional[float]:
        v = self.dict.get(key)
        return default if v is None else float(v)

    def get_bool(self, key: str, default: Optional[bool] = None) -> Optional[bool]:
        v = self.dict.get(key)
        if v is None:
            return default
        return v.strip().lower() == "true"

    def get_duration_us(self, key: str, default: Optional[int] = None) -> Optional[int]:
        v = self.dict.get(key)
        if v is None:
            if default is None:
                return None
            return default
        return parse_duration_micros(v)

    def get_duration_option(self, key: str) -> Optional[int]:
        return self.get_duration_us(key)

    def get_string_seq(self, key: str) -> Optional[List[str]]:
        v = self.dict.get(key)
        if v is None:
            return None
        seq = [s for s in v.split(VALUE_SEP) if s]
        return seq or None

    # -- namespaces ----------------------------------------------------------------------------------------------
    def _with_prefix(self, prefix: str) -> Dict[str, str]:
        return {k: v for k, v in self.dict.items() if k.startswith(prefix)}

    def sub_dictionary(self, prefix: str) -> "SettingDictionary":
        return SettingDictionary({k[len(prefix):]: v for k, v in self._with_prefix(prefix).items()
                                  if len(k) > len(prefix)}, self.parent_prefix + prefix)

    def group_by_sub_namespace(self, prefix: Optional[str] = None) -> Dict[str, "SettingDictionary"]:
        if prefix:
            sub = {k[len(prefix):]: v for k, v in self._with_prefix(prefix).items() if len(k) > len(prefix)}
        else:
            sub = dict(self.dict)
        groups: Dict[str, Dict[str, str]] = {}
        for k, v in sub.items():
            ns = sub_namespace(k, 0)
            if ns is None:
                continue
            g = groups.setdefault(ns, {})
            if k == ns:
                g[""] = v
            else:
                g[k[len(ns) + 1:]] = v
        return {ns: SettingDictionary(d, self.parent_prefix + ns + SEP) for ns, d in groups.items()}

    def build_config_map(self, builder: Callable[["SettingDictionary", str], object], prefix: Optional[str] = None):
        return {k: builder(v, k) for k, v in self.group_by_sub_namespace(prefix).items()}

    def build_config_iterable(self, builder, prefix: Optional[str] = None):
        return [builder(v, k) for k, v in self.group_by_sub_namespace(prefix).items()]

    # -- job-level conveniences ----------------------------------------------------------------------------------
    def app_name(self) -> str:
        return self.dict.get(ARG_APPNAME, DEFAULT_APP_NAME)

    def job_name(self) -> str:
        return self.dict.get(JOB_NAME, self.app_name())

    def metric_app_name(self) -> str:
        return METRIC_APP_PREFIX + self.job_name()

    def app_conf_file(self) -> Optional[str]:
        return self.dict.get(ARG_APPCONF)

    def checkpoint_enabled(self) -> bool:
        return (self.dict.get(ARG_CHECKPOINT) or "false").lower() == "true"

    def merged(self, other: Dict[str, str]) -> "SettingDictionary":
        d = dict(self.dict)
        d.update(other)
        return SettingDictionary(d, self.parent_prefix)

    def __repr__(self):
        return f"SettingDictionary({len(self.dict)} settings)"


# ---------------------------------------------------------------------------------------------------------------
# ConfigManager equivalent
# ---------------------------------------------------------------------------------------------------------------

_active: Optional[SettingDictionary] = None
_lock = threading.Lock()


def local_env_settings() -> Dict[str, str]:
    return {k: v for k, v in os.environ.items() if k.startswith(ENV_PREFIX)}


def named_args(argv: Iterable[str]) -> Dict[str, str]:
    """``k=v`` command line arguments (reference ArgumentsParser)."""
    out = {}
    for a in argv:
        if "=" in a:
            k, v = a.split("=", 1)
            out[k.strip()] = v.strip()
    return out


def settings_from_arguments(argv: Iterable[str]) -> SettingDictionary:
    args = named_args(argv)
    if "conf" not in args:
        raise SettingError("configuration file is not specified.")
    conv = {ARG_APPCONF: args.get("conf"), ARG_DRIVERLOGLEVEL: args.get("driverLogLevel"),
            ARG_LOGLEVEL: args.get("executorLogLevel"), ARG_CHECKPOINT: args.get("checkpointEnabled")}
    d = local_env_settings()
    d.update(args)
    d.update({k: v for k, v in conv.items() if v is not None})
    sd = SettingDictionary(d)
    set_active(sd)
    return sd


def replace_tokens(src: Optional[str], tokens: Optional[Dict[str, str]]) -> Optional[str]:
    if not tokens or not src:
        return src
    for k, v in tokens.items():
        src = src.replace("${" + k + "}", v)
    return src


def parse_conf_lines(lines: Iterable[str], replacements: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    out = {}
    for line in lines:
        if line is None:
            continue
        s = line.strip()
        if not s or s.startswith("#"):
            continue
        pos = s.find("=")
        if pos == 0:
            k, v = "", s
        elif pos > 0:
            k, v = s[:pos].strip(), s[pos + 1:].strip()
        else:
            k, v = s, None
        out[k.lstrip("﻿")] = replace_tokens(v, replacements)
    return out


def read_conf_file(path: str, replacements: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    if path is None:
        raise SettingError("No conf file is provided")
    if not path.lower().endswith(".conf"):
        raise SettingError("non-conf file is not supported as configuration input")
    from ..io.fs import read_text
    return parse_conf_lines(read_text(path).splitlines(), replacements)


def load_config(settings: Optional[SettingDictionary] = None) -> SettingDictionary:
    d = settings or get_active()
    props = read_conf_file(d.app_conf_file(), d.dict)
    nd = d.merged(props)
    set_active(nd)
    return nd


def get_active() -> SettingDictionary:
    global _active
    with _lock:
        if _active is None:
            _active = SettingDictionary(local_env_settings())
        return _active


def set_active(d: SettingDictionary):
    global _active
    with _lock:
        _active = d
