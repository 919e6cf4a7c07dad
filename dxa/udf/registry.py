"""Build the UDF/UDAF registry of a job from its settings.

Keys (reference handlers): ``datax.job.process.udf.<name>=<class>`` dynamic UDFs (ExtendedUDFHandler.scala:16-104),
``datax.job.process.jar.udf.<name>.class`` / ``jar.udaf.<name>.class`` (JarUDFHandler.scala:14-63),
``datax.job.process.azurefunction.<name>.{serviceendpoint,api,code,methodtype,params}`` (AzureFunctionHandler.scala:
14-65), ``datax.job.process.hipudf.<name>.{source,entry,returntype,argtypes,nullsafe}`` (HIP device functions,
``dxa.udf.hip``), ``datax.job.process.hipudaf.<name>.*`` (HIP device aggregates), plus the built-in ``stringToTimestamp`` / ``filterNull`` which the expression engine implements natively.
"""
from __future__ import annotations

import importlib
from typing import Callable, Dict, List, Tuple

from ..config import settings as S
from ..config.secrets import resolve
from .api import FunctionUDF, Generator, RowUDF, UDAF, VectorUDF
from .samples import REFERENCE_CLASS_MAP


class UdfError(Exception):
    pass


def load_class(name: str):
    if name in REFERENCE_CLASS_MAP:
        return REFERENCE_CLASS_MAP[name]
    if ":" in name:
        mod, attr = name.split(":", 1)
    else:
        mod, _, attr = name.rpartition(".")
    try:
        return getattr(importlib.import_module(mod), attr)
    except (ImportError, AttributeError) as e:
        raise UdfError(f"cannot load UDF class {name!r}: {e}") from e


def _instantiate(name: str):
    obj = load_class(name)
    return obj() if isinstance(obj, type) else obj


def build_udfs(d: S.SettingDictionary, udfs: Dict, udafs: Dict) -> Tuple[Dict, Dict, List[Callable]]:
    out_udfs: Dict[str, object] = {k.lower(): v for k, v in udfs.items()}
    out_udafs: Dict[str, object] = {k.lower(): v for k, v in udafs.items()}
    refreshers: List[Callable] = []
    # dynamic UDFs
    for name, cls in d.sub_dictionary(S.PROCESS_PREFIX + "udf.").items():
        inst = _instantiate(cls)
        if isinstance(inst, Generator):
            fn, on_interval = inst.initialize(d)
            out_udfs[name.lower()] = fn
            if on_interval:
                refreshers.append(on_interval)
        else:
            out_udfs[name.lower()] = inst
    # jar UDFs / UDAFs (Python classes here)
    for name, sub in d.group_by_sub_namespace(S.PROCESS_PREFIX + "jar.udf.").items():
        inst = _instantiate(sub.get_string("class"))
        if isinstance(inst, Generator):
            fn, on_interval = inst.initialize(d)
            inst = fn
            if on_interval:
                refreshers.append(on_interval)
        out_udfs[name.lower()] = inst
    for name, sub in d.group_by_sub_namespace(S.PROCESS_PREFIX + "jar.udaf.").items():
        out_udafs[name.lower()] = _instantiate(sub.get_string("class"))
    # HIP-source device UDFs (the MI355X form of a jar UDF)
    from .hip import from_settings as hip_udf
    for name, sub in d.group_by_sub_namespace(S.PROCESS_PREFIX + "hipudf.").items():
        out_udfs[name.lower()] = hip_udf(name, sub)
    from .hip import udaf_from_settings as hip_udaf
    for name, sub in d.group_by_sub_namespace(S.PROCESS_PREFIX + "hipudaf.").items():
        out_udafs[name.lower()] = hip_udaf(name, sub)
    # HTTP functions
    from .http import HttpFunctionUDF
    for name, sub in d.group_by_sub_namespace(S.PROCESS_PREFIX + "azurefunction.").items():
        params = sub.get_string_seq("params") or []
        if len(params) > 3:
            raise UdfError("AzureFunction with more than 3 input parameters are currently not supported")
        out_udfs[name.lower()] = HttpFunctionUDF(sub.get("serviceendpoint"), sub.get("api"),
                                                 resolve(sub.get("code")), sub.get("methodtype") or "get", params)
    return out_udfs, out_udafs, refreshers
