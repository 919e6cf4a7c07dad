"""Logical data types and Spark ``StructType`` JSON schema (de)serialisation.

Input schemas in DataX are Spark ``DataType.fromJson`` documents (reference: DataProcessing/datax-host/src/main/
scala/datax/input/SchemaFile.scala:22-26), optionally carrying SimulatedData/DataGenerator metadata
(minValue/maxValue/allowedValues/useCurrentTimeMillis, datax-utility/.../DataGenerator.scala:20-26).

Physical mapping (device columns):
  boolean → torch.bool; byte/short/int/long → int64 holding a value of the logical width (Spark's ByteType,
  ShortType, IntegerType, LongType: every operator that can leave the range wraps two's-complement to it —
  ``wrap_int_tensor`` / ``wrap_int_value``); float/double → float64; timestamp → int64 µs since epoch (UTC);
  date → int64 days; string → (arena uint8, starts int64, lens int32); struct/map → child columns;
  array → fixed-arity element columns or raw JSON text.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

SCALAR_TYPES = ("boolean", "byte", "short", "int", "long", "float", "double", "string", "timestamp", "date", "null",
                "binary", "decimal")
INTEGRAL = ("byte", "short", "int", "long")
INT_BITS = {"byte": 8, "short": 16, "int": 32, "long": 64}
INT_RANGE = {t: (-(1 << (b - 1)), (1 << (b - 1)) - 1) for t, b in INT_BITS.items()}
# Spark's simpleString of each logical type (typeof, schema strings, generated column names)
SIMPLE_NAME = {"byte": "tinyint", "short": "smallint", "int": "int", "long": "bigint"}


def wrap_int_value(v: int, dtype: str) -> int:
    """A Python integer reduced to the two's-complement range of ``dtype`` (JVM int/long/short/byte overflow)."""
    b = INT_BITS.get(dtype, 64)
    m = 1 << b
    v = int(v) & (m - 1)
    return v - m if v >= (m >> 1) else v


def wrap_int_tensor(t, dtype: str):
    """An int64 tensor reduced to the range of ``dtype``: the low bits, sign-extended (shift left, arithmetic shift
    right — two elementwise kernels, on the host or the device).  ``long`` is already int64."""
    b = INT_BITS.get(dtype, 64)
    if b == 64:
        return t
    s = 64 - b
    return (t << s) >> s


def int_type_of_value(v: int) -> str:
    """Spark's type of an integer literal: INT when it fits, else BIGINT (larger ones become decimals in the
    parser)."""
    return "int" if INT_RANGE["int"][0] <= v <= INT_RANGE["int"][1] else "long"
FRACTIONAL = ("float", "double", "decimal")
NUMERIC = INTEGRAL + FRACTIONAL


@dataclass(frozen=True)
class StructField:
    name: str
    dtype: Any
    nullable: bool = True
    metadata: Dict[str, Any] = field(default_factory=dict, compare=False, hash=False)


@dataclass(frozen=True)
class StructType:
    fields: tuple

    def names(self):
        return [f.name for f in self.fields]

    def field(self, name: str) -> Optional[StructField]:
        for f in self.fields:
            if f.name == name:
                return f
        low = name.lower()
        for f in self.fields:
            if f.name.lower() == low:
                return f
        return None

    def __str__(self):
        return "struct<" + ",".join(f"{f.name}:{type_str(f.dtype)}" for f in self.fields) + ">"


@dataclass(frozen=True)
class MapType:
    key: Any
    value: Any
    value_contains_null: bool = True

    def __str__(self):
        return f"map<{type_str(self.key)},{type_str(self.value)}>"


@dataclass(frozen=True)
class ArrayType:
    element: Any
    contains_null: bool = True

    def __str__(self):
        return f"array<{type_str(self.element)}>"


def type_str(t) -> str:
    return t if isinstance(t, str) else str(t)


def is_numeric(t) -> bool:
    return isinstance(t, str) and (t in NUMERIC or _is_dec(t))


def _is_dec(t) -> bool:
    from .decimal import is_decimal
    return is_decimal(t)


def is_integral(t) -> bool:
    return isinstance(t, str) and t in INTEGRAL


def is_nested(t) -> bool:
    return isinstance(t, (StructType, MapType, ArrayType))


_SPARK_NAMES = {"integer": "int", "bigint": "long", "smallint": "short", "tinyint": "byte", "real": "float",
                "bool": "boolean", "str": "string", "varchar": "string"}


def from_json_obj(o) -> Any:
    """Spark ``DataType.fromJson`` object → our type."""
    if isinstance(o, str):
        t = _SPARK_NAMES.get(o.lower(), o.lower())
        if t.startswith("decimal"):
            from .decimal import parse_decimal_type
            return parse_decimal_type(t)
        if t not in SCALAR_TYPES:
            raise ValueError(f"unsupported data type {o!r}")
        return t
    kind = o.get("type")
    if kind == "struct":
        return StructType(tuple(StructField(f["name"], from_json_obj(f["type"]), f.get("nullable", True),
                                            f.get("metadata") or {}) for f in o.get("fields", [])))
    if kind == "map":
        return MapType(from_json_obj(o["keyType"]), from_json_obj(o["valueType"]), o.get("valueContainsNull", True))
    if kind == "array":
        return ArrayType(from_json_obj(o["elementType"]), o.get("containsNull", True))
    if isinstance(kind, (str, dict)):
        return from_json_obj(kind)
    raise ValueError(f"unsupported schema node {o!r}")


def schema_from_json(text: str) -> StructType:
    t = from_json_obj(json.loads(text))
    if not isinstance(t, StructType):
        raise ValueError("input schema must be a struct")
    return t


def to_json_obj(t) -> Any:
    if isinstance(t, str):
        return {"int": "integer"}.get(t, t)
    if isinstance(t, StructType):
        return {"type": "struct", "fields": [
            {"name": f.name, "type": to_json_obj(f.dtype), "nullable": f.nullable, "metadata": f.metadata or {}}
            for f in t.fields]}
    if isinstance(t, MapType):
        return {"type": "map", "keyType": to_json_obj(t.key), "valueType": to_json_obj(t.value),
                "valueContainsNull": t.value_contains_null}
    if isinstance(t, ArrayType):
        return {"type": "array", "elementType": to_json_obj(t.element), "containsNull": t.contains_null}
    raise ValueError(t)


def schema_to_json(t: StructType) -> str:
    return json.dumps(to_json_obj(t))


def parse_ddl_schema(text: str) -> StructType:
    """'deviceId long, deviceType string, MaxEventTime Timestamp' (state-table schema syntax,
    reference: Services/DataX.Config/DataX.Config.Test/Resource/jobConfig.conf:45)."""
    fields = []
    depth = 0
    cur = ""
    parts = []
    for ch in text:
        if ch in "<(":
            depth += 1
        elif ch in ">)":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur)
    for p in parts:
        bits = p.strip().split(None, 1)
        if len(bits) != 2:
            raise ValueError(f"bad schema column {p!r}")
        name, ty = bits[0].strip("`"), bits[1].strip()
        fields.append(StructField(name, _ddl_type(ty)))
    return StructType(tuple(fields))


def _ddl_type(ty: str):
    low = ty.strip().lower()
    if low.startswith("array<"):
        return ArrayType(_ddl_type(ty.strip()[6:-1]))
    if low.startswith("map<"):
        inner = ty.strip()[4:-1]
        depth = 0
        for i, ch in enumerate(inner):
            if ch in "<(":
                depth += 1
            elif ch in ">)":
                depth -= 1
            elif ch == "," and depth == 0:
                return MapType(_ddl_type(inner[:i]), _ddl_type(inner[i + 1:]))
        raise ValueError(ty)
    if low.startswith("struct<"):
        inner = ty.strip()[7:-1]
        return parse_ddl_schema(inner.replace(":", " "))
    if low.startswith(("decimal", "numeric", "dec(")) or low == "dec":
        from .decimal import parse_decimal_type
        return parse_decimal_type(low)
    return from_json_obj(low)


def common_type(a, b):
    """Type widening for binary arithmetic/comparison/union (Spark's findTightestCommonType, simplified)."""
    if a == b:
        return a
    if a == "null":
        return b
    if b == "null":
        return a
    if is_numeric(a) and is_numeric(b):
        if _is_dec(a) or _is_dec(b):
            return _wider_decimal(a, b)
        if a in FRACTIONAL or b in FRACTIONAL:
            return "double"
        return a if INT_BITS.get(a, 64) >= INT_BITS.get(b, 64) else b      # the wider integral type
    if {a, b} <= {"timestamp", "date"}:
        return "timestamp"
    if "string" in (a, b) and not is_nested(a) and not is_nested(b):
        return "string"
    return a


def _wider_decimal(a, b):
    """Spark DecimalPrecision.widerDecimalType / findTightestCommonType: a double or float wins; integers take
    part as decimal(10,0) / decimal(20,0)."""
    from .decimal import DecimalType, bounded, is_decimal, of_integral
    if a in ("double", "float") or b in ("double", "float"):
        return "double"
    da = a if is_decimal(a) else of_integral(a)
    db = b if is_decimal(b) else of_integral(b)
    s = max(da.scale, db.scale)
    return bounded(max(da.precision - da.scale, db.precision - db.scale) + s, s)
