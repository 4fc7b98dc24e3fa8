"""Minimal Go-encoding/json-compatible dataclass (de)serialisation.

* field names come from ``jf("name", omitempty=...)`` metadata, like Go struct tags;
* ``omitempty`` drops "", 0, False, None, empty list/dict — but NOT nested
  structs (Go never treats a struct value as empty);
* decoding matches keys case-insensitively, as Go's encoding/json does (this is
  how the service's ``hpalogs`` key fills barrelman's ``HpaLogs`` field,
  foremast-barrelman/pkg/client/analyst/analystclient.go:64 vs
  foremast-service/pkg/models/models.go:90).
"""
from __future__ import annotations

import dataclasses
import functools
import typing
from typing import Any


def jf(name: str, omitempty: bool = False, default=dataclasses.MISSING, default_factory=dataclasses.MISSING):
    md = {"json": name, "omitempty": omitempty}
    if default_factory is not dataclasses.MISSING:
        return dataclasses.field(default_factory=default_factory, metadata=md)
    if default is not dataclasses.MISSING:
        return dataclasses.field(default=default, metadata=md)
    return dataclasses.field(metadata=md)


def _empty(v: Any) -> bool:
    if dataclasses.is_dataclass(v):
        return False
    return v is None or v == "" or v is False or (isinstance(v, (int, float)) and not isinstance(v, bool) and v == 0) \
        or (isinstance(v, (list, dict, tuple)) and len(v) == 0)


def to_json(obj: Any) -> Any:
    if dataclasses.is_dataclass(obj):
        out = {}
        for f in dataclasses.fields(obj):
            name = f.metadata.get("json", f.name)
            if name == "-":
                continue
            v = getattr(obj, f.name)
            if f.metadata.get("omitempty") and _empty(v):
                continue
            out[name] = to_json(v)
        return out
    if isinstance(obj, dict):
        return {k: to_json(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [to_json(v) for v in obj]
    return obj


def _ci_get(d: dict, key: str):
    if key in d:
        return True, d[key]
    lk = key.lower()
    for k, v in d.items():
        if isinstance(k, str) and k.lower() == lk:
            return True, v
    return False, None


def _convert(tp, v):
    if v is None:
        return None
    origin = typing.get_origin(tp)
    args = typing.get_args(tp)
    if origin is typing.Union:
        non_none = [a for a in args if a is not type(None)]
        return _convert(non_none[0], v) if non_none else v
    if dataclasses.is_dataclass(tp):
        return from_json(tp, v) if isinstance(v, dict) else tp()
    if origin in (list, typing.List):
        return [_convert(args[0], x) for x in v] if isinstance(v, list) else []
    if origin in (dict, typing.Dict):
        return {k: _convert(args[1], x) for k, x in v.items()} if isinstance(v, dict) else {}
    if tp is float and isinstance(v, (int, float)) and not isinstance(v, bool):
        return float(v)
    if tp is int and isinstance(v, (int, float)) and not isinstance(v, bool):
        return int(v)
    return v


def _str_or_none(v):
    return v


@functools.lru_cache(maxsize=None)
def _converter(tp):
    """The decoder of one field type, resolved once per type (``_convert``
    re-inspected the type on every value: half of a job document's decode)."""
    if tp is str or tp is Any:
        return _str_or_none                     # JSON strings decode as themselves
    origin = typing.get_origin(tp)
    if origin is typing.Union:
        non_none = [a for a in typing.get_args(tp) if a is not type(None)]
        if not non_none:
            return _str_or_none
        inner = _converter(non_none[0])
        return lambda v: None if v is None else inner(v)
    if dataclasses.is_dataclass(tp):
        return lambda v: None if v is None else (from_json(tp, v) if isinstance(v, dict) else tp())
    if origin in (list, typing.List):
        el = _converter(typing.get_args(tp)[0])
        return lambda v: None if v is None else ([el(x) for x in v] if isinstance(v, list) else [])
    if origin in (dict, typing.Dict):
        el = _converter(typing.get_args(tp)[1])
        return lambda v: None if v is None else ({k: el(x) for k, x in v.items()} if isinstance(v, dict) else {})
    if tp is float:                       # (the scalar cases of _convert, without its per-value type inspection)
        return lambda v: float(v) if isinstance(v, (int, float)) and v.__class__ is not bool else v
    if tp is int:
        return lambda v: int(v) if isinstance(v, (int, float)) and v.__class__ is not bool else v
    if origin is None and isinstance(tp, type):
        return _str_or_none                     # bool / other scalars decode as themselves
    return lambda v: _convert(tp, v)


@functools.lru_cache(maxsize=None)
def _plan(cls) -> tuple:
    """(attribute, json key, lower-cased key, decoder) per field — resolved
    once per class (type-hint evaluation dominated decoding otherwise)."""
    hints = typing.get_type_hints(cls)
    out = []
    for f in dataclasses.fields(cls):
        name = f.metadata.get("json", f.name)
        out.append((f.name, name, name.lower(), _converter(hints[f.name])))
    return tuple(out)


def from_json(cls, data: dict):
    if data is None:
        return cls()
    kw = {}
    lower = None
    for attr, name, lname, conv in _plan(cls):
        if name in data:
            kw[attr] = conv(data[name])
            continue
        if lower is None:   # case-insensitive fallback, built once per object
            lower = {k.lower(): v for k, v in data.items() if isinstance(k, str)}
        if lname in lower:
            kw[attr] = conv(lower[lname])
    return cls(**kw)
