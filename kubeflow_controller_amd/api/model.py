"""Minimal JSON-keyed object model.

The reference's API surface is Go structs whose ``json:"..."`` tags are the wire
contract (``VCS/apis/kubeflow/v1alpha1/types.go:30-184``).  This module gives the
same contract in Python: every API class is a dataclass whose fields carry the
exact JSON key, an ``omitempty`` flag and a type used to decode nested objects.

Unknown keys found while decoding are preserved in ``_extra`` so that a
``load -> dump`` round trip of a user's YAML is lossless (the reference keeps
whole ``v1.PodTemplateSpec`` objects; we only model the fields the controller
and the supervisor read).
"""
from __future__ import annotations

import copy
import dataclasses
import typing
from typing import Any, Dict, List, Optional

__all__ = ["Model", "jfield", "to_json", "from_json", "deep_copy"]


def jfield(key: str, default: Any = None, *, omitempty: bool = True, factory=None, ptr: bool = False):
    """Declare a JSON-keyed dataclass field.

    ``ptr=True`` mirrors a Go pointer field: it is omitted only when ``None``,
    so an explicit ``0`` / ``false`` / ``""`` survives a round trip.
    """
    md = {"json": key, "omitempty": omitempty, "ptr": ptr}
    if factory is not None:
        return dataclasses.field(default_factory=factory, metadata=md)
    return dataclasses.field(default=default, metadata=md)


def _is_empty(v: Any) -> bool:
    if v is None:
        return True
    if isinstance(v, (str, list, dict, tuple)) and len(v) == 0:
        return True
    if isinstance(v, bool):
        return v is False
    if isinstance(v, (int, float)) and v == 0:
        return True
    if isinstance(v, Model):
        return v.is_empty()
    return False


class Model:
    """Base class for API dataclasses (subclasses must be ``@dataclass``)."""

    # preserved unknown keys: set per instance by from_json
    def _get_extra(self) -> Dict[str, Any]:
        return self.__dict__.setdefault("_extra", {})

    def is_empty(self) -> bool:
        for f in dataclasses.fields(self):
            if not _is_empty(getattr(self, f.name)):
                return False
        return not self.__dict__.get("_extra")

    def to_json(self) -> Dict[str, Any]:
        out: Dict[str, Any] = {}
        for f in dataclasses.fields(self):
            key = f.metadata.get("json", f.name)
            val = getattr(self, f.name)
            if f.metadata.get("inline"):
                out.update(to_json(val))
                continue
            if val is None:
                if not f.metadata.get("omitempty", True):
                    out[key] = None
                continue
            if f.metadata.get("omitempty", True) and not f.metadata.get("ptr") and _is_empty(val):
                continue
            out[key] = to_json(val)
        extra = self.__dict__.get("_extra")
        if extra:
            for k, v in extra.items():
                out.setdefault(k, copy.deepcopy(v))
        return out

    @classmethod
    def from_json(cls, data: Optional[Dict[str, Any]]):
        if data is None:
            return None
        if isinstance(data, cls):
            return data
        if not isinstance(data, dict):
            raise TypeError(f"{cls.__name__}: expected object, got {type(data).__name__}")
        hints = typing.get_type_hints(cls)
        kwargs = {}
        known = set()
        for f in dataclasses.fields(cls):
            key = f.metadata.get("json", f.name)
            known.add(key)
            if key in data:
                kwargs[f.name] = from_json(hints[f.name], data[key])
        obj = cls(**kwargs)
        extra = {k: copy.deepcopy(v) for k, v in data.items() if k not in known}
        if extra:
            obj.__dict__["_extra"] = extra
        return obj

    def deep_copy(self):
        return deep_copy(self)

    def __eq__(self, other):  # structural equality on the wire form
        if type(self) is not type(other):
            return NotImplemented
        return self.to_json() == other.to_json()

    __hash__ = None  # type: ignore[assignment]


def to_json(v: Any) -> Any:
    if isinstance(v, Model):
        return v.to_json()
    if isinstance(v, list):
        return [to_json(x) for x in v]
    if isinstance(v, tuple):
        return [to_json(x) for x in v]
    if isinstance(v, dict):
        return {str(k): to_json(x) for k, x in v.items()}
    return v


def _unwrap_optional(tp):
    if typing.get_origin(tp) is typing.Union:
        args = [a for a in typing.get_args(tp) if a is not type(None)]
        if len(args) == 1:
            return args[0]
    return tp


def from_json(tp: Any, v: Any) -> Any:
    if v is None:
        return None
    tp = _unwrap_optional(tp)
    origin = typing.get_origin(tp)
    if origin in (list, List):
        (inner,) = typing.get_args(tp) or (Any,)
        return [from_json(inner, x) for x in v]
    if origin in (dict, Dict):
        args = typing.get_args(tp)
        inner = args[1] if len(args) == 2 else Any
        return {k: from_json(inner, x) for k, x in v.items()}
    if isinstance(tp, type) and issubclass(tp, Model):
        return tp.from_json(v)
    if tp is int and isinstance(v, (int, float, str)) and not isinstance(v, bool):
        return int(v)
    if tp is float and isinstance(v, (int, float, str)):
        return float(v)
    if tp is str and not isinstance(v, str):
        return str(v)
    return copy.deepcopy(v)


def deep_copy(obj):
    """Deep copy of an API object (``zz_generated.deepcopy.go`` equivalent)."""
    if isinstance(obj, Model):
        return type(obj).from_json(obj.to_json())
    return copy.deepcopy(obj)
