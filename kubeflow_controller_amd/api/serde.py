"""YAML/JSON load + dump, ``envsubst`` and the kind registry (the "scheme").

The reference's user flow is ``envsubst < examples/tfjob/dist.yml | kubectl
create -f -`` (``docs/get_started.md:7-63``); ``load_objects(..., env=...)``
performs the same ``$VAR`` substitution before parsing.
"""
from __future__ import annotations

import json
import os
import re
from typing import Any, Dict, Iterable, List, Optional

import yaml

from . import v1alpha1
from .core import Event, Pod, ReplicaSet, Service
from .model import Model

# kind -> class ; (apiVersion check is lenient for core kinds)
SCHEME = {
    v1alpha1.TFJOB_KIND: v1alpha1.TFJob,
    "Pod": Pod,
    "Service": Service,
    "Event": Event,
    "ReplicaSet": ReplicaSet,
}

# plural resource names used by the REST store / CLI
RESOURCES = {
    "tfjobs": v1alpha1.TFJOB_KIND, "tfjob": v1alpha1.TFJOB_KIND, "tfj": v1alpha1.TFJOB_KIND,
    "pods": "Pod", "pod": "Pod", "po": "Pod",
    "services": "Service", "service": "Service", "svc": "Service",
    "events": "Event", "event": "Event", "ev": "Event",
    "replicasets": "ReplicaSet", "replicaset": "ReplicaSet", "rs": "ReplicaSet",
}

_ENV_RE = re.compile(r"\$(\{([A-Za-z_][A-Za-z0-9_]*)\}|([A-Za-z_][A-Za-z0-9_]*))")


def envsubst(text: str, env: Optional[Dict[str, str]] = None) -> str:
    """GNU ``envsubst``: replace ``$VAR`` / ``${VAR}``; unset vars become ``""``."""
    env = os.environ if env is None else env

    def rep(m):
        name = m.group(2) or m.group(3)
        return env.get(name, "")

    return _ENV_RE.sub(rep, text)


def decode(doc: Dict[str, Any]) -> Model:
    kind = doc.get("kind")
    if kind == "CustomResourceDefinition":
        return doc  # type: ignore[return-value]  # accepted, registered by the store
    cls = SCHEME.get(kind)
    if cls is None:
        raise ValueError(f"no kind {kind!r} is registered (known: {sorted(SCHEME)})")
    if kind == v1alpha1.TFJOB_KIND and doc.get("apiVersion", v1alpha1.API_VERSION) != v1alpha1.API_VERSION:
        raise ValueError(f"TFJob apiVersion must be {v1alpha1.API_VERSION!r}, got {doc.get('apiVersion')!r}")
    return cls.from_json(doc)


def load_objects(text: str, *, env: Optional[Dict[str, str]] = None, substitute: bool = True) -> List[Any]:
    """Parse a (multi-document) YAML or JSON string into API objects."""
    if substitute:
        text = envsubst(text, env)
    docs = [d for d in yaml.safe_load_all(text) if d is not None]
    out = []
    for d in docs:
        if d.get("kind", "").endswith("List") and "items" in d:
            out.extend(decode(x) for x in d["items"])
        else:
            out.append(decode(d))
    return out


def load_file(path: str, *, env: Optional[Dict[str, str]] = None, substitute: bool = True) -> List[Any]:
    with open(path) as f:
        return load_objects(f.read(), env=env, substitute=substitute)


def dump_yaml(obj: Any) -> str:
    data = obj.to_json() if isinstance(obj, Model) else obj
    return yaml.safe_dump(data, sort_keys=False)


def dump_json(obj: Any, indent: Optional[int] = 2) -> str:
    data = obj.to_json() if isinstance(obj, Model) else obj
    return json.dumps(data, indent=indent)


def dump_many_yaml(objs: Iterable[Any]) -> str:
    return "---\n".join(dump_yaml(o) for o in objs)
