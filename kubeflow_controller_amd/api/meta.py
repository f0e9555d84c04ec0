"""ObjectMeta / OwnerReference / TypeMeta — the subset of k8s ``metav1`` the
controller relies on.

Reference behaviour re-created here:
* ``metav1.GetControllerOf`` (``VAM/pkg/apis/meta/v1/controller_ref.go:33``)
* controller ownerRef built by ``newControllerRef`` (``pkg/controller/util.go:44-55``)
* ``SimpleNameGenerator`` 5-char suffix (``vendor/k8s.io/kubernetes/pkg/api/v1/generate.go:48-64``)
"""
from __future__ import annotations

import datetime as _dt
import random
from dataclasses import dataclass
from typing import Dict, List, Optional

from .model import Model, jfield

# k8s.io/apimachinery/pkg/util/rand: consonants + digits without look-alikes.
_ALPHANUMS = "bcdfghjklmnpqrstvwxz2456789"
_MAX_NAME_LENGTH = 63
_RANDOM_LENGTH = 5
_MAX_GENERATED_NAME_LENGTH = _MAX_NAME_LENGTH - _RANDOM_LENGTH

_rng = random.SystemRandom()


def rand_string(n: int) -> str:
    return "".join(_rng.choice(_ALPHANUMS) for _ in range(n))


def generate_name(base: str) -> str:
    """``SimpleNameGenerator.GenerateName``: base (truncated) + 5 random chars."""
    if len(base) > _MAX_GENERATED_NAME_LENGTH:
        base = base[:_MAX_GENERATED_NAME_LENGTH]
    return base + rand_string(_RANDOM_LENGTH)


def now_rfc3339() -> str:
    return _dt.datetime.now(_dt.timezone.utc).replace(microsecond=0).strftime("%Y-%m-%dT%H:%M:%SZ")


@dataclass(eq=False)
class OwnerReference(Model):
    apiVersion: str = jfield("apiVersion", "", omitempty=False)
    kind: str = jfield("kind", "", omitempty=False)
    name: str = jfield("name", "", omitempty=False)
    uid: str = jfield("uid", "", omitempty=False)
    controller: Optional[bool] = jfield("controller", None, ptr=True)
    blockOwnerDeletion: Optional[bool] = jfield("blockOwnerDeletion", None, ptr=True)


@dataclass(eq=False)
class ObjectMeta(Model):
    name: str = jfield("name", "")
    generateName: str = jfield("generateName", "")
    namespace: str = jfield("namespace", "")
    selfLink: str = jfield("selfLink", "")
    uid: str = jfield("uid", "")
    resourceVersion: str = jfield("resourceVersion", "")
    generation: int = jfield("generation", 0)
    creationTimestamp: Optional[str] = jfield("creationTimestamp", None)
    deletionTimestamp: Optional[str] = jfield("deletionTimestamp", None)
    labels: Dict[str, str] = jfield("labels", factory=dict)
    annotations: Dict[str, str] = jfield("annotations", factory=dict)
    ownerReferences: List[OwnerReference] = jfield("ownerReferences", factory=list)
    finalizers: List[str] = jfield("finalizers", factory=list)


@dataclass(eq=False)
class ListMeta(Model):
    resourceVersion: str = jfield("resourceVersion", "")


def get_controller_of(obj) -> Optional[OwnerReference]:
    """Return the ownerReference with ``controller: true`` (``GetControllerOf``)."""
    meta = getattr(obj, "metadata", None)
    if meta is None:
        return None
    for ref in meta.ownerReferences:
        if ref.controller:
            return ref
    return None


def key_of(obj) -> str:
    """``cache.MetaNamespaceKeyFunc``: ``ns/name`` (or ``name`` when cluster-scoped)."""
    ns = obj.metadata.namespace
    return f"{ns}/{obj.metadata.name}" if ns else obj.metadata.name


def split_key(key: str):
    """``cache.SplitMetaNamespaceKey``."""
    parts = key.split("/")
    if len(parts) == 1:
        return "", parts[0]
    if len(parts) == 2:
        return parts[0], parts[1]
    raise ValueError(f"unexpected key format: {key!r}")
