"""Typed clientset over an object store (``ObjectStore`` in-process or
``RESTStore`` remote).

Mirrors the shape the reference uses:
``tfJobClient.KubeflowV1alpha1().TFJobs(ns).{Create,Update,Delete,Get,List,Watch,Patch}``
(``VCS/clientset/versioned/typed/kubeflow/v1alpha1/tfjob.go:33-153``) and
``kubeClient.CoreV1().{Pods,Services,Events}(ns)``.
"""
from __future__ import annotations

from typing import Dict, List, Optional

from ..api import v1alpha1
from ..api.labels import Selector
from ..api.model import Model


class ResourceClient:
    def __init__(self, store, kind: str, namespace: str):
        self.store = store
        self.kind = kind
        self.namespace = namespace

    def create(self, obj: Model) -> Model:
        return self.store.create(obj, namespace=self.namespace or obj.metadata.namespace or "default")

    def get(self, name: str) -> Model:
        return self.store.get(self.kind, self.namespace or "default", name)

    def list(self, selector: Optional[Selector] = None) -> List[Model]:
        return self.store.list(self.kind, self.namespace or None, selector)

    def update(self, obj: Model) -> Model:
        if not obj.metadata.namespace:
            obj.metadata.namespace = self.namespace or "default"
        return self.store.update(obj)

    def update_status(self, obj: Model) -> Model:
        if not obj.metadata.namespace:
            obj.metadata.namespace = self.namespace or "default"
        return self.store.update_status(obj)

    def patch(self, name: str, patch: Dict, expect_uid: Optional[str] = None) -> Model:
        return self.store.patch(self.kind, self.namespace or "default", name, patch, expect_uid=expect_uid)

    def delete(self, name: str, propagation: str = "Background", expect_uid: Optional[str] = None) -> None:
        self.store.delete(self.kind, self.namespace or "default", name, propagation=propagation, expect_uid=expect_uid)

    def watch(self, selector: Optional[Selector] = None, resource_version: Optional[str] = None):
        return self.store.watch(self.kind, self.namespace or None, selector, resource_version)


class _KubeflowV1alpha1:
    def __init__(self, store):
        self._store = store

    def tfjobs(self, namespace: str = "") -> ResourceClient:
        return ResourceClient(self._store, v1alpha1.TFJOB_KIND, namespace)

    TFJobs = tfjobs


class _CoreV1:
    def __init__(self, store):
        self._store = store

    def pods(self, namespace: str = "") -> ResourceClient:
        return ResourceClient(self._store, "Pod", namespace)

    def services(self, namespace: str = "") -> ResourceClient:
        return ResourceClient(self._store, "Service", namespace)

    def events(self, namespace: str = "") -> ResourceClient:
        return ResourceClient(self._store, "Event", namespace)

    def replica_sets(self, namespace: str = "") -> ResourceClient:
        """extensions/v1beta1 ReplicaSets (served here for the reference's ReplicaSet control)."""
        return ResourceClient(self._store, "ReplicaSet", namespace)

    Pods = pods
    Services = services
    Events = events


class Clientset:
    """Both the "kube" and the "tfjob" clientsets of ``cmd/controller/main.go:36-44``."""

    def __init__(self, store):
        self.store = store
        self._kf = _KubeflowV1alpha1(store)
        self._core = _CoreV1(store)

    def kubeflow_v1alpha1(self) -> _KubeflowV1alpha1:
        return self._kf

    def core_v1(self) -> _CoreV1:
        return self._core

    KubeflowV1alpha1 = kubeflow_v1alpha1
    CoreV1 = core_v1
