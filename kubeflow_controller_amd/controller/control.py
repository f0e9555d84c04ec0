"""Pod (replica process) and Service (endpoint) control.

* ``RealPodControl`` — ``VKC/controller_utils.go:441-605``:
  ``create_pods_with_controller_ref`` validates the owner ref, builds the pod
  from the template (``GetPodFromTemplate``: copies labels / finalizers /
  annotations, adds ``kubernetes.io/created-by``, ``generateName =
  "<tfjob>-"``, appends the owner ref, deep-copies the spec), POSTs it and
  records ``Normal SuccessfulCreate "Created pod: <name>"`` or
  ``Warning FailedCreate "Error creating: <err>"``.
* ``RealServiceControl`` — ``pkg/controller/control/service.go:32-80``: same
  for Services (requires non-empty labels) with ``"Created service: <name>"``.
* ``FakePodControl`` / ``FakeServiceControl`` — test doubles recording
  templates / owner refs / patches, with injectable ``err`` and
  ``create_limit`` (``VKC/controller_utils.go:622-709``).

Here a Pod *is* a replica process: the supervisor (``kubelet/``) turns it into
one process pinned to its GPU(s).
"""
from __future__ import annotations

import json
import threading
from typing import Dict, List, Optional

from ..utils import metrics
from ..api.core import CREATED_BY_ANNOTATION, Pod, PodTemplateSpec, Service
from ..api.meta import ObjectMeta, OwnerReference
from ..api.model import deep_copy
from ..client.events import NORMAL, WARNING

# event reasons (VKC/controller_utils.go:384-397, control/types.go:17-26)
FAILED_CREATE_POD_REASON = "FailedCreate"
SUCCESSFUL_CREATE_POD_REASON = "SuccessfulCreate"
FAILED_DELETE_POD_REASON = "FailedDelete"
SUCCESSFUL_DELETE_POD_REASON = "SuccessfulDelete"
FAILED_CREATE_SERVICE_REASON = "FailedCreate"
SUCCESSFUL_CREATE_SERVICE_REASON = "SuccessfulCreate"
FAILED_DELETE_SERVICE_REASON = "FailedDelete"
FAILED_CREATE_REPLICASET_REASON = "FailedCreate"
SUCCESSFUL_CREATE_REPLICASET_REASON = "SuccessfulCreate"
SUCCESSFUL_DELETE_SERVICE_REASON = "SuccessfulDelete"


def validate_controller_ref(ref: Optional[OwnerReference]) -> None:
    """``validateControllerRef`` (``control/util.go:22-39``)."""
    if ref is None:
        raise ValueError("controllerRef is nil")
    if not ref.apiVersion:
        raise ValueError("controllerRef has empty APIVersion")
    if not ref.kind:
        raise ValueError("controllerRef has empty Kind")
    if not ref.controller:
        raise ValueError("controllerRef.Controller is not set to true")
    if not ref.blockOwnerDeletion:
        raise ValueError("controllerRef.BlockOwnerDeletion is not set")


def _created_by(owner) -> str:
    return json.dumps({"kind": "SerializedReference", "apiVersion": "v1",
                       "reference": {"kind": owner.kind, "namespace": owner.metadata.namespace,
                                     "name": owner.metadata.name, "uid": owner.metadata.uid,
                                     "apiVersion": owner.apiVersion,
                                     "resourceVersion": owner.metadata.resourceVersion}})


def get_pod_from_template(template: PodTemplateSpec, parent, controller_ref: Optional[OwnerReference]) -> Pod:
    t = deep_copy(template)
    meta = ObjectMeta(labels=dict(t.metadata.labels), annotations=dict(t.metadata.annotations),
                      finalizers=list(t.metadata.finalizers), generateName=f"{parent.metadata.name}-")
    meta.annotations[CREATED_BY_ANNOTATION] = _created_by(parent)
    if controller_ref is not None:
        meta.ownerReferences.append(deep_copy(controller_ref))
    return Pod(metadata=meta, spec=t.spec)


class RealPodControl:
    def __init__(self, clientset, recorder):
        self.client = clientset
        self.recorder = recorder

    def create_pods(self, namespace: str, template: PodTemplateSpec, parent) -> Pod:
        return self._create(namespace, template, parent, None)

    def create_pods_with_controller_ref(self, namespace: str, template: PodTemplateSpec, parent,
                                        controller_ref: OwnerReference) -> Pod:
        validate_controller_ref(controller_ref)
        return self._create(namespace, template, parent, controller_ref)

    def _create(self, namespace, template, parent, controller_ref) -> Pod:
        pod = get_pod_from_template(template, parent, controller_ref)
        if not pod.metadata.labels:
            raise ValueError("unable to create pods, no labels")
        try:
            created = self.client.core_v1().pods(namespace).create(pod)
        except Exception as e:
            self.recorder.event(parent, WARNING, FAILED_CREATE_POD_REASON, f"Error creating: {e}")
            metrics.CHILDREN_CREATED.labels("Pod", "failure").inc()
            raise
        self.recorder.event(parent, NORMAL, SUCCESSFUL_CREATE_POD_REASON, f"Created pod: {created.metadata.name}")
        metrics.CHILDREN_CREATED.labels("Pod", "success").inc()
        return created

    def delete_pod(self, namespace: str, name: str, parent) -> None:
        try:
            self.client.core_v1().pods(namespace).delete(name)
        except Exception as e:
            self.recorder.event(parent, WARNING, FAILED_DELETE_POD_REASON, f"Error deleting: {e}")
            raise
        self.recorder.event(parent, NORMAL, SUCCESSFUL_DELETE_POD_REASON, f"Deleted pod: {name}")

    def patch_pod(self, namespace: str, name: str, patch: Dict, expect_uid: Optional[str] = None) -> Pod:
        return self.client.core_v1().pods(namespace).patch(name, patch, expect_uid=expect_uid)


class RealServiceControl:
    def __init__(self, clientset, recorder):
        self.client = clientset
        self.recorder = recorder

    def patch_service(self, namespace: str, name: str, patch: Dict, expect_uid: Optional[str] = None) -> Service:
        return self.client.core_v1().services(namespace).patch(name, patch, expect_uid=expect_uid)

    def create_services(self, namespace: str, service: Service, parent) -> Service:
        return self._create(namespace, service, parent, None)

    def create_services_with_controller_ref(self, namespace: str, service: Service, parent,
                                            controller_ref: OwnerReference) -> Service:
        validate_controller_ref(controller_ref)
        return self._create(namespace, service, parent, controller_ref)

    def _create(self, namespace, service, parent, controller_ref) -> Service:
        if not service.metadata.labels:
            raise ValueError("unable to create Services, no labels")
        svc = deep_copy(service)
        if controller_ref is not None:
            svc.metadata.ownerReferences.append(deep_copy(controller_ref))
        try:
            created = self.client.core_v1().services(namespace).create(svc)
        except Exception as e:
            self.recorder.event(parent, WARNING, FAILED_CREATE_SERVICE_REASON, f"Error creating: {e}")
            metrics.CHILDREN_CREATED.labels("Service", "failure").inc()
            raise
        metrics.CHILDREN_CREATED.labels("Service", "success").inc()
        self.recorder.event(parent, NORMAL, SUCCESSFUL_CREATE_SERVICE_REASON,
                            f"Created service: {created.metadata.name}")
        return created

    def delete_service(self, namespace: str, name: str, parent) -> None:
        try:
            self.client.core_v1().services(namespace).delete(name)
        except Exception as e:
            self.recorder.event(parent, WARNING, FAILED_DELETE_SERVICE_REASON, f"Error deleting: {e}")
            raise
        self.recorder.event(parent, NORMAL, SUCCESSFUL_DELETE_SERVICE_REASON, f"Deleted service: {name}")


class FakePodControl:
    """Records what would be created; ``err`` fails every create, ``create_limit``
    fails creates beyond N (``VKC/controller_utils.go:622-709``)."""

    def __init__(self, err: Optional[Exception] = None, create_limit: int = 0):
        self.lock = threading.Lock()
        self.templates: List[PodTemplateSpec] = []
        self.controller_refs: List[OwnerReference] = []
        self.delete_pod_names: List[str] = []
        self.patches: List[Dict] = []
        self.err = err
        self.create_limit = create_limit
        self.create_call_count = 0

    def create_pods_with_controller_ref(self, namespace, template, parent, controller_ref):
        with self.lock:
            self.create_call_count += 1
            if self.create_limit and self.create_call_count > self.create_limit:
                raise RuntimeError(f"not creating pod, limit {self.create_limit} already reached "
                                   f"(create call {self.create_call_count})")
            self.templates.append(deep_copy(template))
            self.controller_refs.append(deep_copy(controller_ref))
            if self.err:
                raise self.err

    def create_pods(self, namespace, template, parent):
        with self.lock:
            self.templates.append(deep_copy(template))
            if self.err:
                raise self.err

    def delete_pod(self, namespace, name, parent):
        with self.lock:
            if self.err:
                raise self.err
            self.delete_pod_names.append(name)

    def patch_pod(self, namespace, name, patch, expect_uid=None):
        with self.lock:
            self.patches.append(patch)
            if self.err:
                raise self.err

    def clear(self):
        with self.lock:
            self.templates.clear()
            self.controller_refs.clear()
            self.delete_pod_names.clear()
            self.patches.clear()
            self.create_call_count = 0


class FakeServiceControl:
    def __init__(self, err: Optional[Exception] = None):
        self.lock = threading.Lock()
        self.services: List[Service] = []
        self.controller_refs: List[OwnerReference] = []
        self.patches: List[Dict] = []
        self.err = err

    def create_services_with_controller_ref(self, namespace, service, parent, controller_ref):
        with self.lock:
            self.services.append(deep_copy(service))
            self.controller_refs.append(deep_copy(controller_ref))
            if self.err:
                raise self.err

    def create_services(self, namespace, service, parent):
        with self.lock:
            self.services.append(deep_copy(service))
            if self.err:
                raise self.err

    def patch_service(self, namespace, name, patch, expect_uid=None):
        with self.lock:
            self.patches.append(patch)
            if self.err:
                raise self.err

    def delete_service(self, namespace, name, parent):
        if self.err:
            raise self.err


class RealReplicaSetControl:
    """ReplicaSet control (reference ``pkg/controller/control/replicaset.go:31-79``).

    Dead code in the reference — never referenced by the controller — kept for
    API parity: create (with an optional controller ref) and patch, with the
    same SuccessfulCreate / FailedCreate events."""

    def __init__(self, clientset, recorder):
        self.client = clientset
        self.recorder = recorder

    def patch_replica_set(self, namespace: str, name: str, patch: Dict, expect_uid: Optional[str] = None):
        return self.client.core_v1().replica_sets(namespace).patch(name, patch, expect_uid=expect_uid)

    def create_replica_sets(self, namespace: str, rs, parent):
        return self._create(namespace, rs, parent, None)

    def create_replica_sets_with_controller_ref(self, namespace: str, rs, parent, controller_ref: OwnerReference):
        validate_controller_ref(controller_ref)
        return self._create(namespace, rs, parent, controller_ref)

    def _create(self, namespace, rs, parent, controller_ref):
        if not rs.spec.template.metadata.labels:
            raise ValueError("unable to create ReplicaSet, no labels")
        obj = deep_copy(rs)
        if controller_ref is not None:
            obj.metadata.ownerReferences.append(deep_copy(controller_ref))
        try:
            created = self.client.core_v1().replica_sets(namespace).create(obj)
        except Exception as e:
            self.recorder.event(parent, WARNING, FAILED_CREATE_REPLICASET_REASON, f"Error creating: {e}")
            raise
        self.recorder.event(parent, NORMAL, SUCCESSFUL_CREATE_REPLICASET_REASON,
                            f"Created replicaset: {created.metadata.name}")
        return created
