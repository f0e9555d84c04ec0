"""Core (``k8s.io/api/core/v1``) objects, re-cut for a single-node process world.

A ``Pod`` is one replica *process*; its ``status.phase`` follows the exit code of
that process (``0 -> Succeeded``, ``!=0 -> Failed``).  A ``Service`` is an
endpoint record: the endpoint controller gives it a ``clusterIP`` of
``127.0.0.1`` and a host port, and the supervisor resolves the service name to
that address when it starts a replica (the role kube-dns plays for the
reference, ``pkg/tensorflow/distributed.go:127-188``).

Only fields the controller, supervisor or trainer read are modelled; anything
else in a user's template round-trips through ``Model._extra``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

from .meta import ObjectMeta
from .model import Model, jfield

# Pod phases (k8s.io/api/core/v1 PodPhase)
POD_PENDING = "Pending"
POD_RUNNING = "Running"
POD_SUCCEEDED = "Succeeded"
POD_FAILED = "Failed"
POD_UNKNOWN = "Unknown"

# RestartPolicy
RESTART_ALWAYS = "Always"
RESTART_ON_FAILURE = "OnFailure"
RESTART_NEVER = "Never"

# Resource name used to request MI355X GPUs in a container's limits.
GPU_RESOURCE = "amd.com/gpu"

# Annotation set by GetPodFromTemplate (vendor/k8s.io/api/core/v1/annotation_key_constants.go:52)
CREATED_BY_ANNOTATION = "kubernetes.io/created-by"


@dataclass(eq=False)
class EnvVar(Model):
    name: str = jfield("name", "", omitempty=False)
    value: str = jfield("value", "")


@dataclass(eq=False)
class ContainerPort(Model):
    name: str = jfield("name", "")
    containerPort: int = jfield("containerPort", 0, omitempty=False)
    protocol: str = jfield("protocol", "")


@dataclass(eq=False)
class ResourceRequirements(Model):
    limits: Dict[str, str] = jfield("limits", factory=dict)
    requests: Dict[str, str] = jfield("requests", factory=dict)


@dataclass(eq=False)
class Container(Model):
    name: str = jfield("name", "", omitempty=False)
    image: str = jfield("image", "")
    command: List[str] = jfield("command", factory=list)
    args: List[str] = jfield("args", factory=list)
    workingDir: str = jfield("workingDir", "")
    env: List[EnvVar] = jfield("env", factory=list)
    ports: List[ContainerPort] = jfield("ports", factory=list)
    resources: Optional[ResourceRequirements] = jfield("resources", None)


@dataclass(eq=False)
class PodSpec(Model):
    containers: List[Container] = jfield("containers", factory=list, omitempty=False)
    restartPolicy: str = jfield("restartPolicy", "")
    nodeName: str = jfield("nodeName", "")
    terminationGracePeriodSeconds: Optional[int] = jfield("terminationGracePeriodSeconds", None, ptr=True)


@dataclass(eq=False)
class PodTemplateSpec(Model):
    metadata: ObjectMeta = jfield("metadata", factory=ObjectMeta)
    spec: PodSpec = jfield("spec", factory=PodSpec)

    @property
    def labels(self) -> Dict[str, str]:
        return self.metadata.labels

    @labels.setter
    def labels(self, v: Dict[str, str]) -> None:
        self.metadata.labels = v


@dataclass(eq=False)
class ContainerStateTerminated(Model):
    exitCode: int = jfield("exitCode", 0, omitempty=False)
    signal: int = jfield("signal", 0)
    reason: str = jfield("reason", "")
    startedAt: Optional[str] = jfield("startedAt", None)
    finishedAt: Optional[str] = jfield("finishedAt", None)


@dataclass(eq=False)
class ContainerStatus(Model):
    name: str = jfield("name", "", omitempty=False)
    restartCount: int = jfield("restartCount", 0, omitempty=False)
    pid: int = jfield("pid", 0)
    ready: bool = jfield("ready", False, omitempty=False)
    lastTerminated: Optional[ContainerStateTerminated] = jfield("lastTerminationState", None)
    terminated: Optional[ContainerStateTerminated] = jfield("terminated", None)


@dataclass(eq=False)
class PodStatus(Model):
    phase: str = jfield("phase", "")
    reason: str = jfield("reason", "")
    message: str = jfield("message", "")
    hostIP: str = jfield("hostIP", "")
    podIP: str = jfield("podIP", "")
    startTime: Optional[str] = jfield("startTime", None)
    containerStatuses: List[ContainerStatus] = jfield("containerStatuses", factory=list)
    # MI355X extension: GPUs bound to this replica by the supervisor.
    gpus: List[int] = jfield("gpus", factory=list)


@dataclass(eq=False)
class Pod(Model):
    apiVersion: str = jfield("apiVersion", "v1")
    kind: str = jfield("kind", "Pod")
    metadata: ObjectMeta = jfield("metadata", factory=ObjectMeta)
    spec: PodSpec = jfield("spec", factory=PodSpec)
    status: PodStatus = jfield("status", factory=PodStatus)


@dataclass(eq=False)
class ServicePort(Model):
    name: str = jfield("name", "")
    port: int = jfield("port", 0, omitempty=False)
    targetPort: int = jfield("targetPort", 0)
    nodePort: int = jfield("nodePort", 0)
    protocol: str = jfield("protocol", "")


@dataclass(eq=False)
class ServiceSpec(Model):
    selector: Dict[str, str] = jfield("selector", factory=dict)
    ports: List[ServicePort] = jfield("ports", factory=list)
    clusterIP: str = jfield("clusterIP", "")


@dataclass(eq=False)
class Service(Model):
    apiVersion: str = jfield("apiVersion", "v1")
    kind: str = jfield("kind", "Service")
    metadata: ObjectMeta = jfield("metadata", factory=ObjectMeta)
    spec: ServiceSpec = jfield("spec", factory=ServiceSpec)


@dataclass(eq=False)
class LabelSelector(Model):
    matchLabels: Dict[str, str] = jfield("matchLabels", factory=dict)


@dataclass(eq=False)
class ReplicaSetSpec(Model):
    replicas: Optional[int] = jfield("replicas", None, ptr=True)
    selector: LabelSelector = jfield("selector", factory=LabelSelector)
    template: PodTemplateSpec = jfield("template", factory=PodTemplateSpec)


@dataclass(eq=False)
class ReplicaSetStatus(Model):
    replicas: int = jfield("replicas", 0, omitempty=False)
    readyReplicas: int = jfield("readyReplicas", 0)


@dataclass(eq=False)
class ReplicaSet(Model):
    """``extensions/v1beta1`` ReplicaSet — only for the (unused) ReplicaSet control
    the reference ships (``pkg/controller/control/replicaset.go``)."""
    apiVersion: str = jfield("apiVersion", "extensions/v1beta1")
    kind: str = jfield("kind", "ReplicaSet")
    metadata: ObjectMeta = jfield("metadata", factory=ObjectMeta)
    spec: ReplicaSetSpec = jfield("spec", factory=ReplicaSetSpec)
    status: ReplicaSetStatus = jfield("status", factory=ReplicaSetStatus)


@dataclass(eq=False)
class ObjectReference(Model):
    kind: str = jfield("kind", "")
    namespace: str = jfield("namespace", "")
    name: str = jfield("name", "")
    uid: str = jfield("uid", "")
    apiVersion: str = jfield("apiVersion", "")
    resourceVersion: str = jfield("resourceVersion", "")


@dataclass(eq=False)
class EventSource(Model):
    component: str = jfield("component", "")
    host: str = jfield("host", "")


@dataclass(eq=False)
class Event(Model):
    """``v1.Event`` as written by the event recorder (``VCG/tools/record/event.go``)."""
    apiVersion: str = jfield("apiVersion", "v1")
    kind: str = jfield("kind", "Event")
    metadata: ObjectMeta = jfield("metadata", factory=ObjectMeta)
    involvedObject: ObjectReference = jfield("involvedObject", factory=ObjectReference)
    reason: str = jfield("reason", "")
    message: str = jfield("message", "")
    source: EventSource = jfield("source", factory=EventSource)
    firstTimestamp: Optional[str] = jfield("firstTimestamp", None)
    lastTimestamp: Optional[str] = jfield("lastTimestamp", None)
    count: int = jfield("count", 0)
    type: str = jfield("type", "")


def pod_is_active(pod: Pod) -> bool:
    """``controller.FilterActivePods`` predicate (``VKC/controller_utils.go:817-835``)."""
    return (pod.status.phase not in (POD_SUCCEEDED, POD_FAILED)
            and pod.metadata.deletionTimestamp is None)


def filter_active_pods(pods):
    return [p for p in pods if pod_is_active(p)]


def gpu_request(container: Container) -> int:
    if container.resources is None:
        return 0
    v = container.resources.limits.get(GPU_RESOURCE) or container.resources.requests.get(GPU_RESOURCE)
    try:
        return int(v) if v is not None else 0
    except ValueError:
        return 0
