"""TFJob ``kubeflow.caicloud.io/v1alpha1`` — the API contract, keys unchanged.

Field-for-field the same wire format as the reference's
``VCS/apis/kubeflow/v1alpha1/types.go:30-184`` (note the singular
``tfReplicaSpec`` key holding a list, ``types.go:54``) and the group / version /
kind of ``register.go:25-32``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

from .core import PodTemplateSpec
from .meta import ListMeta, ObjectMeta
from .model import Model, jfield

GROUP_NAME = "kubeflow.caicloud.io"
GROUP_VERSION = "v1alpha1"
API_VERSION = f"{GROUP_NAME}/{GROUP_VERSION}"
TFJOB_KIND = "TFJob"
TFJOB_PLURAL = "tfjobs"
TFJOB_SINGULAR = "tfjob"
CRD_NAME = f"{TFJOB_PLURAL}.{GROUP_NAME}"

# TFReplicaType
PS = "PS"
WORKER = "Worker"
LOCAL = "Local"
REPLICA_TYPES = (PS, WORKER, LOCAL)

# TFJobPhase
PHASE_NONE = ""
PHASE_UNKNOWN = "Unknown"
PHASE_PENDING = "Pending"
PHASE_RUNNING = "Running"
PHASE_SUCCEEDED = "Succeeded"
PHASE_FAILED = "Failed"

# TFJobConditionType
COND_SCHEDULED = "Scheduled"
COND_READY = "Ready"
COND_RECOVERING = "Recovering"
COND_RECYCLING = "Recycling"

# TFReplicaState
STATE_UNKNOWN = "Unknown"
STATE_WAITING = "Waiting"
STATE_RUNNING = "Running"
STATE_SUCCEEDED = "Succeeded"
STATE_FAILED = "Failed"


@dataclass(eq=False)
class ChiefSpec(Model):
    tfReplicaName: str = jfield("tfReplicaName", "", omitempty=False)
    tfReplicaIndex: int = jfield("tfReplicaIndex", 0, omitempty=False)


@dataclass(eq=False)
class TerminationPolicySpec(Model):
    chief: Optional[ChiefSpec] = jfield("chief", None)


@dataclass(eq=False)
class TFReplicaSpec(Model):
    replicas: Optional[int] = jfield("replicas", None, ptr=True)
    tfReplicaType: Optional[str] = jfield("tfReplicaType", None, ptr=True)
    template: Optional[PodTemplateSpec] = jfield("template", None)
    terminationPolicy: Optional[TerminationPolicySpec] = jfield("terminationPolicy", None)


@dataclass(eq=False)
class TFJobSpec(Model):
    runtimeID: str = jfield("runtimeID", "", omitempty=False)
    dataDir: str = jfield("dataDir", "")
    modelDir: str = jfield("modelDir", "")
    logDir: str = jfield("logDir", "")
    exportDir: str = jfield("exportDir", "")
    specs: List[TFReplicaSpec] = jfield("tfReplicaSpec", factory=list, omitempty=False)


@dataclass(eq=False)
class TFJobCondition(Model):
    type: str = jfield("type", "", omitempty=False)
    status: str = jfield("status", "", omitempty=False)
    reason: str = jfield("reason", "", omitempty=False)
    lastTransitionTime: Optional[str] = jfield("lastTransitionTime", None)


@dataclass(eq=False)
class TFReplicaStatus(Model):
    type: Optional[str] = jfield("type", None, omitempty=False)
    state: str = jfield("state", "", omitempty=False)
    tfReplicasStates: Dict[str, int] = jfield("tfReplicasStates", factory=dict)


@dataclass(eq=False)
class TFJobStatus(Model):
    phase: str = jfield("phase", "", omitempty=False)
    reason: str = jfield("reason", "", omitempty=False)
    conditions: Optional[List[TFJobCondition]] = jfield("conditions", None, omitempty=False)
    tfReplicaStatuses: Optional[List[TFReplicaStatus]] = jfield("tfReplicaStatuses", None, omitempty=False)


@dataclass(eq=False)
class TFJob(Model):
    apiVersion: str = jfield("apiVersion", API_VERSION)
    kind: str = jfield("kind", TFJOB_KIND)
    metadata: ObjectMeta = jfield("metadata", factory=ObjectMeta)
    spec: TFJobSpec = jfield("spec", factory=TFJobSpec, omitempty=False)
    status: TFJobStatus = jfield("status", factory=TFJobStatus, omitempty=False)

    # Convenience accessors mirroring the Go field names.
    @property
    def name(self) -> str:
        return self.metadata.name

    @property
    def namespace(self) -> str:
        return self.metadata.namespace

    @property
    def uid(self) -> str:
        return self.metadata.uid


@dataclass(eq=False)
class TFJobList(Model):
    apiVersion: str = jfield("apiVersion", API_VERSION)
    kind: str = jfield("kind", "TFJobList")
    metadata: ListMeta = jfield("metadata", factory=ListMeta)
    items: List[TFJob] = jfield("items", factory=list, omitempty=False)


def crd_manifest() -> Dict:
    """The CustomResourceDefinition of ``examples/crd/crd.yml:1-12``."""
    return {
        "apiVersion": "apiextensions.k8s.io/v1beta1",
        "kind": "CustomResourceDefinition",
        "metadata": {"name": CRD_NAME},
        "spec": {
            "group": GROUP_NAME,
            "version": GROUP_VERSION,
            "names": {"kind": TFJOB_KIND, "singular": TFJOB_SINGULAR, "plural": TFJOB_PLURAL},
            "scope": "Namespaced",
        },
    }
