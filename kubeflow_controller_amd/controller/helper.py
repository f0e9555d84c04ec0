"""Helper: create children with a controller ref and claim existing ones.

Reference ``pkg/controller/helper.go:42-179``.  Before adopting orphans a
fresh (uncached) GET of the TFJob must still show the same uid and no
deletionTimestamp (``RecheckDeletionTimestamp``).

Fix: the reference claims with the 4-label selector INCLUDING ``job_type``
(``helper.go:112-119``), so ``GetPodsForTFJob(job, PS)`` sees the job's own
Worker pods as "owned but not matching" and RELEASES them (orphans that the
next Worker claim re-adopts, and that the owner's cascade delete misses).
Here the claim uses the job-level labels (``kubeflow.caicloud.io``,
``runtime_id``, ``tf_job_name``) and the replica type is a filter applied to
the claimed set.
"""
from __future__ import annotations

from typing import List, Optional

from ..api import v1alpha1
from ..api.core import Pod, PodTemplateSpec, Service
from ..api.labels import Selector
from .ref import PodControllerRefManager, ServiceControllerRefManager, recheck_deletion_timestamp
from .util import new_controller_ref


def claim_selector(tfjob: v1alpha1.TFJob, typ: Optional[str] = None) -> Selector:
    labels = {"kubeflow.caicloud.io": "true", "runtime_id": tfjob.spec.runtimeID,
              "tf_job_name": tfjob.metadata.name}
    if typ is not None:
        labels["job_type"] = typ
    return Selector.from_match_labels(labels)


def _of_type(typ: str):
    return lambda o: o.metadata.labels.get("job_type") == typ


class Helper:
    def __init__(self, tfjob_client, pod_lister, pod_control, service_lister, service_control):
        self.tfjob_client = tfjob_client
        self.pod_lister = pod_lister
        self.pod_control = pod_control
        self.service_lister = service_lister
        self.service_control = service_control

    def create_service(self, tfjob: v1alpha1.TFJob, service: Service):
        return self.service_control.create_services_with_controller_ref(
            tfjob.metadata.namespace, service, tfjob, new_controller_ref(tfjob))

    def create_pod(self, tfjob: v1alpha1.TFJob, template: PodTemplateSpec):
        return self.pod_control.create_pods_with_controller_ref(
            tfjob.metadata.namespace, template, tfjob, new_controller_ref(tfjob))

    def _can_adopt(self, tfjob: v1alpha1.TFJob):
        def fresh():
            f = self.tfjob_client.kubeflow_v1alpha1().tfjobs(tfjob.metadata.namespace).get(tfjob.metadata.name)
            if f.metadata.uid != tfjob.metadata.uid:
                raise RuntimeError(f"original Job {tfjob.metadata.namespace}/{tfjob.metadata.name} is gone: "
                                   f"got uid {f.metadata.uid}, wanted {tfjob.metadata.uid}")
            return f
        return recheck_deletion_timestamp(fresh)

    def get_pods_for_tfjob(self, tfjob: v1alpha1.TFJob, typ: str) -> List[Pod]:
        pods = self.pod_lister.list(tfjob.metadata.namespace)
        cm = PodControllerRefManager(self.pod_control, tfjob, claim_selector(tfjob), v1alpha1.TFJOB_KIND,
                                     v1alpha1.API_VERSION, self._can_adopt(tfjob))
        return [p for p in cm.claim_pods(pods) if _of_type(typ)(p)]

    def get_services_for_tfjob(self, tfjob: v1alpha1.TFJob, typ: str) -> List[Service]:
        svcs = self.service_lister.list(tfjob.metadata.namespace)
        cm = ServiceControllerRefManager(self.service_control, tfjob, claim_selector(tfjob),
                                         v1alpha1.TFJOB_KIND, v1alpha1.API_VERSION, self._can_adopt(tfjob))
        return [s for s in cm.claim_services(svcs) if _of_type(typ)(s)]
