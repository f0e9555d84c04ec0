"""Helper: create children with a controller ref and claim existing ones.

Reference ``pkg/controller/helper.go:42-179``.  The claim selector is the 4
labels WITHOUT ``index`` (``helper.go:112-119``); before adopting orphans a
fresh (uncached) GET of the TFJob must still show the same uid and no
deletionTimestamp (``RecheckDeletionTimestamp``).
"""
from __future__ import annotations

from typing import List

from ..api import v1alpha1
from ..api.core import Pod, PodTemplateSpec, Service
from ..api.labels import Selector
from .ref import PodControllerRefManager, ServiceControllerRefManager, recheck_deletion_timestamp
from .util import new_controller_ref


def claim_selector(tfjob: v1alpha1.TFJob, typ: str) -> Selector:
    return Selector.from_match_labels({
        "kubeflow.caicloud.io": "true",
        "job_type": typ,
        "runtime_id": tfjob.spec.runtimeID,
        "tf_job_name": tfjob.metadata.name,
    })


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
        cm = PodControllerRefManager(self.pod_control, tfjob, claim_selector(tfjob, typ), v1alpha1.TFJOB_KIND,
                                     v1alpha1.API_VERSION, self._can_adopt(tfjob))
        return cm.claim_pods(pods)

    def get_services_for_tfjob(self, tfjob: v1alpha1.TFJob, typ: str) -> List[Service]:
        svcs = self.service_lister.list(tfjob.metadata.namespace)
        cm = ServiceControllerRefManager(self.service_control, tfjob, claim_selector(tfjob, typ),
                                         v1alpha1.TFJOB_KIND, v1alpha1.API_VERSION, self._can_adopt(tfjob))
        return cm.claim_services(svcs)
