"""Controller utilities (reference ``pkg/controller/util.go:22-55``)."""
from __future__ import annotations

from typing import List, Tuple

from ..api import v1alpha1
from ..api.core import POD_FAILED, POD_SUCCEEDED, Pod
from ..api.meta import OwnerReference

INDEX_LABEL_NAME = "worker_index"  # declared, unused (as in the reference)


def filter_pods(pods: List[Pod], phase: str) -> int:
    return sum(1 for p in pods if p.status.phase == phase)


def get_status(pods: List[Pod]) -> Tuple[int, int]:
    """(succeeded, failed) counts."""
    return filter_pods(pods, POD_SUCCEEDED), filter_pods(pods, POD_FAILED)


def new_controller_ref(tfjob: v1alpha1.TFJob) -> OwnerReference:
    return OwnerReference(apiVersion=v1alpha1.API_VERSION, kind=v1alpha1.TFJOB_KIND, name=tfjob.metadata.name,
                          uid=tfjob.metadata.uid, blockOwnerDeletion=True, controller=True)


def succeeded_indices(pods: List[Pod]) -> List[int]:
    out = []
    for p in pods:
        if p.status.phase == POD_SUCCEEDED:
            try:
                out.append(int(p.metadata.labels.get("index", "")))
            except ValueError:
                pass
    return out
