"""Local (single-replica) job planner (reference ``pkg/tensorflow/local.go``).

A local job has exactly one replica (``ExpectedLocalWorkerNumber = 1``,
``local.go:22-24``).  If a replica already succeeded nothing happens; if none
is active, ``compose()`` stamps the runtime ID and the 4 claim labels on
``Specs[0].template`` and the planner asks for one worker.

Fix vs the reference: the runtime ID is minted only when the job has none, so
a restarted replica keeps matching the job's selector.
"""
from __future__ import annotations

import logging
from typing import Dict, List

from ..api import v1alpha1
from ..api.core import Pod
from .types import Action, Event
from .util import generate_runtime_id, with_job_dirs

EXPECTED_LOCAL_WORKER_NUMBER = 1
log = logging.getLogger("kfa.planner")


def job_labels(tfjob: v1alpha1.TFJob, typ: str) -> Dict[str, str]:
    """The 4 child labels (``local.go:83-90``, ``distributed.go:221-228``)."""
    return {
        "kubeflow.caicloud.io": "true",
        "job_type": typ,
        "runtime_id": tfjob.spec.runtimeID,
        "tf_job_name": tfjob.metadata.name,
    }


class LocalJob:
    def __init__(self, tfjob: v1alpha1.TFJob, active_pods: List[Pod], succeeded: int):
        self.tfjob = tfjob
        self.pod = None
        if len(active_pods) == 1:
            self.pod = active_pods[0]
        elif len(active_pods) > 1:
            log.info("Local job %s has more than one active replica", tfjob.metadata.name)
            self.pod = active_pods[0]
        self.succeeded = succeeded

    def action(self) -> Event:
        if self.succeeded > 0:
            return Event(Action.Nothing)
        active = 1 if self.pod is not None else 0
        if active < EXPECTED_LOCAL_WORKER_NUMBER:
            self.compose()
            return Event(Action.ShouldAddWorker, EXPECTED_LOCAL_WORKER_NUMBER - active)
        return Event(Action.Nothing)

    def compose(self) -> None:
        if not self.tfjob.spec.runtimeID:
            self.tfjob.spec.runtimeID = generate_runtime_id(self.tfjob.metadata.uid)
        self.tfjob.spec.specs[0].template.metadata.labels = self.labels()

    def labels(self) -> Dict[str, str]:
        return job_labels(self.tfjob, self.tfjob.spec.specs[0].tfReplicaType)

    def get_template(self):
        return with_job_dirs(self.tfjob.spec.specs[0].template, self.tfjob)
