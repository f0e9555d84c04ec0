"""Status updaters (reference ``pkg/controller/updater/``).

``should_update()`` mutates ``tfjob.status`` and reports whether a write is
needed — same phase rules and replica-state histogram as the reference:

* Local (``updater/local.go:50-78``): ``Succeeded`` iff the succeeded count is
  1, else ``Running``; ``tfReplicaStatuses = [{type: Local,
  tfReplicasStates: {<podPhase>: 1}}]`` whenever a replica exists.
* Distributed (``updater/distributed.go:41-66``, ``updater/util.go:25-86``):
  ``Succeeded`` iff succeeded workers == worker replicas, else ``Running``;
  a per-type histogram of replica phases is upserted (<= 2 entries, one per
  type).

Differences (SURVEY §7.4 "fix the mechanism, keep the API"):
* ``should_update`` returns True only when the status actually CHANGED (the
  reference returns True on every sync with pods and relies on the apiserver
  no-op'ing identical writes; our store also no-ops, this just avoids the PUT);
* ``Failed`` phase: set when a worker replica failed and its restartPolicy
  will not restart it (``Never``), or a failed Local replica with ``Never``.
  The reference never sets ``Failed`` (``types.go:145``); with the samples'
  ``OnFailure`` policy the behaviour is identical.
"""
from __future__ import annotations

from typing import Dict, List, Optional

from ..api import v1alpha1
from ..api.core import POD_FAILED, POD_SUCCEEDED, RESTART_NEVER, Pod
from ..api.meta import now_rfc3339
from ..api.model import to_json
from ..planner.local import EXPECTED_LOCAL_WORKER_NUMBER


def set_condition(st: v1alpha1.TFJobStatus, ctype: str, status: str, reason: str) -> None:
    """Upsert a condition; lastTransitionTime changes only when status flips."""
    conds = st.conditions or []
    for c in conds:
        if c.type == ctype:
            if c.status != status:
                c.status, c.lastTransitionTime = status, now_rfc3339()
            c.reason = reason
            st.conditions = conds
            return
    conds.append(v1alpha1.TFJobCondition(type=ctype, status=status, reason=reason, lastTransitionTime=now_rfc3339()))
    st.conditions = conds


def _histogram(pods: List[Pod]) -> Dict[str, int]:
    h: Dict[str, int] = {}
    for p in pods:
        ph = p.status.phase or "Pending"
        h[ph] = h.get(ph, 0) + 1
    return h


def _restart_policy(tfjob: v1alpha1.TFJob, typ: str) -> str:
    for s in tfjob.spec.specs:
        if s.tfReplicaType == typ and s.template is not None:
            return s.template.spec.restartPolicy or "Always"
    return "Always"


def update_tf_replica_statuses(tfjob: v1alpha1.TFJob, pods: List[Pod], typ: str) -> bool:
    """Upsert the ``typ`` histogram; False when there are no pods or >2 entries."""
    if not pods:
        return False
    statuses = tfjob.status.tfReplicaStatuses or []
    if len(statuses) > 2:
        return False
    entry = v1alpha1.TFReplicaStatus(type=typ, tfReplicasStates=_histogram(pods))
    for i, st in enumerate(statuses):
        if st.type == typ:
            statuses[i] = entry
            break
    else:
        statuses.append(entry)
    tfjob.status.tfReplicaStatuses = statuses
    return True


class LocalUpdater:
    def __init__(self, tfjob: v1alpha1.TFJob, succeeded_worker_pods: int, worker_pods: List[Pod]):
        if len(worker_pods) > 1:
            # the reference errors out here (updater/local.go:41-43); we report the newest replica
            worker_pods = sorted(worker_pods, key=lambda p: p.metadata.creationTimestamp or "")[-1:]
        self.tfjob = tfjob
        self.succeeded = succeeded_worker_pods
        self.pod: Optional[Pod] = worker_pods[0] if worker_pods else None

    def should_update(self) -> bool:
        before = to_json(self.tfjob.status)
        st = self.tfjob.status
        if self.succeeded == EXPECTED_LOCAL_WORKER_NUMBER:
            st.phase = v1alpha1.PHASE_SUCCEEDED
        elif (self.pod is not None and self.pod.status.phase == POD_FAILED
              and _restart_policy(self.tfjob, v1alpha1.LOCAL) == RESTART_NEVER):
            st.phase = v1alpha1.PHASE_FAILED
        elif st.phase != v1alpha1.PHASE_RUNNING:
            st.phase = v1alpha1.PHASE_RUNNING
        if self.pod is not None:
            st.tfReplicaStatuses = [v1alpha1.TFReplicaStatus(
                type=v1alpha1.LOCAL, tfReplicasStates={self.pod.status.phase or "Pending": 1})]
        return to_json(st) != before


class DistributedUpdater:
    def __init__(self, tfjob: v1alpha1.TFJob, succeeded_worker_pods: int, worker_pods: List[Pod],
                 ps_pods: List[Pod]):
        self.tfjob = tfjob
        self.succeeded = succeeded_worker_pods
        self.worker_pods = worker_pods
        self.ps_pods = ps_pods

    def expected_workers(self) -> int:
        for s in self.tfjob.spec.specs:
            if s.tfReplicaType == v1alpha1.WORKER:
                return 1 if s.replicas is None else int(s.replicas)
        return 0

    def should_update(self) -> bool:
        before = to_json(self.tfjob.status)
        st = self.tfjob.status
        failed_for_good = any(p.status.phase == POD_FAILED for p in self.worker_pods) and \
            _restart_policy(self.tfjob, v1alpha1.WORKER) == RESTART_NEVER
        if self.succeeded == self.expected_workers():
            st.phase = v1alpha1.PHASE_SUCCEEDED
        elif failed_for_good:
            st.phase = v1alpha1.PHASE_FAILED
        elif st.phase != v1alpha1.PHASE_RUNNING:
            st.phase = v1alpha1.PHASE_RUNNING
        update_tf_replica_statuses(self.tfjob, self.worker_pods, v1alpha1.WORKER)
        update_tf_replica_statuses(self.tfjob, self.ps_pods, v1alpha1.PS)
        if st.phase == v1alpha1.PHASE_SUCCEEDED and self.ps_pods:
            # TFJobRecycling (types.go:153-155): workers done, PS replicas being reclaimed
            recycling = any(p.status.phase not in (POD_SUCCEEDED, POD_FAILED) for p in self.ps_pods)
            set_condition(st, v1alpha1.COND_RECYCLING, "True" if recycling else "False",
                          "WorkersSucceeded" if recycling else "PSRecycled")
        return to_json(st) != before


# Go-style aliases
NewLocal = LocalUpdater
NewDistributed = DistributedUpdater
