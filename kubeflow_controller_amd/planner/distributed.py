"""Distributed (Worker + PS) job planner and cluster-spec generator.

Reference: ``pkg/tensorflow/distributed.go``.  Same action
sequence, names, labels and argument strings:

* services first (worker, then PS), then worker replicas, then PS replicas;
* service name ``<job>-<worker|ps>-<i>-<5 random>``, port 2222 named
  ``kubeflow-port``, selector = the 4 labels + ``index``;
* replica args REPLACE ``containers[0].args`` with
  ``--worker_hosts=<svc>:2222,...  --ps_hosts=...  --job_name=<worker|ps>  --task_index=<i>``.

MI355X-side additions: ``TF_CONFIG`` is exported on the replica's first
container (``{"cluster": {"worker": [...], "ps": [...]}, "task": {...}}``,
SURVEY §5.6), and a Worker-only job (no PS spec — the "8-worker all-reduce"
config) is accepted.

Fixes of the reference quirks, keeping the strings:

1. service names come from the services that exist (``index`` label) plus the
   ones generated in this sync, so re-created replicas never get ``:2222``
   host lists;
2. ``runtime_id`` is minted once (surviving replicas are not orphaned);
3. only MISSING replica indices / services are created (not ``0..n-1`` again);
4. Worker/PS specs are looked up by type (any order), not only at [0]/[1].
"""
from __future__ import annotations

import json
import logging
from typing import Dict, List, Optional

from ..api import v1alpha1
from ..api.core import EnvVar, Pod, PodTemplateSpec, Service, ServicePort, ServiceSpec
from ..api.meta import ObjectMeta
from ..api.model import deep_copy
from .local import job_labels
from .types import Action, Event
from .util import generate_name, generate_runtime_id, with_job_dirs

PORT_NAME = "kubeflow-port"
WORKER_PORT = 2222
TF_CONFIG_ENV = "TF_CONFIG"

log = logging.getLogger("kfa.planner")


def _index_of(obj) -> Optional[int]:
    try:
        return int(obj.metadata.labels.get("index", ""))
    except ValueError:
        return None


class DistributedJob:
    def __init__(self, tfjob: v1alpha1.TFJob, active_worker_pods: List[Pod], active_ps_pods: List[Pod],
                 worker_services: List[Service], ps_services: List[Service], succeeded_worker_pods: int,
                 succeeded_worker_indices: Optional[List[int]] = None,
                 succeeded_ps_indices: Optional[List[int]] = None):
        self.tfjob = tfjob
        self.active_worker_pods = active_worker_pods
        self.active_ps_pods = active_ps_pods
        self.worker_services = worker_services
        self.ps_services = ps_services
        self.succeeded_worker_pods = succeeded_worker_pods
        self.succeeded_worker_indices = set(succeeded_worker_indices or [])
        self.succeeded_ps_indices = set(succeeded_ps_indices or [])
        # logical service name (<job>-<type>-<i>) -> generated object name
        self.service_names: Dict[str, str] = {}
        for typ, svcs in ((v1alpha1.WORKER, worker_services), (v1alpha1.PS, ps_services)):
            for s in svcs:
                i = _index_of(s)
                if i is not None:
                    self.service_names[self.get_service_name(typ, i)] = s.metadata.name

    # ------------------------------------------------------------------ spec lookup
    def _spec(self, typ: str) -> Optional[v1alpha1.TFReplicaSpec]:
        for s in self.tfjob.spec.specs:
            if s.tfReplicaType == typ:
                return s
        return None

    def get_worker_spec(self) -> v1alpha1.TFReplicaSpec:
        s = self._spec(v1alpha1.WORKER)
        if s is None:
            raise ValueError(f"TFJob {self.tfjob.metadata.name}: no Worker spec")
        return s

    def get_ps_spec(self) -> Optional[v1alpha1.TFReplicaSpec]:
        return self._spec(v1alpha1.PS)

    def replicas(self, typ: str) -> int:
        s = self._spec(typ)
        return 0 if s is None else (1 if s.replicas is None else int(s.replicas))

    # ------------------------------------------------------------------ planning
    def action(self) -> List[Event]:
        events: List[Event] = []
        n_worker = self.replicas(v1alpha1.WORKER)
        n_ps = self.replicas(v1alpha1.PS)
        expected_worker = n_worker - self.succeeded_worker_pods
        if n_worker and expected_worker <= 0:
            # every worker succeeded: the job is complete, PS replicas are being
            # recycled (TFJobRecycling) — never re-create anything for it
            return [Event(Action.Nothing)]
        expected_ps = n_ps - len(self.succeeded_ps_indices)

        have_wsvc = {_index_of(s) for s in self.worker_services}
        miss_wsvc = [i for i in range(n_worker) if i not in have_wsvc]
        if miss_wsvc and n_worker:
            log.debug("Expected worker services to be %d but got %d, create %d", n_worker, len(have_wsvc),
                      len(miss_wsvc))
            events.append(Event(Action.ShouldAddWorkerService, len(miss_wsvc), miss_wsvc))

        have_psvc = {_index_of(s) for s in self.ps_services}
        miss_psvc = [i for i in range(n_ps) if i not in have_psvc]
        if miss_psvc:
            log.debug("Expected ps services to be %d but got %d, create %d", n_ps, len(have_psvc), len(miss_psvc))
            events.append(Event(Action.ShouldAddPSService, len(miss_psvc), miss_psvc))

        active_w = {_index_of(p) for p in self.active_worker_pods}
        if len(self.active_worker_pods) < expected_worker:
            self.compose()
            missing = [i for i in range(n_worker) if i not in active_w and i not in self.succeeded_worker_indices]
            missing = missing[:expected_worker - len(self.active_worker_pods)]
            events.append(Event(Action.ShouldAddWorker, len(missing), missing))
        elif len(self.active_worker_pods) == expected_worker:
            events.append(Event(Action.Nothing))

        active_p = {_index_of(p) for p in self.active_ps_pods}
        if len(self.active_ps_pods) < expected_ps:
            self.compose()
            missing = [i for i in range(n_ps) if i not in active_p and i not in self.succeeded_ps_indices]
            missing = missing[:expected_ps - len(self.active_ps_pods)]
            events.append(Event(Action.ShouldAddPS, len(missing), missing))
        return events

    def compose(self) -> None:
        """Stamp runtime ID (once) + labels on the Worker/PS templates (``distributed.go:210-219``)."""
        if not self.tfjob.spec.runtimeID:
            self.tfjob.spec.runtimeID = generate_runtime_id(self.tfjob.metadata.uid)
        self.get_worker_spec().template.metadata.labels = self.get_labels(v1alpha1.WORKER)
        ps = self.get_ps_spec()
        if ps is not None:
            ps.template.metadata.labels = self.get_labels(v1alpha1.PS)

    def get_labels(self, typ: str) -> Dict[str, str]:
        return job_labels(self.tfjob, typ)

    # ------------------------------------------------------------------ replicas
    def get_spec(self, typ: str, index: int) -> PodTemplateSpec:
        """Per-index pod template: label ``index=i``, args = cluster spec, env TF_CONFIG."""
        spec = self._spec(typ)
        tmpl = deep_copy(spec.template)
        tmpl.metadata.labels = dict(self.get_labels(typ), index=str(index))
        c0 = tmpl.spec.containers[0]
        c0.args = self.generate_tf_cluster_spec(typ, index)
        c0.env = [e for e in c0.env if e.name != TF_CONFIG_ENV] + [
            EnvVar(name=TF_CONFIG_ENV, value=json.dumps(self.tf_config(typ, index)))]
        return with_job_dirs(tmpl, self.tfjob)

    def _hosts(self, typ: str) -> List[str]:
        return [f"{self.service_names.get(self.get_service_name(typ, i), '')}:{WORKER_PORT}"
                for i in range(self.replicas(typ))]

    def generate_tf_cluster_spec(self, typ: str, index: int) -> List[str]:
        return [
            "--worker_hosts=" + ",".join(self._hosts(v1alpha1.WORKER)),
            "--ps_hosts=" + ",".join(self._hosts(v1alpha1.PS)),
            f"--job_name={typ.lower()}",
            f"--task_index={index}",
        ]

    def tf_config(self, typ: str, index: int) -> Dict:
        cluster = {"worker": self._hosts(v1alpha1.WORKER)}
        if self.replicas(v1alpha1.PS):
            cluster["ps"] = self._hosts(v1alpha1.PS)
        return {"cluster": cluster, "task": {"type": typ.lower(), "index": index}, "environment": "cloud"}

    # ------------------------------------------------------------------ services
    def get_service_name(self, typ: str, index: int) -> str:
        return f"{self.tfjob.metadata.name}-{typ.lower()}-{index}"

    def get_service(self, typ: str, index: int) -> Service:
        labels = dict(self.get_labels(typ), index=str(index))
        name = self.get_service_name(typ, index)
        generated = generate_name(f"{name}-")
        self.service_names[name] = generated
        return Service(metadata=ObjectMeta(name=generated, labels=dict(labels)),
                       spec=ServiceSpec(selector=dict(labels), ports=[ServicePort(name=PORT_NAME, port=WORKER_PORT)]))
