"""The TFJob reconcile loop (reference ``pkg/controller/controller.go``).

Structure kept from the reference: informers for TFJobs,
Pods and Services feed a rate-limited, de-duplicating work queue keyed
``ns/name``; N worker threads run ``sync_handler(key)``, which claims the
job's children, plans (``planner``), creates what is missing under
expectations, runs the status updater and writes the TFJob back.

Behavioural fixes, API strings unchanged:
* objects from listers are deep copies — the shared cache is never mutated;
* a failing sync is re-queued with ``add_rate_limited`` (the reference only
  logs, ``controller.go:227-229``);
* Pod/Service DELETE events enqueue the owner (reference: "To Be Implemented",
  ``:505-508, 587-590``), so a killed replica is recreated immediately;
* expectations accumulate across the events of one sync (``raise``), instead
  of being overwritten per event;
* the spec (runtimeID / template labels) and the status are written only when
  they changed.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import List, Optional

from ..utils import metrics
from ..api import v1alpha1
from ..api.core import filter_active_pods
from ..api.meta import get_controller_of, key_of, split_key
from ..api.model import deep_copy, to_json
from ..checker import is_local_job
from ..client.clientset import Clientset
from ..client.events import EventBroadcaster
from ..client.informer import SharedInformerFactory
from ..client.workqueue import EXPECTATIONS_TIMEOUT, ControllerExpectations, RateLimitingQueue
from ..planner import Action, DistributedJob, LocalJob
from ..store import errors
from .control import RealPodControl, RealServiceControl
from .helper import Helper
from .updater import DistributedUpdater, LocalUpdater
from .util import get_status, succeeded_indices

CONTROLLER_NAME = "kubeflow-controller"
SUCCESS_SYNCED = "Synced"                              # declared, never emitted (as in the reference)
MESSAGE_RESOURCE_SYNCED = "TFJob synced successfully"  # declared, never emitted

log = logging.getLogger("kfa.controller")


class Controller:
    def __init__(self, kube_client: Clientset, tfjob_client: Clientset, kube_informers: SharedInformerFactory,
                 tfjob_informers: SharedInformerFactory, *, recorder=None, pod_control=None, service_control=None,
                 broadcaster: Optional[EventBroadcaster] = None):
        self.kube_client = kube_client
        self.tfjob_client = tfjob_client
        tfjob_inf = tfjob_informers.tfjobs()
        pod_inf = kube_informers.pods()
        svc_inf = kube_informers.services()
        self.broadcaster = broadcaster
        if recorder is None:
            self.broadcaster = broadcaster or EventBroadcaster()
            self.broadcaster.start_logging(log.info)
            self.broadcaster.start_recording_to_sink(kube_client)
            recorder = self.broadcaster.new_recorder(CONTROLLER_NAME)
        self.recorder = recorder
        pod_control = pod_control or RealPodControl(kube_client, recorder)
        service_control = service_control or RealServiceControl(kube_client, recorder)
        self.helper = Helper(tfjob_client, pod_inf.lister(), pod_control, svc_inf.lister(), service_control)
        self.tfjob_lister = tfjob_inf.lister()
        self.tfjob_synced = tfjob_inf.has_synced
        self.informers = (tfjob_informers, kube_informers)
        self.workqueue = RateLimitingQueue(None, "tfJobs")
        self.expectations = ControllerExpectations(EXPECTATIONS_TIMEOUT)
        self.sync_count = 0
        self.last_sync_seconds = 0.0

        tfjob_inf.add_event_handler(on_add=self.enqueue_tfjob, on_update=self._update_tfjob_event,
                                    on_delete=self.enqueue_tfjob)
        pod_inf.add_event_handler(on_add=self.add_pod, on_update=self.update_pod, on_delete=self.delete_pod)
        svc_inf.add_event_handler(on_add=self.add_service, on_update=self.update_service,
                                  on_delete=self.delete_service)

    # ------------------------------------------------------------------ run
    def run(self, threadiness: int, stop: threading.Event, cache_sync_timeout: Optional[float] = None) -> None:
        """Start ``threadiness`` workers and block until ``stop`` (``controller.go:158-182``)."""
        log.info("Starting TFJob controller")
        log.info("Waiting for informer caches to sync")
        deadline = None if cache_sync_timeout is None else time.monotonic() + cache_sync_timeout
        while not self.tfjob_synced():
            if stop.is_set() or (deadline is not None and time.monotonic() > deadline):
                raise RuntimeError("failed to wait for caches to sync")
            time.sleep(0.01)
        log.info("Starting workers")
        threads = [threading.Thread(target=self._run_worker, args=(stop,), name=f"tfjob-worker-{i}", daemon=True)
                   for i in range(threadiness)]
        for t in threads:
            t.start()
        log.info("Started workers")
        stop.wait()
        log.info("Shutting down workers")
        self.workqueue.shut_down()
        for t in threads:
            t.join(timeout=5)

    def _run_worker(self, stop: threading.Event) -> None:
        # wait.Until(c.runWorker, time.Second, stopCh)
        while not stop.is_set():
            while self.process_next_work_item():
                pass
            if self.workqueue.shutting_down():
                return
            stop.wait(1.0)

    def process_next_work_item(self, timeout: float = -1.0) -> bool:
        key, shutdown = self.workqueue.get(timeout)
        if shutdown:
            return False
        if key is None:  # timeout
            return True
        t0 = time.perf_counter()
        try:
            self.sync_handler(key)
            self.last_sync_seconds = time.perf_counter() - t0
            self.sync_count += 1
            self.workqueue.forget(key)
            log.debug("Finished syncing %r (%.3f ms)", key, self.last_sync_seconds * 1e3)
        except Exception as e:  # noqa: BLE001 — runtime.HandleError + requeue
            log.warning("error syncing %r: %s", key, e)
            metrics.SYNC_ERRORS.inc()
            metrics.WORKQUEUE_RETRIES.inc()
            self.workqueue.add_rate_limited(key)
        finally:
            metrics.SYNC_DURATION.observe(time.perf_counter() - t0)
            self.workqueue.done(key)
            metrics.WORKQUEUE_DEPTH.set(len(self.workqueue))
        return True

    # ------------------------------------------------------------------ sync
    def sync_handler(self, key: str) -> None:
        namespace, name = split_key(key)
        if not namespace or not name:
            raise ValueError(f"invalid job key {key!r}: either namespace or name is missing")
        job_needs_sync = self.expectations.satisfied_expectations(key)
        try:
            tfjob = self.tfjob_lister.get(namespace, name)
        except errors.NotFound:
            log.debug("Job has been deleted: %s", key)
            self.expectations.delete_expectations(key)
            return
        original = deep_copy(tfjob)
        if not tfjob.spec.runtimeID:
            # Mint the (UID-derived) runtime ID BEFORE claiming children: a retried
            # sync whose spec write was lost must select the replicas it created.
            from ..planner.util import generate_runtime_id
            tfjob.spec.runtimeID = generate_runtime_id(tfjob.metadata.uid)

        worker_pods: List = []
        ps_pods: List = []
        worker_svcs: List = []
        ps_svcs: List = []
        local = is_local_job(tfjob)
        if local:
            worker_pods = self.helper.get_pods_for_tfjob(tfjob, v1alpha1.LOCAL)
        else:
            worker_pods = self.helper.get_pods_for_tfjob(tfjob, v1alpha1.WORKER)
            ps_pods = self.helper.get_pods_for_tfjob(tfjob, v1alpha1.PS)
            worker_svcs = self.helper.get_services_for_tfjob(tfjob, v1alpha1.WORKER)
            ps_svcs = self.helper.get_services_for_tfjob(tfjob, v1alpha1.PS)

        active_worker = filter_active_pods(worker_pods)
        succeeded, _failed = get_status(worker_pods)
        active_ps = filter_active_pods(ps_pods)

        # Status first (reference order: controller.go:319-335 runs it after the
        # planner): a job that just reached Succeeded/Failed — e.g. a worker failed
        # under restartPolicy Never — must not get replacement replicas.
        if local:
            updater = LocalUpdater(tfjob, succeeded, worker_pods)
        else:
            updater = DistributedUpdater(tfjob, succeeded, worker_pods, ps_pods)
        status_changed = updater.should_update()
        terminal = tfjob.status.phase in (v1alpha1.PHASE_SUCCEEDED, v1alpha1.PHASE_FAILED)

        if job_needs_sync and tfjob.metadata.deletionTimestamp is None and not terminal:
            self.manage_tfjob(active_worker, active_ps, worker_svcs, ps_svcs, succeeded, tfjob,
                              succeeded_indices(worker_pods), succeeded_indices(ps_pods))

        spec_changed = to_json(tfjob.spec) != to_json(original.spec) or \
            to_json(tfjob.metadata) != to_json(original.metadata)
        if status_changed or spec_changed:
            self.update_tfjob(tfjob)
            if tfjob.status.phase != original.status.phase:
                metrics.PHASE_TRANSITIONS.labels(tfjob.status.phase or "").inc()
        log.debug("Sync TFJob: %s", key)

    def manage_tfjob(self, active_worker, active_ps, worker_svcs, ps_svcs, succeeded: int,
                     tfjob: v1alpha1.TFJob, succeeded_idx=None, succeeded_ps_idx=None):
        key = key_of(tfjob)
        log.debug("Manage the TFJob %s, active workers: %d, active parameter servers: %d",
                  tfjob.metadata.name, len(active_worker), len(active_ps))
        if is_local_job(tfjob):
            lj = LocalJob(tfjob, active_worker, succeeded)
            ev = lj.action()
            if ev.action == Action.ShouldAddWorker:
                self.expectations.raise_expectations(key, ev.number, 0)
                try:
                    self.helper.create_pod(tfjob, lj.get_template())
                except Exception:
                    self.expectations.creation_observed(key)
                    raise
            return 1, 0
        dj = DistributedJob(tfjob, active_worker, active_ps, worker_svcs, ps_svcs, succeeded, succeeded_idx,
                            succeeded_ps_idx)
        events = dj.action()
        n_w = n_p = 0
        first_err: Optional[Exception] = None
        for ev in events:
            if ev.action in (Action.ShouldAddWorkerService, Action.ShouldAddPSService):
                typ = v1alpha1.WORKER if ev.action == Action.ShouldAddWorkerService else v1alpha1.PS
                self.expectations.raise_expectations(key, ev.number, 0)
                for i in ev.indices:
                    try:
                        self.helper.create_service(tfjob, dj.get_service(typ, i))
                    except Exception as e:  # reference: log and continue
                        self.expectations.creation_observed(key)
                        first_err = first_err or e
            elif ev.action in (Action.ShouldAddWorker, Action.ShouldAddPS):
                typ = v1alpha1.WORKER if ev.action == Action.ShouldAddWorker else v1alpha1.PS
                self.expectations.raise_expectations(key, ev.number, 0)
                created = 0
                for i in ev.indices:
                    try:
                        self.helper.create_pod(tfjob, dj.get_spec(typ, i))
                        created += 1
                    except Exception:
                        # reference: first pod error aborts the sync; lower the rest
                        for _ in range(len(ev.indices) - created):
                            self.expectations.creation_observed(key)
                        raise
                if typ == v1alpha1.WORKER:
                    n_w = len(active_worker) + ev.number
                else:
                    n_p = len(active_ps) + ev.number
        if first_err is not None:
            raise first_err
        return n_w, n_p

    def update_tfjob(self, tfjob: v1alpha1.TFJob) -> v1alpha1.TFJob:
        """PUT the whole object (spec mutations + status), ``controller.go:630-636``."""
        return self.tfjob_client.kubeflow_v1alpha1().tfjobs(tfjob.metadata.namespace).update(tfjob)

    # ------------------------------------------------------------------ event handlers
    def enqueue_tfjob(self, obj) -> None:
        self.workqueue.add_rate_limited(key_of(obj))
        metrics.WORKQUEUE_ADDS.inc()

    def _update_tfjob_event(self, old, new) -> None:
        if old.metadata.resourceVersion == new.metadata.resourceVersion:
            return  # periodic resync: nothing changed
        self.enqueue_tfjob(new)

    def resolve_controller_ref(self, namespace: str, ref) -> Optional[v1alpha1.TFJob]:
        if ref.kind != v1alpha1.TFJOB_KIND:
            return None
        try:
            job = self.tfjob_lister.get(namespace, ref.name)
        except errors.NotFound:
            return None
        if job.metadata.uid != ref.uid:
            return None
        return job

    def _owner_of(self, obj) -> Optional[v1alpha1.TFJob]:
        ref = get_controller_of(obj)
        if ref is None:
            return None
        return self.resolve_controller_ref(obj.metadata.namespace, ref)

    def add_pod(self, pod) -> None:
        job = self._owner_of(pod)
        if job is None:
            return
        self.expectations.creation_observed(key_of(job))
        self.enqueue_tfjob(job)

    def update_pod(self, old, cur) -> None:
        if old.metadata.resourceVersion == cur.metadata.resourceVersion:
            return
        cur_ref, old_ref = get_controller_of(cur), get_controller_of(old)
        if old_ref is not None and (cur_ref is None or cur_ref.uid != old_ref.uid):
            job = self.resolve_controller_ref(old.metadata.namespace, old_ref)
            if job is not None:
                self.enqueue_tfjob(job)
        job = self._owner_of(cur)
        if job is not None:
            self.enqueue_tfjob(job)

    def delete_pod(self, pod) -> None:
        job = self._owner_of(pod)
        if job is not None:
            self.enqueue_tfjob(job)

    add_service = add_pod
    update_service = update_pod
    delete_service = delete_pod
