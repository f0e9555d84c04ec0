"""Planner, cluster spec, updaters, ref manager, workqueue/expectations, controller loop (fakes)."""
import json
import os
import threading
import time

import pytest

from kubeflow_controller_amd.api import serde, v1alpha1
from kubeflow_controller_amd.api.core import Pod, PodStatus, Service
from kubeflow_controller_amd.api.labels import Selector
from kubeflow_controller_amd.api.meta import ObjectMeta, OwnerReference
from kubeflow_controller_amd.client import workqueue as wq
from kubeflow_controller_amd.client.clientset import Clientset
from kubeflow_controller_amd.client.events import FakeRecorder
from kubeflow_controller_amd.client.informer import SharedInformerFactory
from kubeflow_controller_amd.controller import (Controller, DistributedUpdater, FakePodControl, FakeServiceControl,
                                                LocalUpdater, PodControllerRefManager, get_pod_from_template,
                                                new_controller_ref)
from kubeflow_controller_amd.planner import Action, DistributedJob, LocalJob
from kubeflow_controller_amd.store import ObjectStore

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(name):
    job = serde.load_file(os.path.join(ROOT, "examples", "tfjob", name), env={"KUBEFLOW_HOSTPATH": "/w"})[0]
    job.metadata.uid = "uid-" + name
    job.metadata.namespace = "default"
    return job


def pod(phase, typ="Worker", index=0, job=None):
    labels = {"kubeflow.caicloud.io": "true", "job_type": typ, "index": str(index)}
    if job is not None:
        labels.update(runtime_id=job.spec.runtimeID, tf_job_name=job.metadata.name)
    return Pod(metadata=ObjectMeta(name=f"p{typ}{index}", namespace="default", labels=labels),
               status=PodStatus(phase=phase))


def svc(typ, index):
    return Service(metadata=ObjectMeta(name=f"s-{typ}-{index}-abcde", labels={"index": str(index)}))


# ---------------------------------------------------------------- planners
def test_local_planner():
    job = load("local.yml")
    ev = LocalJob(job, [], 0).action()
    assert ev.action == Action.ShouldAddWorker and ev.number == 1
    assert len(job.spec.runtimeID) == 5
    assert job.spec.specs[0].template.metadata.labels == {
        "kubeflow.caicloud.io": "true", "job_type": "Local", "runtime_id": job.spec.runtimeID,
        "tf_job_name": "local-training-job"}
    rid = job.spec.runtimeID
    assert LocalJob(job, [], 0).action().action == Action.ShouldAddWorker
    assert job.spec.runtimeID == rid  # minted once (fix of distributed.go:95,214)
    assert LocalJob(job, [pod("Running")], 0).action().action == Action.Nothing
    assert LocalJob(job, [], 1).action().action == Action.Nothing


def test_distributed_planner_fresh_job_sequence():
    job = load("dist.yml")
    dj = DistributedJob(job, [], [], [], [], 0)
    evs = dj.action()
    assert [(e.action, e.number) for e in evs] == [
        (Action.ShouldAddWorkerService, 4), (Action.ShouldAddPSService, 2),
        (Action.ShouldAddWorker, 4), (Action.ShouldAddPS, 2)]
    for i in range(4):
        s = dj.get_service(v1alpha1.WORKER, i)
        assert s.metadata.name.startswith(f"dist-training-job-worker-{i}-") and len(s.metadata.name) == len(
            f"dist-training-job-worker-{i}-") + 5
        assert s.spec.ports[0].port == 2222 and s.spec.ports[0].name == "kubeflow-port"
        assert s.spec.selector["index"] == str(i) and s.spec.selector["job_type"] == "Worker"
    for i in range(2):
        dj.get_service(v1alpha1.PS, i)
    t = dj.get_spec(v1alpha1.WORKER, 2)
    args = t.spec.containers[0].args
    workers = [dj.service_names[f"dist-training-job-worker-{i}"] + ":2222" for i in range(4)]
    ps = [dj.service_names[f"dist-training-job-ps-{i}"] + ":2222" for i in range(2)]
    assert args == ["--worker_hosts=" + ",".join(workers), "--ps_hosts=" + ",".join(ps), "--job_name=worker",
                    "--task_index=2"]
    assert t.metadata.labels["index"] == "2"
    tfc = json.loads({e.name: e.value for e in t.spec.containers[0].env}["TF_CONFIG"])
    assert tfc == {"cluster": {"worker": workers, "ps": ps}, "task": {"type": "worker", "index": 2},
                   "environment": "cloud"}
    assert dj.get_spec(v1alpha1.PS, 1).spec.containers[0].args[2:] == ["--job_name=ps", "--task_index=1"]


def test_distributed_planner_partial_states():
    job = load("dist.yml")
    job.spec.runtimeID = "abcde"
    wsv = [svc("worker", i) for i in range(4)]
    psv = [svc("ps", i) for i in range(2)]
    running = [pod("Running", "Worker", i, job) for i in range(4)]
    ps = [pod("Running", "PS", i, job) for i in range(2)]
    assert [e.action for e in DistributedJob(job, running, ps, wsv, psv, 0).action()] == [Action.Nothing]
    # worker 1 failed and is inactive: recreate exactly index 1, keep the runtime id
    evs = DistributedJob(job, [running[0], running[2], running[3]], ps, wsv, psv, 0).action()
    assert [(e.action, e.indices) for e in evs] == [(Action.ShouldAddWorker, [1])]
    assert job.spec.runtimeID == "abcde"
    # one worker already succeeded: expected = replicas - succeeded
    evs = DistributedJob(job, running[1:], ps, wsv, psv, 1, [0]).action()
    assert [e.action for e in evs] == [Action.Nothing]
    # missing service index 3 only
    evs = DistributedJob(job, running, ps, wsv[:3], psv, 0).action()
    assert [(e.action, e.indices) for e in evs] == [(Action.ShouldAddWorkerService, [3]), (Action.Nothing, [])]
    # all workers succeeded: job complete, nothing re-created (PS recycling)
    assert [e.action for e in DistributedJob(job, [], [], wsv, psv, 4, [0, 1, 2, 3]).action()] == [Action.Nothing]
    # re-created replica resolves existing service names (fix of distributed.go:131,142)
    dj = DistributedJob(job, running[1:], ps, wsv, psv, 0)
    dj.action()
    assert ":2222" != dj.get_spec(v1alpha1.WORKER, 0).spec.containers[0].args[0].split("=")[1].split(",")[0]


def test_worker_only_job():
    job = load("dist.yml")
    job.spec.specs = job.spec.specs[1:]
    evs = DistributedJob(job, [], [], [], [], 0).action()
    assert [(e.action, e.number) for e in evs] == [(Action.ShouldAddWorkerService, 4), (Action.ShouldAddWorker, 4)]


# ---------------------------------------------------------------- updaters
def test_local_updater():
    job = load("local.yml")
    assert LocalUpdater(job, 0, [pod("Pending", "Local")]).should_update()
    assert job.status.phase == "Running"
    assert job.status.tfReplicaStatuses[0].to_json() == {"type": "Local", "state": "",
                                                         "tfReplicasStates": {"Pending": 1}}
    assert not LocalUpdater(job, 0, [pod("Pending", "Local")]).should_update()  # unchanged -> no write
    assert LocalUpdater(job, 1, [pod("Succeeded", "Local")]).should_update()
    assert job.status.phase == "Succeeded"


def test_distributed_updater_histogram_and_phases():
    job = load("dist.yml")
    workers = [pod("Running", "Worker", i) for i in range(3)] + [pod("Succeeded", "Worker", 3)]
    ps = [pod("Running", "PS", i) for i in range(2)]
    assert DistributedUpdater(job, 1, workers, ps).should_update()
    st = {s.type: s.tfReplicasStates for s in job.status.tfReplicaStatuses}
    assert job.status.phase == "Running" and st == {"Worker": {"Running": 3, "Succeeded": 1}, "PS": {"Running": 2}}
    done = [pod("Succeeded", "Worker", i) for i in range(4)]
    assert DistributedUpdater(job, 4, done, ps).should_update()
    assert job.status.phase == "Succeeded"
    assert job.status.conditions[0].type == "Recycling" and job.status.conditions[0].status == "True"
    # restartPolicy Never + failed worker -> Failed (the reference never sets Failed)
    job2 = load("dist.yml")
    job2.spec.specs[1].template.spec.restartPolicy = "Never"
    DistributedUpdater(job2, 0, [pod("Failed", "Worker", 0)] + workers[1:3], ps).should_update()
    assert job2.status.phase == "Failed"


# ---------------------------------------------------------------- pod control / ref manager
def test_get_pod_from_template_and_controller_ref():
    job = load("dist.yml")
    ref = new_controller_ref(job)
    assert ref.to_json() == {"apiVersion": "kubeflow.caicloud.io/v1alpha1", "kind": "TFJob",
                             "name": "dist-training-job", "uid": job.metadata.uid, "controller": True,
                             "blockOwnerDeletion": True}
    t = job.spec.specs[1].template
    t.metadata.labels = {"a": "b"}
    p = get_pod_from_template(t, job, ref)
    assert p.metadata.generateName == "dist-training-job-"
    assert "kubernetes.io/created-by" in p.metadata.annotations
    assert p.metadata.ownerReferences[0].uid == job.metadata.uid


def test_claim_pods_matrix():
    job = load("dist.yml")
    job.metadata.uid = "me"
    sel = Selector.from_match_labels({"x": "1"})
    ctl = FakePodControl()
    mgr = PodControllerRefManager(ctl, job, sel, "TFJob", v1alpha1.API_VERSION)

    def mk(name, labels, owner_uid=None):
        meta = ObjectMeta(name=name, namespace="default", labels=labels, uid=name)
        if owner_uid:
            meta.ownerReferences = [OwnerReference(kind="TFJob", name="o", uid=owner_uid, controller=True)]
        return Pod(metadata=meta)

    owned_match = mk("a", {"x": "1"}, "me")
    owned_mismatch = mk("b", {"x": "2"}, "me")
    orphan_match = mk("c", {"x": "1"})
    orphan_mismatch = mk("d", {"x": "2"})
    other = mk("e", {"x": "1"}, "someone-else")
    claimed = mgr.claim_pods([owned_match, owned_mismatch, orphan_match, orphan_mismatch, other])
    assert [p.metadata.name for p in claimed] == ["a", "c"]
    assert len(ctl.patches) == 2  # release b, adopt c
    release, adopt = ctl.patches
    assert release["metadata"]["ownerReferences"] == []
    assert adopt["metadata"]["ownerReferences"][0]["uid"] == "me"
    # a deleting controller neither adopts nor releases
    job.metadata.deletionTimestamp = "2024-01-01T00:00:00Z"
    ctl.clear()
    mgr2 = PodControllerRefManager(ctl, job, sel, "TFJob", v1alpha1.API_VERSION)
    assert [p.metadata.name for p in mgr2.claim_pods([owned_mismatch, orphan_match])] == []
    assert ctl.patches == []


# ---------------------------------------------------------------- workqueue / rate limiters / expectations
def test_workqueue_dedup_and_processing_exclusivity():
    q = wq.RateLimitingQueue(None, "t")
    q.add("a"); q.add("a"); q.add("b")
    assert len(q) == 2
    item, _ = q.get()
    assert item == "a"
    q.add("a")          # re-added while processing: deferred to done()
    assert len(q) == 1
    item2, _ = q.get()
    assert item2 == "b"
    q.done("a")
    assert len(q) == 1 and q.get()[0] == "a"
    q.shut_down()
    assert q.get(0.1) == (None, True)


def test_rate_limiters_with_fake_clock():
    wq.set_fake_clock(1000.0)
    try:
        exp = wq.ItemExponentialFailureRateLimiter(0.005, 1000.0)
        assert [round(exp.when("k"), 4) for _ in range(4)] == [0.005, 0.01, 0.02, 0.04]
        assert exp.num_requeues("k") == 4
        exp.forget("k")
        assert exp.when("k") == 0.005
        for _ in range(40):
            exp.when("z")
        assert exp.when("z") == 1000.0
        bucket = wq.BucketRateLimiter(10.0, 100)
        delays = [bucket.when("x") for _ in range(101)]
        assert all(d == 0 for d in delays[:100]) and abs(delays[100] - 0.1) < 1e-9
        q = wq.RateLimitingQueue(wq.ItemExponentialFailureRateLimiter(1.0, 10.0), "d")
        q.add_rate_limited("k")
        q.poll_delayed()
        assert len(q) == 0 and q.num_waiting() == 1
        wq.advance_fake_clock(1.5)
        q.poll_delayed()
        assert len(q) == 1
        q.shut_down()
    finally:
        wq.use_real_clock()


def test_expectations_ttl_and_accounting():
    wq.set_fake_clock(0.0)
    try:
        e = wq.ControllerExpectations(300.0)
        assert e.satisfied_expectations("k")          # absent
        e.expect_creations("k", 2)
        assert not e.satisfied_expectations("k")
        e.creation_observed("k")
        assert not e.satisfied_expectations("k")
        e.creation_observed("k")
        assert e.satisfied_expectations("k")          # fulfilled
        e.expect_creations("k", 3)
        e.expect_creations("k", 1)                    # overwrite (reference SetExpectations)
        assert e.get_expectations("k")[0] == 1
        e.raise_expectations("k", 2, 0)               # accumulate (fix)
        assert e.get_expectations("k")[0] == 3
        wq.advance_fake_clock(301.0)
        assert e.satisfied_expectations("k")          # expired (5 min TTL)
        e.delete_expectations("k")
        assert e.get_expectations("k") is None
    finally:
        wq.use_real_clock()


# ---------------------------------------------------------------- controller with fake pod/service control
def _controller(store, pod_ctl=None, svc_ctl=None):
    cs = Clientset(store)
    kinf, tinf = SharedInformerFactory(store, 0), SharedInformerFactory(store, 0)
    rec = FakeRecorder()
    c = Controller(cs, cs, kinf, tinf, recorder=rec, pod_control=pod_ctl, service_control=svc_ctl)
    stop = threading.Event()
    kinf.start(stop)
    tinf.start(stop)
    assert kinf.wait_for_cache_sync(5) and tinf.wait_for_cache_sync(5)
    return c, rec, stop


def _drain(c, n=20):
    for _ in range(n):
        if not c.process_next_work_item(timeout=0.3):
            break


def test_controller_creates_with_fake_controls():
    st = ObjectStore()
    pc, sc = FakePodControl(), FakeServiceControl()
    c, rec, stop = _controller(st, pc, sc)
    try:
        st.create(load("dist.yml"))
        _drain(c, 3)
        assert len(sc.services) == 6 and len(pc.templates) == 6
        types = sorted(t.metadata.labels["job_type"] + t.metadata.labels["index"] for t in pc.templates)
        assert types == ["PS0", "PS1", "Worker0", "Worker1", "Worker2", "Worker3"]
        assert all(r.controller and r.blockOwnerDeletion for r in pc.controller_refs)
        job = st.get(v1alpha1.TFJOB_KIND, "default", "dist-training-job")
        assert len(job.spec.runtimeID) == 5  # written back with Update
        # expectations unmet (fakes create nothing): a re-sync must not create again
        c.workqueue.add("default/dist-training-job")
        _drain(c, 2)
        assert len(pc.templates) == 6
    finally:
        stop.set()
        c.workqueue.shut_down()


def test_controller_real_controls_events_and_status():
    st = ObjectStore()
    c, rec, stop = _controller(st)
    try:
        st.create(load("local.yml"))
        _drain(c, 3)
        (p,) = st.list("Pod")
        assert p.metadata.labels["job_type"] == "Local" and p.metadata.generateName == "local-training-job-"
        assert rec.events == [f"Normal SuccessfulCreate Created pod: {p.metadata.name}"]
        job = st.get(v1alpha1.TFJOB_KIND, "default", "local-training-job")
        assert job.status.phase == "Running"
        for phase in ("Running", "Succeeded"):
            p = st.get("Pod", "default", p.metadata.name)
            p.status.phase = phase
            st.update_status(p)
            deadline = time.time() + 5
            while time.time() < deadline:
                _drain(c, 2)
                job = st.get(v1alpha1.TFJOB_KIND, "default", "local-training-job")
                if job.status.tfReplicaStatuses and phase in job.status.tfReplicaStatuses[0].tfReplicasStates:
                    break
        assert job.status.phase == "Succeeded"
        assert job.status.tfReplicaStatuses[0].tfReplicasStates == {"Succeeded": 1}
        assert len(st.list("Pod")) == 1  # nothing re-created after success
    finally:
        stop.set()
        c.workqueue.shut_down()


def test_controller_recreates_deleted_replica():
    st = ObjectStore()
    c, rec, stop = _controller(st)
    try:
        st.create(load("local.yml"))
        _drain(c, 3)
        (p,) = st.list("Pod")
        st.delete("Pod", "default", p.metadata.name)  # delete events enqueue the owner (fix)
        deadline = time.time() + 5
        while time.time() < deadline and not [x for x in st.list("Pod") if x.metadata.name != p.metadata.name]:
            _drain(c, 2)
        (p2,) = st.list("Pod")
        assert p2.metadata.name != p.metadata.name
        assert p2.metadata.labels["runtime_id"] == p.metadata.labels["runtime_id"]
    finally:
        stop.set()
        c.workqueue.shut_down()
