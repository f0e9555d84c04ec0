"""API contract (JSON keys, serde, validation), object store and REST apiserver."""
import json
import os
import threading
import time

import pytest

from kubeflow_controller_amd.api import serde, v1alpha1
from kubeflow_controller_amd.api.core import Pod, Service
from kubeflow_controller_amd.api.labels import Selector
from kubeflow_controller_amd.api.meta import ObjectMeta, OwnerReference, generate_name
from kubeflow_controller_amd.api.validation import ValidationError, set_defaults, validate
from kubeflow_controller_amd.checker import is_local_job
from kubeflow_controller_amd.store import ObjectStore, RESTStore, errors
from kubeflow_controller_amd.store.apiserver import APIServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = {"KUBEFLOW_HOSTPATH": "/tmp/workdir"}


def load(name):
    return serde.load_file(os.path.join(ROOT, "examples", "tfjob", name), env=ENV)[0]


# ---------------------------------------------------------------- checker (port of pkg/checker/checker_test.go)
@pytest.mark.parametrize("t0", [v1alpha1.LOCAL, v1alpha1.PS])
@pytest.mark.parametrize("t1", [v1alpha1.LOCAL, v1alpha1.PS])
def test_is_local_job(t0, t1):
    job = v1alpha1.TFJob(spec=v1alpha1.TFJobSpec(specs=[v1alpha1.TFReplicaSpec(tfReplicaType=t0),
                                                        v1alpha1.TFReplicaSpec(tfReplicaType=t1)]))
    assert is_local_job(job) == (t0 == v1alpha1.LOCAL)


# ---------------------------------------------------------------- serde / JSON contract
def test_examples_round_trip_and_keys():
    for name in ("local.yml", "dist.yml"):
        job = load(name)
        d = job.to_json()
        assert d["apiVersion"] == "kubeflow.caicloud.io/v1alpha1" and d["kind"] == "TFJob"
        assert "tfReplicaSpec" in d["spec"] and isinstance(d["spec"]["tfReplicaSpec"], list)
        assert d["spec"]["runtimeID"] == ""                  # not omitempty (types.go:43)
        assert d["status"] == {"phase": "", "reason": "", "conditions": None, "tfReplicaStatuses": None}
        again = v1alpha1.TFJob.from_json(json.loads(json.dumps(d)))
        assert again.to_json() == d
        # unknown template keys (volumes, volumeMounts, ports...) survive the round trip
        tmpl = d["spec"]["tfReplicaSpec"][0]["template"]["spec"]
        assert tmpl["volumes"][0]["hostPath"]["path"] == "/tmp/workdir"
    dist = load("dist.yml")
    assert [s.tfReplicaType for s in dist.spec.specs] == ["PS", "Worker"]
    assert [s.replicas for s in dist.spec.specs] == [2, 4]
    assert dist.spec.specs[1].template.spec.restartPolicy == "OnFailure"
    assert dist.spec.specs[0].template.spec.restartPolicy == ""  # PS defaults to Always


def test_envsubst():
    assert serde.envsubst("a $X ${Y} $Z", {"X": "1", "Y": "2"}) == "a 1 2 "


def test_replicas_ptr_semantics():
    s = v1alpha1.TFReplicaSpec(replicas=0, tfReplicaType="Worker")
    assert s.to_json()["replicas"] == 0  # pointer: explicit 0 is emitted
    assert "replicas" not in v1alpha1.TFReplicaSpec(tfReplicaType="Worker").to_json()


def test_crd_manifest_matches_example():
    ex = serde.yaml.safe_load(open(os.path.join(ROOT, "examples", "crd", "crd.yml")))
    m = v1alpha1.crd_manifest()
    assert ex["metadata"]["name"] == m["metadata"]["name"] == "tfjobs.kubeflow.caicloud.io"
    assert ex["spec"]["names"] == m["spec"]["names"]


def test_validation_and_defaults():
    job = load("dist.yml")
    job.spec.specs[0].replicas = None
    set_defaults(job)
    assert job.spec.specs[0].replicas == 1 and job.metadata.namespace == "default"
    validate(job)
    bad = load("dist.yml")
    bad.spec.specs[0].tfReplicaType = "Chief"
    with pytest.raises(ValidationError):
        validate(bad)
    bad = load("local.yml")
    bad.spec.specs.append(bad.spec.specs[0].deep_copy())
    with pytest.raises(ValidationError):
        validate(bad)
    ps_only = load("dist.yml")
    ps_only.spec.specs = ps_only.spec.specs[:1]
    with pytest.raises(ValidationError):
        validate(ps_only)


def test_generate_name_and_selector():
    n = generate_name("job-")
    assert n.startswith("job-") and len(n) == 9
    sel = Selector.parse("a=1,b!=2,c,!d")
    assert sel.matches({"a": "1", "c": "x"})
    assert not sel.matches({"a": "1", "c": "x", "d": "y"})
    assert not sel.matches({"a": "1", "b": "2", "c": ""})
    assert Selector.parse(str(sel)).reqs == sel.reqs


# ---------------------------------------------------------------- store
def _pod(name="", gen="p-", labels=None, owner=None):
    meta = ObjectMeta(name=name, generateName=gen, labels=labels or {})
    if owner is not None:
        meta.ownerReferences = [OwnerReference(apiVersion=owner.apiVersion, kind=owner.kind, name=owner.metadata.name,
                                               uid=owner.metadata.uid, controller=True, blockOwnerDeletion=True)]
    return Pod(metadata=meta)


def test_store_semantics():
    st = ObjectStore()
    job = st.create(load("local.yml"))
    assert job.metadata.uid and job.metadata.resourceVersion == "1" and job.metadata.namespace == "default"
    with pytest.raises(errors.AlreadyExists):
        st.create(load("local.yml"))
    p = st.create(_pod(labels={"x": "1"}, owner=job))
    assert p.metadata.name.startswith("p-") and p.status.phase == "Pending"
    # identical update: no-op, same RV, no watch event
    w = st.watch("Pod")
    same = st.update(p)
    assert same.metadata.resourceVersion == p.metadata.resourceVersion
    assert w.next(timeout=0.05) is None
    # stale RV -> Conflict
    p2 = p.deep_copy()
    p2.status.phase = "Running"
    st.update(p2)
    p3 = p.deep_copy()
    p3.status.phase = "Failed"
    with pytest.raises(errors.Conflict):
        st.update(p3)
    assert w.next(timeout=1)[0] == "MODIFIED"
    # merge patch with uid precondition
    out = st.patch("Pod", "default", p.metadata.name, {"metadata": {"labels": {"y": "2"}}}, expect_uid=p.metadata.uid)
    assert out.metadata.labels == {"x": "1", "y": "2"}
    with pytest.raises(errors.Conflict):
        st.patch("Pod", "default", p.metadata.name, {"metadata": {"labels": {}}}, expect_uid="nope")
    assert [o.metadata.name for o in st.list("Pod", selector=Selector.parse("y=2"))] == [p.metadata.name]
    # cascade delete through ownerReferences
    st.delete(v1alpha1.TFJOB_KIND, "default", job.metadata.name)
    assert st.list("Pod") == []
    w.stop()


def test_store_orphan_delete_and_watch_resume():
    st = ObjectStore()
    job = st.create(load("local.yml"))
    rv0 = st.resource_version
    p = st.create(_pod(owner=job))
    st.delete(v1alpha1.TFJOB_KIND, "default", job.metadata.name, propagation="Orphan")
    (left,) = st.list("Pod")
    assert left.metadata.name == p.metadata.name and left.metadata.ownerReferences == []
    w = st.watch("Pod", resource_version=rv0)
    types = [w.next(timeout=1)[0], w.next(timeout=1)[0]]
    assert types == ["ADDED", "MODIFIED"]
    w.stop()


def test_store_persistence(tmp_path):
    st = ObjectStore(str(tmp_path))
    st.create(load("dist.yml"))
    st2 = ObjectStore(str(tmp_path))
    (job,) = st2.list(v1alpha1.TFJOB_KIND)
    assert job.metadata.name == "dist-training-job" and st2.resource_version == st.resource_version


def test_invalid_tfjob_rejected():
    st = ObjectStore()
    bad = load("dist.yml")
    bad.spec.specs[1].tfReplicaType = "Nope"
    with pytest.raises(errors.Invalid):
        st.create(bad)


# ---------------------------------------------------------------- REST apiserver + client
def test_rest_roundtrip_and_watch():
    srv = APIServer(ObjectStore()).start()
    try:
        cl = RESTStore(srv.url)
        job = cl.create(load("dist.yml"))
        assert job.metadata.uid
        got = cl.get(v1alpha1.TFJOB_KIND, "default", "dist-training-job")
        assert got.to_json() == job.to_json()
        w = cl.watch("Pod", "default")
        pod = cl.create(_pod(labels={"a": "b"}))
        etype, obj = w.next(timeout=5)
        assert etype == "ADDED" and obj.metadata.name == pod.metadata.name
        pod.status.phase = "Running"
        cl.update_status(pod)
        etype, obj = w.next(timeout=5)
        assert etype == "MODIFIED" and obj.status.phase == "Running"
        assert [p.metadata.name for p in cl.list("Pod", "default", Selector.parse("a=b"))] == [pod.metadata.name]
        with pytest.raises(errors.NotFound):
            cl.get("Pod", "default", "missing")
        cl.delete("Pod", "default", pod.metadata.name)
        assert w.next(timeout=5)[0] == "DELETED"
        w.stop()
        assert "tfjobs.kubeflow.caicloud.io" in cl.crds()
    finally:
        srv.stop()


def test_replicaset_control_and_rest_route():
    """C15 (dead code in the reference): ReplicaSet create/patch with events, served over REST."""
    from kubeflow_controller_amd.api.core import ReplicaSet
    from kubeflow_controller_amd.client.clientset import Clientset
    from kubeflow_controller_amd.client.events import FakeRecorder
    from kubeflow_controller_amd.controller.control import RealReplicaSetControl
    srv = APIServer(ObjectStore()).start()
    try:
        cl = RESTStore(srv.url)
        job = cl.create(load("local.yml"))
        rec = FakeRecorder()
        ctl = RealReplicaSetControl(Clientset(cl), rec)
        rs = ReplicaSet.from_json({"metadata": {"name": "rs1"}, "spec": {"replicas": 2, "template": {
            "metadata": {"labels": {"a": "b"}}, "spec": {"containers": [{"name": "c"}]}}}})
        ref = OwnerReference(apiVersion=job.apiVersion, kind=job.kind, name=job.metadata.name, uid=job.metadata.uid,
                             controller=True, blockOwnerDeletion=True)
        out = ctl.create_replica_sets_with_controller_ref("default", rs, job, ref)
        assert out.metadata.uid and out.spec.replicas == 2
        assert rec.events == ["Normal SuccessfulCreate Created replicaset: rs1"]
        ctl.patch_replica_set("default", "rs1", {"spec": {"replicas": 3}})
        assert cl.get("ReplicaSet", "default", "rs1").spec.replicas == 3
        with pytest.raises(ValueError):
            ctl.create_replica_sets("default", ReplicaSet(), job)
    finally:
        srv.stop()


def test_all_example_tfjobs_parse_and_validate():
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "examples", "tfjob", "*.yml")))
    assert len(files) >= 6
    for f in files:
        (job,) = serde.load_file(f, env=ENV)
        set_defaults(job)
        validate(job)
        assert job.to_json()["spec"]["tfReplicaSpec"]
