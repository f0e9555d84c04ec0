"""Replica runtime on CPU: checkpoint / resume and job-dir plumbing."""
import json
import os

import torch

from kubeflow_controller_amd.api import v1alpha1
from kubeflow_controller_amd.planner.distributed import DistributedJob
from kubeflow_controller_amd.planner.local import LocalJob
from kubeflow_controller_amd.trainer import checkpoint, replica


def _run_local(capsys, *extra):
    rc = replica.main(["--model", "mnist_softmax", "--optimizer", "sgd", "--learning_rate", "0.5",
                       "--batch_size", "100", "--log_every", "0", "--device", "cpu", *extra])
    assert rc == 0
    return capsys.readouterr().out


def test_checkpoint_resume_local(tmp_path, capsys):
    d = str(tmp_path / "model")
    out = _run_local(capsys, "--train_steps", "20", "--model_dir", d, "--checkpoint_every", "5")
    assert "resumed" not in out
    man = json.load(open(os.path.join(d, "manifest.json")))
    assert man["step"] == 20 and man["world"] == 1
    state = torch.load(os.path.join(d, man["files"][0]), weights_only=True)
    assert state["step"] == 20 and state["opt"]["step_count"] == 20
    out = _run_local(capsys, "--train_steps", "35", "--model_dir", d)
    assert "resumed from" in out and "global step 20" in out
    man = json.load(open(os.path.join(d, "manifest.json")))
    assert man["step"] == 35
    state = torch.load(os.path.join(d, man["files"][0]), weights_only=True)
    assert state["opt"]["step_count"] == 35
    # old checkpoints pruned (keep 2)
    steps = {f.split("-")[1].split(".")[0] for f in os.listdir(d) if f.startswith("ckpt-")}
    assert len(steps) <= 2 and "35" in steps
    # nothing left to do: a third run resumes and trains 0 steps
    out = _run_local(capsys, "--train_steps", "35", "--model_dir", d)
    assert "global step 35" in out


def _job(model_dir):
    spec = {"replicas": 1, "tfReplicaType": "Worker",
            "template": {"spec": {"containers": [{"name": "m", "command": ["x"],
                                                  "env": [{"name": "A", "value": "1"}]}]}}}
    ps = dict(spec, tfReplicaType="PS")
    return v1alpha1.TFJob.from_json({"apiVersion": v1alpha1.API_VERSION, "kind": "TFJob",
                                     "metadata": {"name": "j", "namespace": "default", "uid": "u1"},
                                     "spec": {"modelDir": model_dir, "tfReplicaSpec": [ps, spec]}})


def test_spec_model_dir_reaches_replicas():
    job = _job("/data/ckpt")
    dj = DistributedJob(job, [], [], [], [], 0)
    dj.action()
    env = {e.name: e.value for e in dj.get_spec(v1alpha1.WORKER, 0).spec.containers[0].env}
    assert env["KFA_MODEL_DIR"] == "/data/ckpt" and env["A"] == "1" and "TF_CONFIG" in env
    # the TFJob's own template is not mutated
    assert [e.name for e in job.spec.specs[1].template.spec.containers[0].env] == ["A"]
    local = v1alpha1.TFJob.from_json(dict(_job("/m").to_json(), spec={
        "modelDir": "/m", "tfReplicaSpec": [dict(_job("/m").to_json()["spec"]["tfReplicaSpec"][1],
                                                 tfReplicaType="Local")]}))
    lj = LocalJob(local, [], 0)
    lj.action()
    env = {e.name: e.value for e in lj.get_template().spec.containers[0].env}
    assert env["KFA_MODEL_DIR"] == "/m"
    assert checkpoint.latest("") is None


def test_routes_table_lookup_dump_and_summary(tmp_path, monkeypatch):
    """ops/routes.py: a committed table entry is applied by candidate NAME without
    timing (no GPU needed), summary() names the table by hash and counts table vs
    timed / own vs library picks, dump() writes a re-loadable table."""
    import json
    from kubeflow_controller_amd.ops import routes
    tab = tmp_path / "routes_test.json"
    tab.write_text(json.dumps({"arch": "gfx950", "routes": {"proj|32768,2304,768": "ppp256",
                                                            "conv_fwd|1,2,3": "igemm", "bn_apply|4": "sep",
                                                            "dense_fwd|9": "hipblaslt"}}))
    monkeypatch.setattr(routes, "TABLE_PATH", str(tab))
    monkeypatch.setattr(routes, "MODE", "on")
    monkeypatch.setattr(routes, "_table", None)
    monkeypatch.setattr(routes, "_made", {})
    boom = lambda: (_ for _ in ()).throw(AssertionError("timed a table hit"))  # noqa: E731
    i = routes.decide("proj", (32768, 2304, 768), None, [("hipblaslt", boom), ("ppp192", boom), ("ppp256", boom)])
    assert i == 2
    assert routes.decide("conv_fwd", (1, 2, 3), None, [("igemm", boom), ("pp", boom)]) == 0
    # the separate own BatchNorm apply ("sep") is an own kernel; hipBLASLt is the library
    assert routes.decide("bn_apply", (4,), None, [("pro", boom), ("sep", boom)]) == 1
    assert routes.decide("dense_fwd", (9,), None, [("hipblaslt", boom), ("ppw256", boom)]) == 0
    s = routes.summary()
    assert s["from_table"] == 4 and s["timed"] == 0 and s["own"] == 3 and s["library"] == 1
    assert s["table"] == "routes_test.json" and len(s["table_sha"]) == 12
    out = tmp_path / "dumped.json"
    routes.dump(str(out))
    doc = json.loads(out.read_text())
    assert doc["routes"] == {"conv_fwd|1,2,3": "igemm", "proj|32768,2304,768": "ppp256", "bn_apply|4": "sep",
                             "dense_fwd|9": "hipblaslt"}
