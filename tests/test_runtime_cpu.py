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
