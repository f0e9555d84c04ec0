"""End-to-end on an MI355X: the controller + kubelet run TFJobs whose replicas
train on the GPU bound to them through the HIP kernels."""
import os
import sys

import pytest

from kubeflow_controller_amd.api import v1alpha1
from kubeflow_controller_amd.cli.controller_main import Node
from kubeflow_controller_amd.cli.kfctl import describe_tfjob, wait_for_phase
from kubeflow_controller_amd.store import ObjectStore

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRAIN = [sys.executable, os.path.join(ROOT, "examples", "workdir", "train.py")]


def _job(name, specs):
    out = []
    for typ, n, args, gpu in specs:
        c = {"name": "trainer", "command": TRAIN + args}
        if gpu:
            c["resources"] = {"limits": {"amd.com/gpu": gpu}}
        out.append({"replicas": n, "tfReplicaType": typ,
                    "template": {"spec": {"containers": [c], "restartPolicy": "OnFailure"}}})
    return v1alpha1.TFJob.from_json({"apiVersion": v1alpha1.API_VERSION, "kind": "TFJob",
                                     "metadata": {"name": name}, "spec": {"tfReplicaSpec": out}})


def _logs(root, pod):
    d = os.path.join(root, f"default_{pod.metadata.name}")
    return "".join(open(os.path.join(d, f)).read() for f in os.listdir(d) if f.endswith(".log"))


@pytest.fixture
def node(tmp_path):
    st = ObjectStore()
    n = Node(st, kubelet=True, root_dir=str(tmp_path), num_gpus=1, resync=30, kubelet_backoff=0.5,
             extra_env={"PYTHONPATH": ROOT}).start()
    yield st, n, str(tmp_path)
    n.shutdown()


def test_gpu_local_resnet_tfjob(node):
    st, n, root = node
    args = ["--model", "resnet_tiny", "--batch_size", "32", "--train_steps", "8", "--optimizer", "sgd",
            "--learning_rate", "0.05", "--momentum", "0.9", "--log_every", "4"]
    st.create(_job("rn-local", [("Local", 1, args, 1)]))
    j = wait_for_phase(st, "default", "rn-local", {"Succeeded", "Failed"}, 300)
    (p,) = st.list("Pod")
    out = _logs(root, p)
    assert j.status.phase == "Succeeded", describe_tfjob(st, "default", "rn-local") + out
    assert p.status.gpus == [0] and "device cuda:0" in out and "Final loss" in out


def test_gpu_bert_tiny_worker_plus_ps(node):
    st, n, root = node
    args = ["--model", "bert_tiny", "--batch_size", "8", "--seq_len", "64", "--train_steps", "6",
            "--optimizer", "adam", "--learning_rate", "1e-3", "--log_every", "2"]
    st.create(_job("bert-1w1ps", [("PS", 1, args, 0), ("Worker", 1, args, 1)]))
    j = wait_for_phase(st, "default", "bert-1w1ps", {"Succeeded", "Failed"}, 300)
    pods = st.list("Pod")
    w = next(p for p in pods if p.metadata.labels["job_type"] == "Worker")
    out = _logs(root, w)
    assert j.status.phase == "Succeeded", describe_tfjob(st, "default", "bert-1w1ps") + out
    assert "device cuda:0" in out and "1 workers, 1 ps" in out
