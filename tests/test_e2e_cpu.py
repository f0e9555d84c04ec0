"""End-to-end on CPU: controller + kubelet spawn real replica processes.

BASELINE config "examples/tfjob MNIST local TFJob, 1 worker + 0 PS on CPU (plumbing)"
plus a small PS/worker job, restart policies, deletion cascade and the CLI.
"""
import os
import signal
import subprocess
import sys
import textwrap
import time

import pytest

from kubeflow_controller_amd.api import serde, v1alpha1
from kubeflow_controller_amd.cli.controller_main import Node
from kubeflow_controller_amd.cli.kfctl import describe_tfjob, wait_for_phase
from kubeflow_controller_amd.store import ObjectStore

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = {"KUBEFLOW_HOSTPATH": os.path.join(ROOT, "examples", "workdir")}


@pytest.fixture
def node(tmp_path):
    st = ObjectStore()
    n = Node(st, kubelet=True, root_dir=str(tmp_path / "pods"), num_gpus=0, resync=30, kubelet_backoff=0.2,
             extra_env={"OMP_NUM_THREADS": "1"}).start()
    yield st, n, tmp_path / "pods"
    n.shutdown()


def _job(name, replicas_spec, restart="OnFailure", cmd=None):
    specs = []
    for typ, n, c in replicas_spec:
        specs.append({"replicas": n, "tfReplicaType": typ, "template": {"spec": {
            "containers": [{"name": "main", "command": c or cmd}],
            **({"restartPolicy": restart} if restart and typ != "PS" else {})}}})
    return v1alpha1.TFJob.from_json({"apiVersion": v1alpha1.API_VERSION, "kind": "TFJob",
                                     "metadata": {"name": name}, "spec": {"tfReplicaSpec": specs}})


def _alive(pid):
    """True while pid exists and is not a zombie (tolerates it vanishing mid-check)."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split()[2] != "Z"
    except (FileNotFoundError, ProcessLookupError, IndexError):
        return False


def _logs(root, pod):
    d = os.path.join(root, f"default_{pod.metadata.name}")
    return "".join(open(os.path.join(d, f)).read() for f in os.listdir(d) if f.endswith(".log"))


@pytest.mark.slow
def test_local_mnist_tfjob_succeeds(node):
    st, n, root = node
    job = serde.load_file(os.path.join(ROOT, "examples", "tfjob", "local.yml"), env=ENV)[0]
    st.create(job)
    # the reference's workload: 100,000 GD steps, "step: i" printed for every one
    j = wait_for_phase(st, "default", "local-training-job", {"Succeeded", "Failed"}, 300)
    assert j.status.phase == "Succeeded"
    assert j.status.tfReplicaStatuses[0].type == "Local"
    assert j.status.tfReplicaStatuses[0].tfReplicasStates == {"Succeeded": 1}
    (p,) = st.list("Pod")
    out = _logs(root, p)
    assert "Test accuracy:" in out and "step: 0\n" in out and "step: 99999\n" in out and "step: 50000\n" in out
    acc = float(out.split("Test accuracy:")[1].split()[0])
    assert acc > 0.8
    desc = describe_tfjob(st, "default", "local-training-job")
    assert "Created pod: " + p.metadata.name in desc


@pytest.mark.slow
def test_dist_ps_worker_job_wiring_and_recycling(node):
    st, n, root = node
    job = serde.load_file(os.path.join(ROOT, "examples", "tfjob", "dist.yml"), env=ENV)[0]
    job.spec.specs[0].replicas = 1
    job.spec.specs[1].replicas = 2
    st.create(job)
    j = wait_for_phase(st, "default", "dist-training-job", {"Succeeded", "Failed"}, 180)
    assert j.status.phase == "Succeeded"
    deadline = time.time() + 30
    while time.time() < deadline:  # PS replicas are recycled once the workers are done
        j = st.get(v1alpha1.TFJOB_KIND, "default", "dist-training-job")
        st_map = {s.type: s.tfReplicasStates for s in j.status.tfReplicaStatuses}
        if st_map.get("PS") == {"Succeeded": 1}:
            break
        time.sleep(0.2)
    assert st_map == {"Worker": {"Succeeded": 2}, "PS": {"Succeeded": 1}}, describe_tfjob(st, "default", "dist-training-job")
    pods = st.list("Pod")
    assert len(pods) == 3
    svcs = st.list("Service")
    assert len(svcs) == 3 and all(s.spec.ports[0].nodePort and s.spec.clusterIP == "127.0.0.1" for s in svcs)
    w0 = next(p for p in pods if p.metadata.labels["job_type"] == "Worker" and p.metadata.labels["index"] == "0")
    args = w0.spec.containers[0].args
    assert args[0].startswith("--worker_hosts=dist-training-job-worker-0-") and args[2] == "--job_name=worker"
    out = _logs(root, w0)
    assert "training step" in out and "validation cross entropy" in out
    assert "2 workers, 1 ps" in out


def test_restart_policies(node):
    st, n, root = node
    flag = str(root) + "_flag"
    script = textwrap.dedent(f"""
        import os, sys
        p = {flag!r}
        if not os.path.exists(p):
            open(p, "w").close(); sys.exit(3)
        sys.exit(0)""")
    st.create(_job("retry", [("Local", 1, [sys.executable, "-c", script])], restart="OnFailure"))
    j = wait_for_phase(st, "default", "retry", {"Succeeded", "Failed"}, 60)
    assert j.status.phase == "Succeeded"
    (p,) = st.list("Pod")
    assert p.status.containerStatuses[0].restartCount == 1
    assert p.status.containerStatuses[0].lastTerminated.exitCode == 0
    st.create(_job("never", [("Worker", 1, [sys.executable, "-c", "import sys; sys.exit(7)"])], restart="Never"))
    j = wait_for_phase(st, "default", "never", {"Succeeded", "Failed"}, 60)
    assert j.status.phase == "Failed"
    fp = [p for p in st.list("Pod") if p.metadata.labels.get("tf_job_name") == "never"][0]
    assert fp.status.phase == "Failed" and fp.status.containerStatuses[0].terminated.exitCode == 7


def test_delete_tfjob_kills_replicas(node):
    st, n, root = node
    st.create(_job("sleeper", [("Worker", 2, [sys.executable, "-c", "import time; time.sleep(300)"])]))
    deadline = time.time() + 30
    while time.time() < deadline and len(n.supervisor.running()) < 2:
        time.sleep(0.1)
    pids = list(n.supervisor.running().values())
    assert len(pids) == 2
    st.delete(v1alpha1.TFJOB_KIND, "default", "sleeper")
    deadline = time.time() + 20
    while time.time() < deadline and any(_alive(p) for p in pids):
        time.sleep(0.1)
    left = st.list("Pod") + st.list("Service")
    assert left == [], [(o.kind, o.metadata.name, o.metadata.resourceVersion, o.metadata.ownerReferences) for o in left]
    for p in pids:
        assert not _alive(p)


def test_ps_colocated_gpu_binding(tmp_path):
    """A PS template with KFA_PS_COLOCATE=1 (device-resident async PS) shares GPU
    index % num_gpus with the worker bound there; workers keep exclusive GPUs."""
    st = ObjectStore()
    n = Node(st, kubelet=True, root_dir=str(tmp_path), num_gpus=2, resync=30).start()
    try:
        cmd = [sys.executable, "-c", "import os; print('HIP=' + os.environ['HIP_VISIBLE_DEVICES'])"]
        job = _job("colo", [("PS", 2, cmd), ("Worker", 2, cmd)])
        from kubeflow_controller_amd.api.core import EnvVar
        job.spec.specs[0].template.spec.containers[0].env = [EnvVar(name="KFA_PS_COLOCATE", value="1")]
        st.create(job)
        wait_for_phase(st, "default", "colo", {"Succeeded"}, 60)
        pods = st.list("Pod")
        ps = sorted((p.metadata.labels["index"], p.status.gpus) for p in pods if p.metadata.labels["job_type"] == "PS")
        assert ps == [("0", [0]), ("1", [1])], ps
        w = sorted(p.status.gpus[0] for p in pods if p.metadata.labels["job_type"] == "Worker")
        assert w == [0, 1]
    finally:
        n.shutdown()


def test_gpu_binding_policy(tmp_path):
    """Workers get one GPU each (HIP_VISIBLE_DEVICES), PS none; binding released on exit."""
    st = ObjectStore()
    n = Node(st, kubelet=True, root_dir=str(tmp_path), num_gpus=2, resync=30).start()
    try:
        cmd = [sys.executable, "-c", "import os; print('HIP=' + os.environ['HIP_VISIBLE_DEVICES'])"]
        st.create(_job("g", [("PS", 1, cmd), ("Worker", 2, cmd)]))
        wait_for_phase(st, "default", "g", {"Succeeded"}, 60)
        pods = st.list("Pod")
        w = sorted(p.status.gpus[0] for p in pods if p.metadata.labels["job_type"] == "Worker")
        assert w == [0, 1]
        assert [p.status.gpus for p in pods if p.metadata.labels["job_type"] == "PS"] == [[]]
        for p in pods:
            if p.metadata.labels["job_type"] == "Worker":
                assert f"HIP={p.status.gpus[0]}" in _logs(str(tmp_path), p)
    finally:
        n.shutdown()


def test_gpu_binding_visible_mode(tmp_path):
    """gpu_binding="visible": every node GPU stays visible (the device set bench.py
    sees under torchrun) and each worker gets its own GPU as an ORDINAL
    (KFA_LOCAL_DEVICE), which the replica runtime turns into its device, its
    LOCAL_RANK and the physical index the async PS reports — the reference picks its
    device out of a fully visible set (mnist_replica.py:125-129)."""
    st = ObjectStore()
    n = Node(st, kubelet=True, root_dir=str(tmp_path), num_gpus=4, resync=30, gpu_binding="visible").start()
    try:
        code = ("import os; from kubeflow_controller_amd.trainer.cluster import local_device, parse_cluster; "
                "from kubeflow_controller_amd.parallel.async_ps import physical_gpu; "
                "print('HIP=' + os.environ['HIP_VISIBLE_DEVICES'] + ' DEV=%d' % local_device() + "
                "' LR=' + parse_cluster().torch_env()['LOCAL_RANK'] + ' PHYS=' + physical_gpu())")
        cmd = [sys.executable, "-c", code]
        st.create(_job("vis", [("PS", 1, cmd), ("Worker", 3, cmd)]))
        wait_for_phase(st, "default", "vis", {"Succeeded"}, 60)
        pods = st.list("Pod")
        ws = [p for p in pods if p.metadata.labels["job_type"] == "Worker"]
        assert sorted(p.status.gpus[0] for p in ws) == [0, 1, 2]
        for p in ws:
            g = p.status.gpus[0]
            assert f"HIP=0,1,2,3 DEV={g} LR={g} PHYS={g}" in _logs(str(tmp_path), p), _logs(str(tmp_path), p)
    finally:
        n.shutdown()


def test_local_device_isolated_default(monkeypatch):
    from kubeflow_controller_amd.parallel.async_ps import physical_gpu
    from kubeflow_controller_amd.trainer.cluster import local_device
    monkeypatch.delenv("KFA_LOCAL_DEVICE", raising=False)
    monkeypatch.setenv("KFA_GPUS", "5,2")  # isolated worker on GPU 5 seeing PS GPU 2
    assert local_device() == 0 and physical_gpu() == "5"
    monkeypatch.setenv("KFA_LOCAL_DEVICE", "bogus")
    assert local_device() == 0


@pytest.mark.slow
def test_cli_standalone_controller_and_kfctl(tmp_path):
    url_file = tmp_path / "url"
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", KFA_NODE_GPUS="0", **ENV)
    ctl = subprocess.Popen([sys.executable, os.path.join(ROOT, "bin", "kubeflow-controller"), "--standalone",
                            "--url-file", str(url_file), "--root-dir", str(tmp_path / "pods"), "-v", "4"],
                           env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        deadline = time.time() + 60
        while time.time() < deadline and not (url_file.exists() and url_file.read_text().strip()):
            time.sleep(0.1)
        url = url_file.read_text().strip()
        kf = [sys.executable, os.path.join(ROOT, "bin", "kfctl"), "--master", url]
        run = lambda *a: subprocess.run(kf + list(a), env=env, capture_output=True, text=True, timeout=120)
        r = run("create", "-f", os.path.join(ROOT, "examples", "crd", "crd.yml"))
        assert r.returncode == 0, r.stderr
        r = run("create", "-f", os.path.join(ROOT, "examples", "tfjob", "local.yml"))
        assert r.returncode == 0 and 'tfjob "local-training-job" created' in r.stdout, r.stderr
        r = run("wait", "tfjob", "local-training-job", "--timeout", "120")
        assert r.returncode == 0 and "Succeeded" in r.stdout, r.stdout + r.stderr
        r = run("get", "tfjobs")
        assert "local-training-job" in r.stdout and "Succeeded" in r.stdout
        r = run("get", "pods", "-o", "wide")
        assert "Succeeded" in r.stdout
        r = run("describe", "tfjob", "local-training-job")
        assert "SuccessfulCreate" in r.stdout and "Local: Succeeded=1" in r.stdout
        r = run("get", "tfjob", "local-training-job", "-o", "json")
        assert '"phase": "Succeeded"' in r.stdout
        r = run("metrics")
        assert r.returncode == 0 and "kfa_sync_duration_seconds" in r.stdout, r.stderr
        r = run("delete", "tfjob", "local-training-job")
        assert r.returncode == 0
    finally:
        ctl.send_signal(signal.SIGTERM)
        try:
            ctl.wait(20)
        except subprocess.TimeoutExpired:
            ctl.kill()


def test_fault_injection_restart_and_metrics(node):
    """kill -9 of a running replica (SURVEY §5.3 fault injection): OnFailure restarts
    it and the job still succeeds; the Prometheus metrics record the lifecycle."""
    from kubeflow_controller_amd.utils import metrics
    st, n, root = node
    flag = str(root) + "_fi_flag"
    script = textwrap.dedent(f"""
        import os, sys, time
        p = {flag!r}
        if not os.path.exists(p):
            open(p, "w").close(); time.sleep(60); sys.exit(5)
        sys.exit(0)""")
    st.create(_job("fi", [("Worker", 1, [sys.executable, "-c", script])], restart="OnFailure"))
    deadline = time.time() + 30
    while time.time() < deadline and not (n.supervisor.running() and os.path.exists(flag)):
        time.sleep(0.05)
    (key,) = n.supervisor.running()
    assert n.supervisor.inject_fault(*key.split("/"), signal.SIGKILL) > 0
    j = wait_for_phase(st, "default", "fi", {"Succeeded", "Failed"}, 60)
    assert j.status.phase == "Succeeded"
    (p,) = [p for p in st.list("Pod") if p.metadata.labels.get("tf_job_name") == "fi"]
    cs = p.status.containerStatuses[0]
    assert cs.restartCount == 1 and cs.terminated.exitCode == 0
    text = metrics.exposition().decode()
    if metrics.AVAILABLE:
        assert 'kfa_children_created_total{kind="Pod",result="success"}' in text
        assert "kfa_sync_duration_seconds_count" in text
        assert 'kfa_replica_exits_total{result="failure",type="Worker"}' in text


def _bert_job(name, workers, ps, model_dir, extra=()):
    cmd = [sys.executable, os.path.join(ROOT, "examples", "workdir", "train.py"), "--model", "bert_tiny",
           "--train_steps", "3", "--batch_size", "4", "--seq_len", "32", "--optimizer", "adam",
           "--learning_rate", "0.002", "--sync_replicas", "--log_every", "1", *extra]
    specs = ([("PS", ps, cmd)] if ps else []) + [("Worker", workers, cmd)]
    job = _job(name, specs)
    job.spec.modelDir = model_dir
    return job


def _single_process_bert(steps, world):
    """One process on the concatenation of every worker's synthetic batch."""
    import torch
    from kubeflow_controller_amd.models.bert import BertConfig, BertForPreTraining, bert_loss, synthetic_mlm_batch
    from kubeflow_controller_amd.trainer.engine import Engine
    cfg = BertConfig.tiny()
    torch.manual_seed(1234)
    m = BertForPreTraining(cfg)
    eng = Engine(m, bert_loss, optimizer="adam", lr=0.002, weight_decay=0.0, compute_dtype=None,
                 channels_last=False)
    parts = [synthetic_mlm_batch(cfg, 4, 32, torch.Generator().manual_seed(1234 + 1000 * r)) for r in range(world)]
    ids, tt, _, flat, labels, nsp = (list(x) for x in zip(*parts))
    flat = [f + r * 4 * 32 for r, f in enumerate(flat)]   # positions index the concatenated [B*S] rows
    batch = (torch.cat(ids), torch.cat(tt), None, torch.cat(flat), torch.cat(labels), torch.cat(nsp))
    for _ in range(steps):
        eng.train_step(*batch)
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


def _final_state(model_dir):
    import json
    import torch
    man = json.load(open(os.path.join(model_dir, "manifest.json")))
    return man, torch.load(os.path.join(model_dir, man["files"][0]), weights_only=True)


@pytest.mark.slow
@pytest.mark.parametrize("ps", [0, 1])
def test_multi_worker_tfjob_matches_single_process(node, tmp_path, ps):
    """A Worker-only 2-replica job (bucketed fp32 all-reduce) and a 2 workers + 1 PS
    job (``--ps_mode collective``: push to the PS task's co-located owner, owner-side
    Adam, pull) through controller -> supervisor -> replica runtime both reach
    Succeeded with the weights of one process trained on the concatenated batch."""
    import torch
    st, n, root = node
    model_dir = str(tmp_path / "model")
    name = f"bert-2w{ps}ps"
    st.create(_bert_job(name, 2, ps, model_dir, ["--ps_mode", "collective"] if ps else []))
    j = wait_for_phase(st, "default", name, {"Succeeded", "Failed"}, 240)
    assert j.status.phase == "Succeeded", describe_tfjob(st, "default", name)
    pods = [p for p in st.list("Pod") if p.metadata.labels.get("tf_job_name") == name]
    w0 = next(p for p in pods if p.metadata.labels["job_type"] == "Worker" and p.metadata.labels["index"] == "0")
    out = _logs(root, w0)
    assert ("push/pull to ps owners" if ps else "all-reduce") in out, out
    man, state = _final_state(model_dir)
    assert man["step"] == 3 and man["world"] == 2
    ref = _single_process_bert(3, 2)
    for k, v in ref.items():
        torch.testing.assert_close(state["model"][k], v, atol=1e-4, rtol=1e-4)  # Adam: lr 2e-3


def test_hung_replica_dumps_stacks_and_fails_job(node):
    """A replica wedged mid-training (KFA_TEST_HANG: worker 1 stops at step 2, so
    worker 0 blocks in the next all-reduce) trips the per-step watchdog
    (--hang_timeout): both replicas print every thread's stack into their logs and
    exit 1, and with restartPolicy Never the job ends Failed instead of hanging."""
    from kubeflow_controller_amd.api.core import EnvVar
    st, n, root = node
    cmd = [sys.executable, os.path.join(ROOT, "examples", "workdir", "mnist_replica.py"), "--device", "cpu",
           "--hang_timeout", "6", "--train_steps", "50", "--log_every", "1"]
    job = _job("hang", [("Worker", 2, cmd)], restart="Never")
    job.spec.specs[0].template.spec.containers[0].env = [EnvVar(name="KFA_TEST_HANG", value="worker:1:2")]
    t0 = time.time()
    st.create(job)
    j = wait_for_phase(st, "default", "hang", {"Succeeded", "Failed"}, 120)
    assert j.status.phase == "Failed", describe_tfjob(st, "default", "hang")
    assert time.time() - t0 < 100
    pods = {p.metadata.labels["index"]: p for p in st.list("Pod") if p.metadata.labels.get("tf_job_name") == "hang"}
    w1 = _logs(root, pods["1"])
    assert "hanging at step 2 on purpose" in w1
    for p in pods.values():
        out = _logs(root, p)
        assert "Timeout (0:00:06)!" in out and "most recent call first" in out, out[-3000:]
        assert p.status.containerStatuses[0].terminated.exitCode != 0


def test_async_ps_workers_see_ps_gpus(tmp_path):
    """The 4 workers + 2 PS device-resident async layout (bert-base-async-4w2ps.yml):
    each worker's HIP_VISIBLE_DEVICES lists its own GPU first (its compute device,
    cuda:0) and then the PS replicas' GPUs, so the PS buffers it maps by HIP IPC are
    on GPUs it can see; KFA_GPUS names the physical GPU of every local ordinal."""
    st = ObjectStore()
    n = Node(st, kubelet=True, root_dir=str(tmp_path), num_gpus=8, resync=30).start()
    try:
        job = serde.load_file(os.path.join(ROOT, "examples", "tfjob", "bert-base-async-4w2ps.yml"), env=ENV)[0]
        cmd = [sys.executable, "-c", "import os; print('HIP=' + os.environ['HIP_VISIBLE_DEVICES'] + ' KG=' + "
               "os.environ['KFA_GPUS'] + ' PSG=' + os.environ.get('KFA_PS_GPUS', '-'))"]
        for spec in job.spec.specs:
            spec.template.spec.containers[0].command = cmd
            spec.template.spec.containers[0].args = []
        st.create(job)
        wait_for_phase(st, "default", "bert-base-async-4w2ps", {"Succeeded"}, 60)
        pods = st.list("Pod")
        ps = {p.metadata.labels["index"]: p.status.gpus for p in pods if p.metadata.labels["job_type"] == "PS"}
        assert ps == {"0": [0], "1": [1]}, ps
        workers = [p for p in pods if p.metadata.labels["job_type"] == "Worker"]
        assert len(workers) == 4
        for p in workers:
            own = p.status.gpus[0]
            vis = [own] + [g for g in (0, 1) if g != own]
            want = ",".join(map(str, vis))
            out = _logs(str(tmp_path), p)
            assert f"HIP={want} KG={want} PSG=0,1" in out, out
    finally:
        n.shutdown()


def test_local_ordinal_of_ps_gpu(monkeypatch):
    from kubeflow_controller_amd.parallel.async_ps import local_ordinal, physical_gpu
    monkeypatch.setenv("KFA_GPUS", "5,0,1")
    assert physical_gpu() == "5"
    assert local_ordinal("1")[0] == 2 and local_ordinal("5")[0] == 0
    dev, why = local_ordinal("3")
    assert dev is None and "not visible" in why
    assert local_ordinal("")[0] == 0
    monkeypatch.delenv("KFA_GPUS")
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    assert local_ordinal("4")[0] == 4


@pytest.mark.parametrize("yml,nw,nps,owners", [("resnet50-2w1ps.yml", 2, 1, [0]),
                                               ("wide-deep-8w4ps.yml", 8, 4, [0, 2, 4, 6])])
def test_baseline_ps_layouts_bind_gpus_ranks_and_owners(tmp_path, yml, nw, nps, owners):
    """The BASELINE PS layouts through the real controller + kubelet on an 8-GPU node
    (replica commands swapped for a probe that parses its cluster spec exactly as
    trainer/replica.py does): every worker gets ONE exclusive GPU (HIP_VISIBLE_DEVICES),
    its collective rank is its task index, the PS replicas get no GPU, and the PS
    tasks' variables live on worker ranks ps_owner_ranks(W, P) (co-located owners,
    SURVEY §7.3 H1a)."""
    st = ObjectStore()
    n = Node(st, kubelet=True, root_dir=str(tmp_path), num_gpus=8, resync=30).start()
    try:
        job = serde.load_file(os.path.join(ROOT, "examples", "tfjob", yml), env=ENV)[0]
        probe = textwrap.dedent("""
            import os, sys
            sys.path.insert(0, %r)
            from kubeflow_controller_amd.trainer.cluster import add_cluster_flags, parse_cluster
            from kubeflow_controller_amd.parallel.ps import ps_owner_ranks
            import argparse
            ap = argparse.ArgumentParser(); add_cluster_flags(ap)
            a, _ = ap.parse_known_args()
            s = parse_cluster(a)
            env = s.torch_env()
            print('PROBE', s.job_name, s.task_index, env['RANK'], env['WORLD_SIZE'],
                  os.environ.get('HIP_VISIBLE_DEVICES', '-') or '-', len(s.ps),
                  ','.join(map(str, ps_owner_ranks(s.num_workers, len(s.ps)))))
        """ % ROOT)
        for spec in job.spec.specs:
            spec.template.spec.containers[0].command = [sys.executable, "-c", probe]
        st.create(job)
        wait_for_phase(st, "default", job.metadata.name, {"Succeeded"}, 90)
        pods = st.list("Pod")
        seen = {}
        for p in pods:
            line = [l for l in _logs(str(tmp_path), p).splitlines() if l.startswith("PROBE")][-1].split()
            seen[(line[1], int(line[2]))] = (line[3], line[4], line[5], int(line[6]), line[7], p.status.gpus)
        assert sorted(k for k in seen if k[0] == "worker") == [("worker", i) for i in range(nw)]
        assert sorted(k for k in seen if k[0] == "ps") == [("ps", i) for i in range(nps)]
        gpus = []
        for i in range(nw):
            rank, world, hip, ps_n, own, bound = seen[("worker", i)]
            assert rank == str(i) and world == str(nw) and ps_n == nps
            assert hip == str(bound[0]) and len(bound) == 1, (hip, bound)
            assert own == ",".join(map(str, owners))
            gpus.append(bound[0])
        assert sorted(gpus) == list(range(nw))           # exclusive, all distinct
        for i in range(nps):
            assert seen[("ps", i)][2] == "-" and seen[("ps", i)][5] == []
    finally:
        n.shutdown()
