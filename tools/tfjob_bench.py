#!/usr/bin/env python3
"""Throughput of a TFJob run the way a user runs it: the YAML goes to the
controller, the kubelet starts the replica processes (one per GPU), each runs
``trainer/replica.py`` — controller -> supervisor -> run_worker, the path the
reference drives (``pkg/controller/controller.go`` creating pods,
``examples/workdir/mnist_replica.py`` training).  Prints ONE JSON line with the
job's steady-state examples/s as logged by worker 0 ("Steady-state: ... (job)")
next to the job's phase and wall time.

    python tools/tfjob_bench.py examples/tfjob/resnet50-dp8.yml --workers 1 --steps 60
"""
import argparse
import json
import os
import re
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("yaml")
    ap.add_argument("--workers", type=int, default=None, help="override Worker replicas")
    ap.add_argument("--ps", type=int, default=None, help="override PS replicas")
    ap.add_argument("--steps", type=int, default=None, help="override --train_steps")
    ap.add_argument("--gpus", type=int, default=None, help="GPUs the kubelet hands out (default: visible count)")
    ap.add_argument("--timeout", type=float, default=900)
    a = ap.parse_args(argv)
    from kubeflow_controller_amd.api import serde
    from kubeflow_controller_amd.cli.controller_main import Node
    from kubeflow_controller_amd.cli.kfctl import wait_for_phase
    from kubeflow_controller_amd.store import ObjectStore
    gpus = a.gpus
    if gpus is None:
        import torch  # device_count() does not initialise the GPU on this image
        gpus = torch.cuda.device_count()
    root = tempfile.mkdtemp(prefix="kfa-tfjob-")
    st = ObjectStore()
    n = Node(st, kubelet=True, root_dir=root, num_gpus=gpus, resync=30, kubelet_backoff=0.2).start()
    try:
        job = serde.load_file(os.path.join(ROOT, a.yaml) if not os.path.isabs(a.yaml) else a.yaml,
                              env={"KUBEFLOW_HOSTPATH": os.path.join(ROOT, "examples", "workdir")})[0]
        for spec in job.spec.specs:
            if spec.tfReplicaType == "Worker" and a.workers is not None:
                spec.replicas = a.workers
            if spec.tfReplicaType == "PS" and a.ps is not None:
                spec.replicas = a.ps
            if a.steps is not None:
                for c in spec.template.spec.containers:
                    cmd = list(c.command)
                    if "--train_steps" in cmd:
                        cmd[cmd.index("--train_steps") + 1] = str(a.steps)
                    c.command = cmd
        job.spec.specs = [s for s in job.spec.specs if s.replicas > 0]
        t0 = time.time()
        st.create(job)
        j = wait_for_phase(st, job.metadata.namespace or "default", job.metadata.name, {"Succeeded", "Failed"},
                           a.timeout)
        wall = time.time() - t0
        rate, logs = None, {}
        for p in st.list("Pod"):
            d = os.path.join(root, f"default_{p.metadata.name}")
            if not os.path.isdir(d):
                continue
            out = "".join(open(os.path.join(d, f)).read() for f in sorted(os.listdir(d)) if f.endswith(".log"))
            logs[p.metadata.name] = out[-2000:]
            m = re.search(r"Steady-state: [0-9.]+ steps/s/worker, ([0-9.]+) examples/s \(job\)", out)
            if m and p.metadata.labels.get("job_type") == "Worker" and p.metadata.labels.get("index") in ("0", 0):
                rate = float(m.group(1))
            elif m and rate is None:
                rate = float(m.group(1))
        res = {"yaml": a.yaml, "phase": j.status.phase, "workers": a.workers, "ps": a.ps, "gpus": gpus,
               "job_wall_s": round(wall, 1), "steady_examples_per_s": rate}
        print(json.dumps(res), flush=True)
        if j.status.phase != "Succeeded":
            for k, v in logs.items():
                print(f"--- {k}\n{v}", file=sys.stderr)
        return 0 if j.status.phase == "Succeeded" else 1
    finally:
        n.shutdown()


if __name__ == "__main__":
    sys.exit(main())
