#!/usr/bin/env python3
"""The reference's distributed MNIST TFJob (``examples/tfjob/dist.yml``: 4 workers +
2 PS, async Adam, 200 global steps, batch 100) through controller -> kubelet ->
replica processes on this host's CPUs; prints the figures BASELINE.md compares
with the reference's sample log (``docs/get_started.md``: 9.54 s training
elapsed on worker 2, ≈35,600 examples/s steady-state aggregate):

* per-worker "Training elapsed time" and the max over workers;
* steady-state aggregate examples/s = Σ over workers of each worker's
  steady-state rate (first step -> last step, as derived from the reference log).

    python tools/mnist_dist_bench.py [--workers 4 --ps 2]
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
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--ps", type=int, default=2)
    ap.add_argument("--timeout", type=float, default=300)
    a = ap.parse_args(argv)
    from kubeflow_controller_amd.api import serde
    from kubeflow_controller_amd.cli.controller_main import Node
    from kubeflow_controller_amd.cli.kfctl import wait_for_phase
    from kubeflow_controller_amd.store import ObjectStore
    root = tempfile.mkdtemp(prefix="kfa-mnist-")
    st = ObjectStore()
    n = Node(st, kubelet=True, root_dir=root, num_gpus=0, resync=30, kubelet_backoff=0.2,
             extra_env={"OMP_NUM_THREADS": "1"}).start()
    try:
        job = serde.load_file(os.path.join(ROOT, "examples", "tfjob", "dist.yml"),
                              env={"KUBEFLOW_HOSTPATH": os.path.join(ROOT, "examples", "workdir")})[0]
        job.spec.specs[0].replicas = a.ps
        job.spec.specs[1].replicas = a.workers
        t0 = time.time()
        st.create(job)
        j = wait_for_phase(st, "default", "dist-training-job", {"Succeeded", "Failed"}, a.timeout)
        wall = time.time() - t0
        elapsed, rates = [], []
        for p in st.list("Pod"):
            if p.metadata.labels.get("job_type") != "Worker":
                continue
            d = os.path.join(root, f"default_{p.metadata.name}")
            out = "".join(open(os.path.join(d, f)).read() for f in os.listdir(d) if f.endswith(".log"))
            m = re.search(r"Training elapsed time: ([0-9.]+) s", out)
            r = re.search(r"Steady-state: [0-9.]+ steps/s/worker, ([0-9.]+) examples/s", out)
            if m:
                elapsed.append(float(m.group(1)))
            if r:
                rates.append(float(r.group(1)))
        res = {"phase": j.status.phase, "workers": a.workers, "ps": a.ps, "job_wall_s": round(wall, 2),
               "training_elapsed_s_max": max(elapsed) if elapsed else None,
               "steady_examples_per_s_aggregate": round(sum(rates), 1),
               "reference": {"training_elapsed_s": 9.536664, "steady_examples_per_s": 35600}}
        print(json.dumps(res))
        return 0 if j.status.phase == "Succeeded" else 1
    finally:
        n.shutdown()


if __name__ == "__main__":
    sys.exit(main())
