"""Replica-side cluster spec: what a TFJob replica process learns about its job.

Inputs, exactly as the controller produces them:

* flags ``--worker_hosts=a:2222,b:2222 --ps_hosts=... --job_name=worker|ps
  --task_index=i`` (``pkg/tensorflow/distributed.go:127-159``,
  ``mnist_replica.py:55-85``);
* ``TF_CONFIG`` JSON ``{"cluster": {...}, "task": {"type", "index"}}``;
* ``KFA_SERVICE_HOSTS`` — the supervisor's service-name resolution map
  (``"<svc>:2222" -> "127.0.0.1:<port>"``), the kube-dns stand-in.

Output: the role and the ``torch.distributed`` wiring.  Collective world =
the WORKER replicas (rank = task index); the chief (worker 0) hosts the TCP
rendezvous store on its own endpoint.  PS replicas do not join the RCCL
communicator (RCCL allows one rank per GPU and a PS shares a worker's GPU,
SURVEY §7.3 H1(a)); they attach to the same store as coordinators.
"""
from __future__ import annotations

import argparse
import json
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple


@dataclass
class ClusterSpec:
    workers: List[str] = field(default_factory=list)
    ps: List[str] = field(default_factory=list)
    job_name: str = "local"
    task_index: int = 0
    host_map: Dict[str, str] = field(default_factory=dict)

    @property
    def is_local(self) -> bool:
        return self.job_name == "local" or not self.workers

    @property
    def is_ps(self) -> bool:
        return self.job_name == "ps"

    @property
    def is_chief(self) -> bool:
        return self.job_name in ("local", "worker") and self.task_index == 0

    @property
    def num_workers(self) -> int:
        return max(1, len(self.workers))

    def resolve(self, hostport: str) -> Tuple[str, int]:
        """``<service>:2222`` -> (ip, port) through KFA_SERVICE_HOSTS (identity if unknown)."""
        hp = self.host_map.get(hostport, hostport)
        host, _, port = hp.rpartition(":")
        return host or "127.0.0.1", int(port)

    def rendezvous(self) -> Tuple[str, int]:
        """Chief endpoint = TCPStore / MASTER_ADDR:MASTER_PORT for the worker collective."""
        if not self.workers:
            return "127.0.0.1", 29500
        return self.resolve(self.workers[0])

    def torch_env(self) -> Dict[str, str]:
        """RANK / WORLD_SIZE / MASTER_* / LOCAL_RANK for ``init_process_group`` (workers only)."""
        host, port = self.rendezvous()
        rank = 0 if self.is_local else self.task_index
        return {"RANK": str(rank), "WORLD_SIZE": str(1 if self.is_local else self.num_workers),
                "LOCAL_RANK": str(local_device()), "MASTER_ADDR": host, "MASTER_PORT": str(port)}


def local_device(environ=None) -> int:
    """This replica's own GPU as a device ordinal of this process: 0 when the
    supervisor isolates it (``HIP_VISIBLE_DEVICES=<own>[,PS GPUs]``), its physical
    index when every node GPU is visible (``gpu_binding="visible"``:
    ``KFA_LOCAL_DEVICE``)."""
    env = os.environ if environ is None else environ
    try:
        return max(0, int(env.get("KFA_LOCAL_DEVICE", "0") or 0))
    except ValueError:
        return 0


def add_cluster_flags(ap: argparse.ArgumentParser) -> None:
    """The reference workload's cluster flags (``mnist_replica.py:55-85``)."""
    ap.add_argument("--worker_hosts", default="", help="comma-separated host:port list of workers")
    ap.add_argument("--ps_hosts", default="", help="comma-separated host:port list of parameter servers")
    ap.add_argument("--job_name", default="", help="worker | ps (empty: TF_CONFIG or local)")
    ap.add_argument("--task_index", type=int, default=None)


def parse_cluster(args: Optional[argparse.Namespace] = None, environ=None) -> ClusterSpec:
    env = os.environ if environ is None else environ
    spec = ClusterSpec()
    try:
        spec.host_map = json.loads(env.get("KFA_SERVICE_HOSTS", "") or "{}")
    except ValueError:
        spec.host_map = {}
    tfc = {}
    if env.get("TF_CONFIG"):
        try:
            tfc = json.loads(env["TF_CONFIG"])
        except ValueError:
            tfc = {}
    cl = tfc.get("cluster", {})
    task = tfc.get("task", {})
    spec.workers = list(cl.get("worker", []))
    spec.ps = list(cl.get("ps", []))
    spec.job_name = task.get("type", "") or ""
    spec.task_index = int(task.get("index", 0) or 0)
    if args is not None:  # flags win over TF_CONFIG (the reference passes flags)
        if getattr(args, "worker_hosts", ""):
            spec.workers = [h for h in args.worker_hosts.split(",") if h]
        if getattr(args, "ps_hosts", ""):
            spec.ps = [h for h in args.ps_hosts.split(",") if h]
        if getattr(args, "job_name", ""):
            spec.job_name = args.job_name
        if getattr(args, "task_index", None) is not None:
            spec.task_index = args.task_index
    if not spec.job_name:
        spec.job_name = "worker" if spec.workers else "local"
    return spec
