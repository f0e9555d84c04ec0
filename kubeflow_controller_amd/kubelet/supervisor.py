"""Replica process supervisor — the kubelet of a single 8x MI355X node.

SURVEY §1.2 / §5.3: a Pod is ONE local process.  The supervisor watches Pods
and for each new one:

1. binds GPUs: ``resources.limits["amd.com/gpu"]`` if the template asks, else
   the node policy (``gpu_policy="auto"``: every Worker / Local replica gets one
   GPU, round-robin over the free ones; PS replicas get none — parameter
   shards are owned by worker ranks); pins them with
   ``HIP_VISIBLE_DEVICES`` (``gpu_binding="isolate"``, the default) or — with
   ``gpu_binding="visible"`` — keeps every node GPU visible and names the
   replica's own ordinal in ``KFA_LOCAL_DEVICE`` / ``LOCAL_RANK`` (the
   reference picks its device out of a fully visible set,
   ``examples/workdir/mnist_replica.py:125-129``; the same device set as
   ``bench.py`` under torchrun, so RCCL sees the same peers and transports);
2. resolves the cluster spec: ``<svc>:2222`` endpoints in the args are served
   by the endpoint controller, the resolution map is exported as
   ``KFA_SERVICE_HOSTS`` (the kube-dns role) — the replica keeps the
   reference's exact ``--worker_hosts/--ps_hosts`` strings;
3. emulates ``hostPath`` volume mounts by rewriting ``mountPath`` prefixes in
   the command / args / workingDir to the host path (the samples run
   ``python /workdir/mnist_replica.py`` with ``/workdir`` a hostPath);
4. spawns the process in its own session through the native launcher
   (``posix_spawn``; logs to ``<root>/<ns>_<pod>/<container>.log``);
5. reaps it: exit 0 -> ``Succeeded``, != 0 -> ``Failed``, applying
   ``restartPolicy`` (``Always`` / ``OnFailure`` restart in place with
   exponential back-off and bump ``restartCount``; ``Never`` does not);
6. on Pod deletion (incl. the owner TFJob's cascade) kills the process group
   (SIGTERM, SIGKILL after the grace period) and frees its GPUs.
"""
from __future__ import annotations

import json
import logging
import os
import re
import signal
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..utils import metrics
from ..api import v1alpha1
from ..api.core import (GPU_RESOURCE, POD_FAILED, POD_PENDING, POD_RUNNING, POD_SUCCEEDED, RESTART_ALWAYS,
                        RESTART_NEVER, RESTART_ON_FAILURE, ContainerStateTerminated, ContainerStatus, Pod,
                        gpu_request)
from ..api.meta import now_rfc3339
from ..native import load as _native
from ..store import errors
from .endpoints import service_host_map

log = logging.getLogger("kfa.kubelet")

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_HOSTPORT_RE = re.compile(r"([A-Za-z0-9][-A-Za-z0-9.]*):(\d+)")


def detect_gpus() -> int:
    """Number of GPUs on the node WITHOUT initialising HIP in this process."""
    env = os.environ.get("KFA_NODE_GPUS")
    if env is not None:
        return int(env)
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        return len([v for v in vis.split(",") if v.strip()])
    try:
        return len([d for d in os.listdir("/sys/class/kfd/kfd/topology/nodes")
                    if _is_gpu_node(os.path.join("/sys/class/kfd/kfd/topology/nodes", d))])
    except OSError:
        return 0


def _is_gpu_node(path: str) -> bool:
    try:
        with open(os.path.join(path, "properties")) as f:
            for line in f:
                if line.startswith("simd_count"):
                    return int(line.split()[1]) > 0
    except OSError:
        pass
    return False


@dataclass
class _Proc:
    key: str
    pid: int = 0
    gpus: List[int] = field(default_factory=list)
    restarts: int = 0
    started: float = 0.0
    next_start: float = 0.0
    state: str = "starting"  # starting | running | backoff | done
    log_path: str = ""
    term_sent: float = 0.0
    recycled: bool = False  # terminated because its job finished (PS recycling)


class Supervisor:
    def __init__(self, clientset, pod_informer, service_informer, root_dir: str, *, num_gpus: Optional[int] = None,
                 gpu_policy: str = "auto", backoff_base: float = 1.0, backoff_max: float = 60.0,
                 grace_period: float = 10.0, extra_env: Optional[Dict[str, str]] = None, tfjob_informer=None,
                 gpu_binding: Optional[str] = None):
        self.client = clientset
        self.pods = pod_informer.lister()
        self.services = service_informer.lister()
        self.tfjobs = tfjob_informer.lister() if tfjob_informer is not None else None
        self.root = os.path.abspath(root_dir)
        os.makedirs(self.root, exist_ok=True)
        self.num_gpus = detect_gpus() if num_gpus is None else num_gpus
        self.gpu_policy = gpu_policy
        self.gpu_binding = (gpu_binding or os.environ.get("KFA_GPU_BINDING", "isolate")).lower()
        if self.gpu_binding not in ("isolate", "visible"):
            raise ValueError(f"gpu_binding {self.gpu_binding!r}: isolate | visible")
        self.backoff_base = backoff_base
        self.backoff_max = backoff_max
        self.grace = grace_period
        self.extra_env = dict(extra_env or {})
        self.rt = _native()
        self._procs: Dict[str, _Proc] = {}
        self._gpu_owner: Dict[int, str] = {}
        self._lock = threading.RLock()
        self._rr = 0
        pod_informer.add_event_handler(on_add=self._on_pod, on_update=lambda o, n: self._on_pod(n),
                                       on_delete=self._on_pod_delete)

    # ------------------------------------------------------------------ events
    @staticmethod
    def _key(pod: Pod) -> str:
        return f"{pod.metadata.namespace}/{pod.metadata.name}"

    def _on_pod(self, pod: Pod) -> None:
        key = self._key(pod)
        with self._lock:
            if pod.metadata.deletionTimestamp is not None:
                self._terminate(key)
                return
            if key not in self._procs and pod.status.phase in ("", POD_PENDING):
                self._procs[key] = _Proc(key=key)

    def _on_pod_delete(self, pod: Pod) -> None:
        self._terminate(self._key(pod))

    def _terminate(self, key: str) -> None:
        with self._lock:
            p = self._procs.get(key)
            if p is None:
                return
            if p.state == "running" and p.pid:
                self.rt.kill_group(p.pid, signal.SIGTERM)
                p.term_sent = time.monotonic()
                p.state = "terminating"
            else:
                self._release(p)
                self._procs.pop(key, None)

    # ------------------------------------------------------------------ GPU binding
    def _wants_gpus(self, pod: Pod) -> int:
        c0 = pod.spec.containers[0]
        req = gpu_request(c0)
        if req or (c0.resources and GPU_RESOURCE in (c0.resources.limits or {})):
            return req
        if self.gpu_policy == "none" or self.num_gpus == 0:
            return 0
        typ = pod.metadata.labels.get("job_type", "")
        return 1 if typ in (v1alpha1.WORKER, v1alpha1.LOCAL, "") else 0

    def _colocated_gpu(self, pod: Pod) -> Optional[List[int]]:
        """A PS replica whose template sets ``KFA_PS_COLOCATE=1`` shares GPU
        ``index % num_gpus`` with the worker bound there (not an exclusive
        binding): the device-resident async parameter server keeps its variables
        in that GPU's HBM (``parallel/async_ps.py``)."""
        if pod.metadata.labels.get("job_type", "") != v1alpha1.PS or self.num_gpus == 0:
            return None
        env = {e.name: e.value for e in pod.spec.containers[0].env}
        if env.get("KFA_PS_COLOCATE") != "1":
            return None
        return [int(pod.metadata.labels.get("index", "0")) % self.num_gpus]

    def _colocated_ps_gpus(self, pod: Pod) -> List[int]:
        """Physical GPUs of the job's GPU-co-located PS replicas, by PS index, for a
        Worker pod of a job whose PS template sets ``KFA_PS_COLOCATE=1``; else [].

        The device-resident async PS keeps its variables and the workers' gradient
        mailboxes in its GPU's HBM and every worker reads / writes them by HIP IPC
        peer copies over xGMI (``parallel/async_ps.py``).  A worker must therefore
        SEE those GPUs: they are appended to its ``HIP_VISIBLE_DEVICES`` after its
        own (exclusive) GPU, which stays ordinal 0 for its compute.  The PS count
        and template come from the TFJob spec (or, without a TFJob informer, the
        worker's ``--ps_hosts`` and the job's PS pods)."""
        if pod.metadata.labels.get("job_type", "") != v1alpha1.WORKER or self.num_gpus == 0:
            return []
        name = pod.metadata.labels.get("tf_job_name")
        nps, colocate = 0, False
        job = None
        if self.tfjobs is not None and name:
            try:
                job = self.tfjobs.get(pod.metadata.namespace, name)
            except errors.NotFound:
                job = None
        if job is not None:
            for spec in job.spec.specs:
                if spec.tfReplicaType == v1alpha1.PS:
                    nps = spec.replicas if spec.replicas is not None else 1
                    cs = spec.template.spec.containers if spec.template and spec.template.spec else []
                    colocate = bool(cs) and any(e.name == "KFA_PS_COLOCATE" and e.value == "1" for e in cs[0].env)
        else:
            for a in pod.spec.containers[0].args:
                if a.startswith("--ps_hosts="):
                    nps = len([h for h in a.split("=", 1)[1].split(",") if h])
            colocate = any(p.metadata.labels.get("tf_job_name") == name and p.metadata.labels.get("job_type") == v1alpha1.PS
                           and any(e.name == "KFA_PS_COLOCATE" and e.value == "1" for e in p.spec.containers[0].env)
                           for p in self.pods.list(pod.metadata.namespace))
        if not colocate:
            return []
        return [i % self.num_gpus for i in range(nps)]

    def _bind_gpus(self, key: str, n: int) -> Optional[List[int]]:
        if n == 0:
            return []
        free = [g for g in range(self.num_gpus) if g not in self._gpu_owner]
        if len(free) < n:
            if self.gpu_policy == "share" and self.num_gpus:
                out = [(self._rr + i) % self.num_gpus for i in range(n)]
                self._rr += n
                return out
            return None
        # round-robin start so consecutive jobs spread over the node
        free = sorted(free, key=lambda g: (g - self._rr) % max(self.num_gpus, 1))
        out = free[:n]
        self._rr = (out[-1] + 1) % max(self.num_gpus, 1)
        for g in out:
            self._gpu_owner[g] = key
        return out

    def _release(self, p: _Proc) -> None:
        for g in p.gpus:
            if self._gpu_owner.get(g) == p.key:
                del self._gpu_owner[g]
        p.gpus = []

    # ------------------------------------------------------------------ launch
    @staticmethod
    def _mounts(pod: Pod):
        vols = {v.get("name"): v for v in (pod.spec._get_extra().get("volumes") or [])}
        out = []
        for m in pod.spec.containers[0]._get_extra().get("volumeMounts") or []:
            v = vols.get(m.get("name"), {})
            hp = (v.get("hostPath") or {}).get("path")
            if hp and m.get("mountPath"):
                out.append((m["mountPath"].rstrip("/"), hp.rstrip("/")))
        out.sort(key=lambda x: -len(x[0]))
        return out

    @staticmethod
    def _rewrite(s: str, mounts) -> str:
        for mp, hp in mounts:
            if s == mp or s.startswith(mp + "/"):
                return hp + s[len(mp):]
            s = s.replace("=" + mp + "/", "=" + hp + "/")
        return s

    def _argv_env(self, pod: Pod, gpus: List[int], hosts: Dict[str, str]):
        c = pod.spec.containers[0]
        mounts = self._mounts(pod)
        argv = [self._rewrite(a, mounts) for a in list(c.command) + list(c.args)]
        if not argv:
            raise ValueError("container has neither command nor args")
        if argv[0] in ("python", "python3"):
            argv[0] = sys.executable
        env = dict(os.environ)
        env.update(self.extra_env)
        for e in c.env:
            env[e.name] = e.value
        pp = env.get("PYTHONPATH", "")
        env["PYTHONPATH"] = REPO_ROOT + (os.pathsep + pp if pp else "")
        visible = list(gpus)
        ps_gpus = self._colocated_ps_gpus(pod) if gpus else []
        if ps_gpus:  # the job's PS GPUs after the worker's own: IPC peer copies need them visible
            visible += [g for g in dict.fromkeys(ps_gpus) if g not in visible]
            env["KFA_PS_GPUS"] = ",".join(str(g) for g in ps_gpus)
        env.pop("KFA_LOCAL_DEVICE", None)
        if gpus and self.gpu_binding == "visible":
            # every node GPU visible in physical order; the replica's own GPU by ordinal
            visible = list(range(self.num_gpus))
            env["KFA_LOCAL_DEVICE"] = str(gpus[0])
        env["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in visible) if visible else ""
        env.pop("ROCR_VISIBLE_DEVICES", None)
        env.pop("CUDA_VISIBLE_DEVICES", None)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        env["KFA_SERVICE_HOSTS"] = json.dumps(hosts)
        env["KFA_POD_NAME"] = pod.metadata.name
        env["KFA_POD_NAMESPACE"] = pod.metadata.namespace
        env["KFA_REPLICA_TYPE"] = pod.metadata.labels.get("job_type", "")
        env["KFA_REPLICA_INDEX"] = pod.metadata.labels.get("index", "0")
        env["KFA_TFJOB_NAME"] = pod.metadata.labels.get("tf_job_name", "")
        env["KFA_GPUS"] = ",".join(str(g) for g in visible)  # physical GPU of each local ordinal
        cwd = self._rewrite(c.workingDir, mounts) if c.workingDir else self._pod_dir(pod)
        return argv, env, cwd

    def _pod_dir(self, pod: Pod) -> str:
        d = os.path.join(self.root, f"{pod.metadata.namespace}_{pod.metadata.name}")
        os.makedirs(d, exist_ok=True)
        return d

    def _hosts_ready(self, pod: Pod, hosts: Dict[str, str]) -> bool:
        c = pod.spec.containers[0]
        for a in c.args:
            if a.startswith("--worker_hosts=") or a.startswith("--ps_hosts="):
                for hp in a.split("=", 1)[1].split(","):
                    if hp and hp not in hosts:
                        return False
        return True

    def _start(self, p: _Proc, pod: Pod) -> None:
        hosts = service_host_map(self.services.list(pod.metadata.namespace))
        if not self._hosts_ready(pod, hosts):
            return  # endpoints not allocated yet: stay Pending
        if not p.gpus:
            g = self._colocated_gpu(pod)
            if g is None:
                g = self._bind_gpus(p.key, self._wants_gpus(pod))
            if g is None:
                return  # wait for free GPUs
            p.gpus = g
        try:
            argv, env, cwd = self._argv_env(pod, p.gpus, hosts)
            p.log_path = os.path.join(self._pod_dir(pod), f"{pod.spec.containers[0].name or 'main'}.log")
            p.pid = self.rt.spawn(argv, env, cwd, p.log_path)
        except Exception as e:  # bad command: the container "fails to start"
            log.warning("pod %s failed to start: %s", p.key, e)
            self._set_status(pod, POD_FAILED if pod.spec.restartPolicy == RESTART_NEVER else POD_PENDING,
                             reason="StartError", message=str(e), exit_code=127)
            if pod.spec.restartPolicy == RESTART_NEVER:
                p.state = "done"
                self._release(p)
            else:
                p.state = "backoff"
                p.next_start = time.monotonic() + self._backoff(p)
                p.restarts += 1
            return
        p.started = time.monotonic()
        p.state = "running"
        metrics.REPLICA_STARTS.labels(pod.metadata.labels.get("job_type", "")).inc()
        log.info("started pod %s pid=%d gpus=%s: %s", p.key, p.pid, p.gpus, " ".join(argv))
        self._set_status(pod, POD_RUNNING, pid=p.pid)

    def _backoff(self, p: _Proc) -> float:
        return min(self.backoff_base * (2 ** p.restarts), self.backoff_max)

    # ------------------------------------------------------------------ status
    def _set_status(self, pod: Pod, phase: str, *, pid: int = 0, reason: str = "", message: str = "",
                    exit_code: Optional[int] = None, signal_no: int = 0) -> None:
        key = self._key(pod)
        p = self._procs.get(key)
        for _ in range(5):
            try:
                cur = self.client.core_v1().pods(pod.metadata.namespace).get(pod.metadata.name)
            except errors.NotFound:
                return
            st = cur.status
            st.phase = phase
            st.reason = reason
            st.message = message
            st.hostIP = st.podIP = "127.0.0.1"
            st.startTime = st.startTime or now_rfc3339()
            if p and p.gpus:  # keep the last binding visible after the replica exits
                st.gpus = list(p.gpus)
            cs = st.containerStatuses[0] if st.containerStatuses else ContainerStatus(
                name=cur.spec.containers[0].name or "main")
            cs.restartCount = p.restarts if p else 0
            cs.pid = pid
            cs.ready = phase == POD_RUNNING
            if exit_code is not None:
                term = ContainerStateTerminated(exitCode=exit_code, signal=signal_no, reason=reason or (
                    "Completed" if exit_code == 0 else "Error"), finishedAt=now_rfc3339())
                cs.lastTerminated = term
                cs.terminated = term if phase in (POD_SUCCEEDED, POD_FAILED) else None
            else:
                cs.terminated = None
            st.containerStatuses = [cs]
            try:
                self.client.core_v1().pods(pod.metadata.namespace).update_status(cur)
                return
            except errors.Conflict:
                continue
            except errors.NotFound:
                return

    # ------------------------------------------------------------------ PS recycling
    def _job_finished(self, pod: Pod) -> bool:
        """Owner TFJob already Succeeded/Failed (TFJobRecycling, ``types.go:153-155``)."""
        if self.tfjobs is None:
            return False
        name = pod.metadata.labels.get("tf_job_name")
        if not name:
            return False
        try:
            job = self.tfjobs.get(pod.metadata.namespace, name)
        except errors.NotFound:
            return False
        if job.status.phase in (v1alpha1.PHASE_SUCCEEDED, v1alpha1.PHASE_FAILED):
            return True
        # the controller may not have written the phase yet: look at the workers directly
        want = next((s.replicas for s in job.spec.specs if s.tfReplicaType == v1alpha1.WORKER), None)
        if not want:
            return False
        done = [p for p in self.pods.list(pod.metadata.namespace)
                if p.metadata.labels.get("tf_job_name") == name and p.metadata.labels.get("job_type") == v1alpha1.WORKER
                and p.metadata.labels.get("runtime_id") == pod.metadata.labels.get("runtime_id")
                and p.status.phase == POD_SUCCEEDED]
        return len(done) >= want

    # ------------------------------------------------------------------ main loop
    def tick(self) -> None:
        now = time.monotonic()
        with self._lock:
            items = list(self._procs.items())
        for key, p in items:
            ns, name = key.split("/", 1)
            try:
                pod = self.pods.get(ns, name)
            except errors.NotFound:
                pod = None
            with self._lock:
                if p.state == "terminating":
                    res = self.rt.poll(p.pid)
                    if res is not None:
                        self._release(p)
                        if p.recycled and pod is not None:
                            p.state = "done"
                            self._set_status(pod, POD_SUCCEEDED, exit_code=0, reason="Recycled")
                        else:
                            self._procs.pop(key, None)
                    elif now - p.term_sent > self.grace:
                        self.rt.kill_group(p.pid, signal.SIGKILL)
                    continue
                if pod is None:
                    if p.state == "running":
                        self._terminate(key)
                    else:
                        self._release(p)
                        self._procs.pop(key, None)
                    continue
                if p.state == "backoff" and now >= p.next_start and p.restarts and self._job_finished(pod):
                    # a replica that exited cleanly while its job was finishing is not restarted
                    p.state = "done"
                    self._release(p)
                    self._set_status(pod, POD_SUCCEEDED, exit_code=0, reason="Completed")
                    continue
                if p.state == "starting" or (p.state == "backoff" and now >= p.next_start):
                    self._start(p, pod)
                    continue
                if p.state != "running":
                    continue
                res = self.rt.poll(p.pid)
                finished = pod.metadata.labels.get("job_type") == v1alpha1.PS and self._job_finished(pod)
                if res is None:
                    if finished:  # PS replicas never exit on their own in TF: recycle them
                        log.info("recycling PS pod %s: job finished", key)
                        self.rt.kill_group(p.pid, signal.SIGTERM)
                        p.term_sent = now
                        p.state = "terminating"
                        p.recycled = True
                    continue
                code, sig = res
                metrics.REPLICA_EXITS.labels(pod.metadata.labels.get("job_type", ""),
                                             "success" if code == 0 else "failure").inc()
                policy = pod.spec.restartPolicy or RESTART_ALWAYS
                restart = (policy == RESTART_ALWAYS or (policy == RESTART_ON_FAILURE and code != 0)) and not (
                    finished or (code == 0 and self._job_finished(pod)))
                log.info("pod %s pid=%d exited code=%d (policy %s%s)", key, p.pid, code, policy,
                         ", restarting" if restart else "")
                if restart:
                    p.state = "backoff"
                    p.next_start = now + self._backoff(p)
                    p.restarts += 1
                    self._set_status(pod, POD_RUNNING, reason="CrashLoopBackOff" if code else "Completed",
                                     exit_code=code, signal_no=sig)
                else:
                    p.state = "done"
                    self._release(p)
                    self._set_status(pod, POD_SUCCEEDED if code == 0 else POD_FAILED, exit_code=code,
                                     signal_no=sig, reason="Completed" if code == 0 else "Error")

    def run(self, stop: threading.Event, period: float = 0.05) -> None:
        while not stop.is_set():
            try:
                self.tick()
            except Exception:
                log.exception("supervisor tick failed")
            stop.wait(period)
        self.shutdown()

    def shutdown(self) -> None:
        with self._lock:
            for key, p in list(self._procs.items()):
                if p.state in ("running", "terminating") and p.pid:
                    self.rt.kill_group(p.pid, signal.SIGTERM)
            deadline = time.monotonic() + self.grace
            for key, p in list(self._procs.items()):
                if p.pid:
                    while self.rt.poll(p.pid) is None and time.monotonic() < deadline:
                        time.sleep(0.05)
                    if self.rt.pid_alive(p.pid):
                        self.rt.kill_group(p.pid, signal.SIGKILL)
                        self.rt.poll(p.pid)

    def running(self) -> Dict[str, int]:
        with self._lock:
            return {k: p.pid for k, p in self._procs.items() if p.state == "running"}

    def inject_fault(self, namespace: str, name: str, sig: int = signal.SIGKILL) -> int:
        """Fault injection: signal a running replica's process group,
        as a node/container crash would.  The normal exit path then applies the
        pod's restartPolicy.  Returns the pid signalled (0 if not running)."""
        with self._lock:
            p = self._procs.get(f"{namespace}/{name}")
            if p is None or p.state != "running" or not p.pid:
                return 0
            self.rt.kill_group(p.pid, sig)
            return p.pid

    def gpu_bindings(self) -> Dict[int, str]:
        with self._lock:
            return dict(self._gpu_owner)
