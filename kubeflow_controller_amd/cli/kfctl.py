"""``kfctl`` — the kubectl-equivalent client, plus the node daemons.

Subcommands (the user flow of ``docs/get_started.md``: create the CRD, run the
controller, ``envsubst < tfjob.yml | kubectl create -f -``, read pod logs):

  kfctl apiserver  [--listen H:P] [--data-dir D]     run the object store's REST apiserver
  kfctl kubelet    --master URL [--num-gpus N]       run the replica supervisor + endpoint controller
  kfctl up         [--listen H:P] ...                 apiserver + controller + kubelet in one process
  kfctl create -f FILE|-  [--no-envsubst]            create objects (TFJob / Pod / Service / CRD)
  kfctl get RESOURCE [NAME] [-n NS] [-l SEL] [-o wide|yaml|json]
  kfctl describe tfjob NAME                          spec summary, status, replicas, events
  kfctl delete RESOURCE NAME [--cascade=orphan]
  kfctl logs POD [--root-dir D]                      replica process output
  kfctl wait tfjob NAME [--for Succeeded] [--timeout S]

The server is taken from ``--master``, ``--kubeconfig`` or ``KUBEFLOW_MASTER``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from typing import List, Optional

from ..api import serde, v1alpha1
from ..api.labels import Selector


def _store(args):
    from ..store import connect
    st = connect(getattr(args, "master", ""), getattr(args, "kubeconfig", ""))
    if st is None:
        raise SystemExit("no apiserver: pass --master URL (or --kubeconfig, or set KUBEFLOW_MASTER)")
    return st


def _kind(resource: str) -> str:
    k = serde.RESOURCES.get(resource.lower())
    if k is None:
        raise SystemExit(f'error: the server doesn\'t have a resource type "{resource}"')
    return k


def _age(ts: Optional[str]) -> str:
    if not ts:
        return "<unknown>"
    import datetime as dt
    t = dt.datetime.strptime(ts, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=dt.timezone.utc)
    s = int((dt.datetime.now(dt.timezone.utc) - t).total_seconds())
    return f"{s}s" if s < 120 else (f"{s // 60}m" if s < 7200 else f"{s // 3600}h")


def _row(obj, wide: bool) -> List[str]:
    m = obj.metadata
    if obj.kind == v1alpha1.TFJOB_KIND:
        reps = ",".join(f"{s.tfReplicaType}:{s.replicas}" for s in obj.spec.specs)
        states = ";".join(f"{st.type}:" + ",".join(f"{k}={v}" for k, v in sorted(st.tfReplicasStates.items()))
                          for st in (obj.status.tfReplicaStatuses or []))
        r = [m.name, obj.status.phase or "-", reps, _age(m.creationTimestamp)]
        return r + [obj.spec.runtimeID or "-", states or "-"] if wide else r
    if obj.kind == "Pod":
        cs = obj.status.containerStatuses[0] if obj.status.containerStatuses else None
        r = [m.name, obj.status.phase, str(cs.restartCount if cs else 0), _age(m.creationTimestamp)]
        return r + [",".join(map(str, obj.status.gpus)) or "-", str(cs.pid if cs else "-")] if wide else r
    if obj.kind == "Service":
        ports = ",".join(f"{p.port}:{p.nodePort}" for p in obj.spec.ports)
        return [m.name, obj.spec.clusterIP or "<pending>", ports, _age(m.creationTimestamp)]
    if obj.kind == "Event":
        return [_age(obj.lastTimestamp), obj.type, obj.reason, f"{obj.involvedObject.kind.lower()}/"
                f"{obj.involvedObject.name}", obj.message]
    return [m.name]


_HEAD = {
    v1alpha1.TFJOB_KIND: (["NAME", "PHASE", "REPLICAS", "AGE"], ["RUNTIME-ID", "REPLICA-STATES"]),
    "Pod": (["NAME", "STATUS", "RESTARTS", "AGE"], ["GPUS", "PID"]),
    "Service": (["NAME", "CLUSTER-IP", "PORT(S)", "AGE"], []),
    "Event": (["LAST SEEN", "TYPE", "REASON", "OBJECT", "MESSAGE"], []),
}


def _table(rows: List[List[str]]) -> str:
    if not rows:
        return ""
    w = [max(len(r[i]) for r in rows) for i in range(len(rows[0]))]
    return "\n".join("   ".join(c.ljust(w[i]) for i, c in enumerate(r)).rstrip() for r in rows)


def cmd_get(args) -> int:
    st = _store(args)
    kind = _kind(args.resource)
    ns = None if args.all_namespaces else args.namespace
    if args.name:
        objs = [st.get(kind, ns or "default", args.name)]
    else:
        objs = st.list(kind, ns, Selector.parse(args.selector))
    if args.output in ("yaml", "json"):
        data = [o.to_json() for o in objs]
        payload = data[0] if args.name else {"apiVersion": "v1", "kind": "List", "items": data}
        print(json.dumps(payload, indent=2) if args.output == "json" else serde.dump_yaml(payload), end="")
        return 0
    if not objs:
        print(f"No resources found in {ns or 'any'} namespace.", file=sys.stderr)
        return 0
    head, extra = _HEAD.get(kind, (["NAME"], []))
    wide = args.output == "wide"
    print(_table([head + (extra if wide else [])] + [_row(o, wide) for o in objs]))
    return 0


def cmd_create(args) -> int:
    st = _store(args)
    text = sys.stdin.read() if args.filename == "-" else open(args.filename).read()
    objs = serde.load_objects(text, substitute=not args.no_envsubst)
    for o in objs:
        if isinstance(o, dict):
            st.create(o)
            print(f"customresourcedefinition \"{o['metadata']['name']}\" created")
            continue
        created = st.create(o, namespace=args.namespace if args.namespace != "default" else None)
        print(f"{created.kind.lower()} \"{created.metadata.name}\" created")
    return 0


def cmd_delete(args) -> int:
    st = _store(args)
    kind = _kind(args.resource)
    prop = "Orphan" if args.cascade == "orphan" else "Background"
    st.delete(kind, args.namespace, args.name, propagation=prop)
    print(f"{kind.lower()} \"{args.name}\" deleted")
    return 0


def describe_tfjob(st, ns: str, name: str) -> str:
    job = st.get(v1alpha1.TFJOB_KIND, ns, name)
    out = [f"Name:         {job.metadata.name}", f"Namespace:    {job.metadata.namespace}",
           f"UID:          {job.metadata.uid}", f"API Version:  {job.apiVersion}", f"Kind:         {job.kind}",
           f"Runtime ID:   {job.spec.runtimeID or '<none>'}", "Spec:"]
    for s in job.spec.specs:
        c0 = s.template.spec.containers[0] if s.template and s.template.spec.containers else None
        out.append(f"  {s.tfReplicaType}: replicas={s.replicas} restartPolicy="
                   f"{(s.template.spec.restartPolicy if s.template else '') or 'Always'}"
                   f" command={' '.join((c0.command if c0 else []))}")
    out.append("Status:")
    out.append(f"  Phase:  {job.status.phase or '<none>'}")
    for rs in job.status.tfReplicaStatuses or []:
        out.append(f"  {rs.type}: " + ", ".join(f"{k}={v}" for k, v in sorted(rs.tfReplicasStates.items())))
    pods = [p for p in st.list("Pod", ns) if p.metadata.labels.get("tf_job_name") == name]
    if pods:
        out.append("Replicas:")
        for p in pods:
            cs = p.status.containerStatuses[0] if p.status.containerStatuses else None
            out.append(f"  {p.metadata.name:<32} {p.metadata.labels.get('job_type', ''):<7} "
                       f"index={p.metadata.labels.get('index', '0'):<3} {p.status.phase:<10} "
                       f"gpus={','.join(map(str, p.status.gpus)) or '-'} restarts={cs.restartCount if cs else 0}")
    evs = [e for e in st.list("Event", ns) if e.involvedObject.uid == job.metadata.uid]
    evs.sort(key=lambda e: e.firstTimestamp or "")
    out.append("Events:")
    if not evs:
        out.append("  <none>")
    for e in evs:
        out.append(f"  {e.type:<8} {e.reason:<18} {e.source.component:<20} {e.message}"
                   + (f" (x{e.count})" if e.count > 1 else ""))
    return "\n".join(out)


def cmd_describe(args) -> int:
    st = _store(args)
    if _kind(args.resource) != v1alpha1.TFJOB_KIND:
        print(serde.dump_yaml(st.get(_kind(args.resource), args.namespace, args.name)), end="")
        return 0
    print(describe_tfjob(st, args.namespace, args.name))
    return 0


def cmd_logs(args) -> int:
    d = os.path.join(os.path.expanduser(args.root_dir), f"{args.namespace}_{args.pod}")
    if not os.path.isdir(d):
        raise SystemExit(f"no logs for pod {args.pod} under {args.root_dir}")
    for f in sorted(os.listdir(d)):
        if f.endswith(".log"):
            with open(os.path.join(d, f)) as fh:
                sys.stdout.write(fh.read())
    return 0


def wait_for_phase(st, ns: str, name: str, phases, timeout: float, poll: float = 0.2):
    deadline = time.monotonic() + timeout
    while True:
        job = st.get(v1alpha1.TFJOB_KIND, ns, name)
        if job.status.phase in phases:
            return job
        if time.monotonic() > deadline:
            raise TimeoutError(f"tfjob {name}: phase {job.status.phase!r} after {timeout}s")
        time.sleep(poll)


def cmd_wait(args) -> int:
    st = _store(args)
    job = wait_for_phase(st, args.namespace, args.name, set(args.phase.split(",")), args.timeout)
    print(f"tfjob \"{args.name}\" phase {job.status.phase}")
    return 0 if job.status.phase != v1alpha1.PHASE_FAILED else 1


def cmd_apiserver(args) -> int:
    from ..store import ObjectStore
    from ..store.apiserver import APIServer
    from .signals import setup_signal_handler
    stop = setup_signal_handler()
    host, _, port = args.listen.rpartition(":")
    srv = APIServer(ObjectStore(args.data_dir or None), host or "127.0.0.1", int(port or 0)).start()
    print(srv.url, flush=True)
    if args.url_file:
        with open(args.url_file, "w") as f:
            f.write(srv.url + "\n")
    stop.wait()
    srv.stop()
    return 0


def cmd_kubelet(args) -> int:
    from ..client.clientset import Clientset
    from ..client.informer import SharedInformerFactory
    from ..kubelet import EndpointController, Supervisor
    from .signals import setup_signal_handler
    stop = setup_signal_handler()
    st = _store(args)
    inf = SharedInformerFactory(st, 30.0)
    cs = Clientset(st)
    EndpointController(cs, inf.services())
    sup = Supervisor(cs, inf.pods(), inf.services(), args.root_dir, num_gpus=args.num_gpus,
                     gpu_policy=args.gpu_policy, tfjob_informer=inf.tfjobs(),
                     gpu_binding=getattr(args, "gpu_binding", None))
    inf.start(stop)
    sup.run(stop)
    return 0


def cmd_up(args) -> int:
    from .controller_main import main as controller_main
    argv = ["--standalone", "--listen", args.listen, "--root-dir", args.root_dir, "-v", str(args.v)]
    if args.data_dir:
        argv += ["--data-dir", args.data_dir]
    if args.num_gpus is not None:
        argv += ["--num-gpus", str(args.num_gpus)]
    if args.url_file:
        argv += ["--url-file", args.url_file]
    return controller_main(argv)


def cmd_kill(args) -> int:
    """Fault injection: signal a running replica's process group
    (pid from the pod's container status), as a crashed container would be; the
    kubelet then applies the pod's restartPolicy."""
    import signal as _signal
    st = _store(args)
    pod = st.get("Pod", args.namespace, args.pod)
    cs = pod.status.containerStatuses[0] if pod.status.containerStatuses else None
    if not cs or not cs.pid or pod.status.phase != "Running":
        raise ValueError(f"pod {args.pod} has no running replica process")
    sig = getattr(_signal, args.signal if args.signal.startswith("SIG") else "SIG" + args.signal)
    os.killpg(cs.pid, sig)
    print(f"pod \"{args.pod}\" pid {cs.pid} sent {sig.name}")
    return 0


def cmd_metrics(args) -> int:
    """Print the controller's Prometheus metrics (GET /metrics on the apiserver)."""
    import urllib.request
    if not args.master:
        raise ValueError("kfctl metrics needs --master (the standalone apiserver URL)")
    with urllib.request.urlopen(args.master.rstrip("/") + "/metrics", timeout=10) as r:
        sys.stdout.write(r.read().decode())
    return 0


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="kfctl", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--master", "-s", default="")
    ap.add_argument("--kubeconfig", default="")
    sub = ap.add_subparsers(dest="cmd", required=True)

    def ns(p):
        p.add_argument("-n", "--namespace", default="default")

    p = sub.add_parser("get"); ns(p)
    p.add_argument("resource"); p.add_argument("name", nargs="?")
    p.add_argument("-l", "--selector", default="")
    p.add_argument("-o", "--output", default="", choices=["", "wide", "yaml", "json"])
    p.add_argument("-A", "--all-namespaces", action="store_true")
    p.set_defaults(fn=cmd_get)
    p = sub.add_parser("create"); ns(p)
    p.add_argument("-f", "--filename", required=True)
    p.add_argument("--no-envsubst", action="store_true")
    p.set_defaults(fn=cmd_create)
    p = sub.add_parser("delete"); ns(p)
    p.add_argument("resource"); p.add_argument("name")
    p.add_argument("--cascade", default="background", choices=["background", "orphan"])
    p.set_defaults(fn=cmd_delete)
    p = sub.add_parser("describe"); ns(p)
    p.add_argument("resource"); p.add_argument("name")
    p.set_defaults(fn=cmd_describe)
    p = sub.add_parser("logs"); ns(p)
    p.add_argument("pod"); p.add_argument("--root-dir", default="~/.kfa/pods")
    p.set_defaults(fn=cmd_logs)
    p = sub.add_parser("wait"); ns(p)
    p.add_argument("resource", choices=["tfjob", "tfjobs"]); p.add_argument("name")
    p.add_argument("--for", dest="phase", default="Succeeded,Failed")
    p.add_argument("--timeout", type=float, default=600.0)
    p.set_defaults(fn=cmd_wait)
    p = sub.add_parser("kill"); ns(p)
    p.add_argument("pod"); p.add_argument("--signal", default="SIGKILL")
    p.set_defaults(fn=cmd_kill)
    p = sub.add_parser("metrics")
    p.set_defaults(fn=cmd_metrics)
    p = sub.add_parser("apiserver")
    p.add_argument("--listen", default="127.0.0.1:8443"); p.add_argument("--data-dir", default="")
    p.add_argument("--url-file", default="")
    p.set_defaults(fn=cmd_apiserver)
    p = sub.add_parser("kubelet")
    p.add_argument("--root-dir", default=os.path.expanduser("~/.kfa/pods"))
    p.add_argument("--num-gpus", type=int, default=None)
    p.add_argument("--gpu-policy", default="auto", choices=["auto", "none", "share"])
    p.add_argument("--gpu-binding", default=None, choices=["isolate", "visible"])
    p.set_defaults(fn=cmd_kubelet)
    p = sub.add_parser("up")
    p.add_argument("--listen", default="127.0.0.1:8443"); p.add_argument("--data-dir", default="")
    p.add_argument("--root-dir", default=os.path.expanduser("~/.kfa/pods"))
    p.add_argument("--num-gpus", type=int, default=None); p.add_argument("-v", type=int, default=0)
    p.add_argument("--url-file", default="")
    p.set_defaults(fn=cmd_up)
    return ap


def main(argv: Optional[List[str]] = None) -> int:
    args = build_parser().parse_args(argv)
    try:
        return args.fn(args)
    except Exception as e:  # kubectl-style one-line errors
        from ..store import errors
        if isinstance(e, (errors.StatusError, TimeoutError, ValueError)):
            print(f"Error from server ({type(e).__name__}): {e}", file=sys.stderr)
            return 1
        raise


if __name__ == "__main__":
    sys.exit(main())
