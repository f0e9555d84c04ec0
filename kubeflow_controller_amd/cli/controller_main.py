"""``kubeflow-controller`` — the controller binary (reference ``cmd/controller/main.go``).

Same flags as the reference: ``-kubeconfig``, ``-master``, ``-version`` plus
the glog flags (``-v``, ``-logtostderr``, ``-alsologtostderr``,
``-stderrthreshold``, ``-vmodule``, ``-log_backtrace_at``, ``-log_dir``).
``-master`` / ``-kubeconfig`` point at a ``kfctl apiserver`` (the local object
store's REST endpoint).  With neither set (and no ``KUBEFLOW_MASTER`` env, the
"in-cluster" fallback) the controller runs ``--standalone``: object store +
REST apiserver + controller + kubelet (replica supervisor) in one process.

Hard-coded tunables of the reference are kept as defaults and exposed as
flags: threadiness 2, informer resync 30 s, expectations TTL 5 min.
"""
from __future__ import annotations

import argparse
import logging
import os
import sys
import threading
from typing import List, Optional

from .. import version
from .signals import setup_signal_handler

log = logging.getLogger("kfa.main")


def add_glog_flags(ap: argparse.ArgumentParser) -> None:
    ap.add_argument("-v", "--v", type=int, default=0, dest="verbosity", help="log level for V logs")
    ap.add_argument("-logtostderr", "--logtostderr", action="store_true", help="log to standard error")
    ap.add_argument("-alsologtostderr", "--alsologtostderr", action="store_true")
    ap.add_argument("-stderrthreshold", "--stderrthreshold", default="ERROR")
    ap.add_argument("-vmodule", "--vmodule", default="")
    ap.add_argument("-log_backtrace_at", "--log_backtrace_at", default="")
    ap.add_argument("-log_dir", "--log_dir", default="")


def setup_logging(args) -> None:
    level = logging.DEBUG if args.verbosity >= 4 else (logging.INFO if args.verbosity >= 0 else logging.WARNING)
    handlers: List[logging.Handler] = []
    if args.log_dir:
        os.makedirs(args.log_dir, exist_ok=True)
        handlers.append(logging.FileHandler(os.path.join(args.log_dir, "kubeflow-controller.log")))
    if args.logtostderr or args.alsologtostderr or not args.log_dir:
        h = logging.StreamHandler(sys.stderr)
        if not (args.logtostderr or args.alsologtostderr) and args.log_dir:
            h.setLevel(getattr(logging, args.stderrthreshold.upper(), logging.ERROR))
        handlers.append(h)
    logging.basicConfig(level=level, handlers=handlers, force=True,
                        format="%(levelname).1s%(asctime)s %(threadName)s %(name)s] %(message)s")


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="kubeflow-controller", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-kubeconfig", "--kubeconfig", default="", help="Path to a kubeconfig (apiserver URL)")
    ap.add_argument("-master", "--master", default="", help="The address of the apiserver (overrides kubeconfig)")
    ap.add_argument("-version", "--version", action="store_true", help="Show version and exit")
    add_glog_flags(ap)
    ap.add_argument("--standalone", action="store_true",
                    help="run object store + apiserver + kubelet in-process (default when no master is given)")
    ap.add_argument("--listen", default="127.0.0.1:0", help="standalone apiserver address")
    ap.add_argument("--data-dir", default="", help="standalone store persistence directory")
    ap.add_argument("--kubelet", choices=["auto", "on", "off"], default="auto",
                    help="run the replica supervisor in this process (auto: on in standalone mode)")
    ap.add_argument("--root-dir", default=os.path.expanduser("~/.kfa/pods"), help="replica working/log dirs")
    ap.add_argument("--num-gpus", type=int, default=None, help="GPUs on this node (default: detect)")
    ap.add_argument("--gpu-policy", choices=["auto", "none", "share"], default="auto")
    ap.add_argument("--gpu-binding", choices=["isolate", "visible"], default=None,
                    help="isolate: HIP_VISIBLE_DEVICES=<the replica's GPU> (default, or KFA_GPU_BINDING); "
                         "visible: every node GPU visible, the replica's ordinal in KFA_LOCAL_DEVICE / LOCAL_RANK")
    ap.add_argument("--threadiness", type=int, default=2)
    ap.add_argument("--resync", type=float, default=30.0)
    ap.add_argument("--url-file", default="", help="write the standalone apiserver URL to this file")
    return ap


class Node:
    """Everything one `kubeflow-controller` process runs (handy for tests)."""

    def __init__(self, store, *, threadiness: int = 2, resync: float = 30.0, kubelet: bool = True,
                 root_dir: str = "", num_gpus: Optional[int] = None, gpu_policy: str = "auto",
                 kubelet_backoff: float = 1.0, extra_env=None, gpu_binding: Optional[str] = None):
        from ..client.clientset import Clientset
        from ..client.informer import SharedInformerFactory
        from ..controller.controller import Controller

        self.store = store
        self.threadiness = threadiness
        self.kube_client = Clientset(store)
        self.tfjob_client = Clientset(store)
        self.kube_informers = SharedInformerFactory(store, resync)
        self.tfjob_informers = SharedInformerFactory(store, resync)
        self.controller = Controller(self.kube_client, self.tfjob_client, self.kube_informers, self.tfjob_informers)
        self.supervisor = None
        self.endpoints = None
        if kubelet:
            from ..kubelet import EndpointController, Supervisor
            kinf = SharedInformerFactory(store, resync)
            self.kubelet_informers = kinf
            self.endpoints = EndpointController(self.kube_client, kinf.services())
            self.supervisor = Supervisor(self.kube_client, kinf.pods(), kinf.services(),
                                         root_dir or os.path.expanduser("~/.kfa/pods"), num_gpus=num_gpus,
                                         gpu_policy=gpu_policy, backoff_base=kubelet_backoff, extra_env=extra_env,
                                         tfjob_informer=kinf.tfjobs(), gpu_binding=gpu_binding)
        self.stop = threading.Event()
        self._threads: List[threading.Thread] = []

    def start(self) -> "Node":
        self.kube_informers.start(self.stop)
        self.tfjob_informers.start(self.stop)
        if self.supervisor is not None:
            self.kubelet_informers.start(self.stop)
            t = threading.Thread(target=self.supervisor.run, args=(self.stop,), name="kubelet", daemon=True)
            t.start()
            self._threads.append(t)
        t = threading.Thread(target=self.controller.run, args=(self.threadiness, self.stop), name="controller",
                             daemon=True)
        t.start()
        self._threads.append(t)
        return self

    def shutdown(self, timeout: float = 15.0) -> None:
        self.stop.set()
        for t in self._threads:
            t.join(timeout)
        if self.controller.broadcaster is not None:
            self.controller.broadcaster.shutdown()


def main(argv: Optional[List[str]] = None) -> int:
    args = build_parser().parse_args(argv)
    setup_logging(args)
    vi = version.version_info()
    log.info("Run kubeflow-controller version %s, git SHA %s, python %s, %s", vi["version"], vi["gitSHA"],
             vi["python"], vi["platform"])
    if args.version:
        print(f"kubeflow-controller {vi['version']} (git {vi['gitSHA']}, python {vi['python']}, {vi['platform']})")
        return 0
    from ..store import ObjectStore, connect
    from ..store.apiserver import APIServer

    stop = setup_signal_handler()
    store = None if args.standalone else connect(args.master, args.kubeconfig)
    server = None
    standalone = store is None
    if standalone:
        store = ObjectStore(args.data_dir or None)
        host, _, port = args.listen.rpartition(":")
        server = APIServer(store, host or "127.0.0.1", int(port or 0)).start()
        log.info("standalone apiserver listening on %s", server.url)
        if args.url_file:
            with open(args.url_file, "w") as f:
                f.write(server.url + "\n")
    run_kubelet = args.kubelet == "on" or (args.kubelet == "auto" and standalone)
    node = Node(store, threadiness=args.threadiness, resync=args.resync, kubelet=run_kubelet,
                root_dir=args.root_dir, num_gpus=args.num_gpus, gpu_policy=args.gpu_policy,
                gpu_binding=args.gpu_binding)
    node.start()
    stop.wait()
    log.info("shutting down")
    node.shutdown()
    if server is not None:
        server.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
