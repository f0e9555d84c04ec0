"""Object store (apiserver/etcd/GC replacement): in-process, REST server and REST client."""
from . import errors
from .memory import ADDED, DELETED, MODIFIED, ObjectStore, Watch, merge_patch
from .rest import RESTStore


def connect(master: str = "", kubeconfig: str = ""):
    """``clientcmd.BuildConfigFromFlags`` equivalent (``VCG/tools/clientcmd/client_config.go:527-539``).

    ``master`` wins; else ``kubeconfig`` (a YAML/JSON file with ``server:`` or
    ``clusters[0].cluster.server``); else the ``KUBEFLOW_MASTER`` env var (the
    "in-cluster" fallback); else ``None`` meaning "run an in-process store".
    """
    import os
    import yaml
    if master:
        return RESTStore(master)
    if kubeconfig:
        with open(kubeconfig) as f:
            cfg = yaml.safe_load(f) or {}
        server = cfg.get("server")
        if not server and cfg.get("clusters"):
            server = cfg["clusters"][0].get("cluster", {}).get("server")
        if not server:
            raise ValueError(f"{kubeconfig}: no server URL found")
        return RESTStore(server)
    env = os.environ.get("KUBEFLOW_MASTER")
    if env:
        return RESTStore(env)
    return None
