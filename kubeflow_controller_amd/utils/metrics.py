"""Prometheus metrics for the control plane and the replica runtime.

The reference's workqueue metrics provider is a no-op
(``VCG/util/workqueue/metrics.go:128-195``) and it has no Prometheus endpoint;
here the controller, the kubelet supervisor and the REST apiserver publish:

* ``kfa_workqueue_adds_total`` / ``_retries_total`` / ``_depth``
* ``kfa_sync_duration_seconds`` (reconcile latency histogram), ``kfa_sync_errors_total``
* ``kfa_children_created_total{kind,result}`` (Pods / Services, success | failure)
* ``kfa_tfjob_phase_transitions_total{phase}``
* ``kfa_replica_starts_total{type}``, ``kfa_replica_exits_total{type,result}``, ``kfa_replicas_running``

Scraped at ``GET /metrics`` on the apiserver (``kubeflow-controller --standalone``)
or printed by ``kfctl metrics``.  When ``prometheus_client`` is not importable
every metric is a no-op, so nothing in the hot path depends on it.
"""
from __future__ import annotations

try:  # pragma: no cover - import guard
    from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest
    from prometheus_client import CONTENT_TYPE_LATEST
    AVAILABLE = True
except Exception:  # noqa: BLE001
    AVAILABLE = False

REGISTRY = CollectorRegistry(auto_describe=True) if AVAILABLE else None


class _Noop:
    def labels(self, *a, **k):
        return self

    def inc(self, *a, **k):
        pass

    def dec(self, *a, **k):
        pass

    def set(self, *a, **k):
        pass

    def observe(self, *a, **k):
        pass

    def set_function(self, *a, **k):
        pass


def _m(cls, name, doc, labels=(), **kw):
    if not AVAILABLE:
        return _Noop()
    return cls(name, doc, list(labels), registry=REGISTRY, **kw)


if AVAILABLE:
    _C, _G, _H = Counter, Gauge, Histogram
else:  # pragma: no cover
    _C = _G = _H = None

WORKQUEUE_ADDS = _m(_C, "kfa_workqueue_adds_total", "TFJob keys added to the controller workqueue")
WORKQUEUE_RETRIES = _m(_C, "kfa_workqueue_retries_total", "TFJob keys re-queued with rate limiting after an error")
WORKQUEUE_DEPTH = _m(_G, "kfa_workqueue_depth", "keys waiting in the controller workqueue")
SYNC_DURATION = _m(_H, "kfa_sync_duration_seconds", "TFJob reconcile (syncHandler) latency",
                   buckets=(0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5))
SYNC_ERRORS = _m(_C, "kfa_sync_errors_total", "failed TFJob syncs")
CHILDREN_CREATED = _m(_C, "kfa_children_created_total", "Pods / Services created for TFJobs", ("kind", "result"))
PHASE_TRANSITIONS = _m(_C, "kfa_tfjob_phase_transitions_total", "TFJob status.phase transitions", ("phase",))
REPLICA_STARTS = _m(_C, "kfa_replica_starts_total", "replica processes started by the kubelet", ("type",))
REPLICA_EXITS = _m(_C, "kfa_replica_exits_total", "replica process exits", ("type", "result"))
REPLICAS_RUNNING = _m(_G, "kfa_replicas_running", "replica processes currently running")


def exposition() -> bytes:
    """Prometheus text exposition of every kfa_* metric."""
    if not AVAILABLE:
        return b"# prometheus_client not available\n"
    return generate_latest(REGISTRY)


def content_type() -> str:
    return CONTENT_TYPE_LATEST if AVAILABLE else "text/plain; version=0.0.4"
