"""HTTP front end of the object store — a small Kubernetes-style REST API.

This is what ``-master`` / ``-kubeconfig`` point the controller at
(``cmd/controller/main.go:31,59-63``).  Paths follow the k8s layout so the
same URL shapes work:

* ``/apis/kubeflow.caicloud.io/v1alpha1/namespaces/{ns}/tfjobs[/{name}]``
* ``/api/v1/namespaces/{ns}/{pods|services|events}[/{name}]``
* ``/apis/kubeflow.caicloud.io/v1alpha1/tfjobs`` (all namespaces), likewise for core kinds
* ``/apis/apiextensions.k8s.io/v1beta1/customresourcedefinitions`` (CRD registration)
* ``GET ...?watch=true&resourceVersion=N&labelSelector=...`` streams one JSON
  event per line (``{"type": "ADDED", "object": {...}}``), chunked.
* ``PATCH`` takes ``application/merge-patch+json``; ``DELETE`` honours
  ``propagationPolicy`` and a ``preconditions.uid`` body.
"""
from __future__ import annotations

import json
import re
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Optional, Tuple
from urllib.parse import parse_qs, urlparse

from ..api import serde, v1alpha1
from ..api.labels import Selector
from . import errors
from .memory import ObjectStore

_CORE_PLURALS = {"pods": "Pod", "services": "Service", "events": "Event"}
_KF_PLURALS = {v1alpha1.TFJOB_PLURAL: v1alpha1.TFJOB_KIND}
_EXT_PLURALS = {"replicasets": "ReplicaSet"}  # extensions/v1beta1

_PATH_RE = re.compile(
    r"^/(?:api/v1|apis/(?P<group>[^/]+)/(?P<version>[^/]+))"
    r"(?:/namespaces/(?P<ns>[^/]+))?/(?P<plural>[a-z]+)(?:/(?P<name>[^/]+))?(?:/(?P<sub>status))?$")


def _route(path: str) -> Tuple[str, Optional[str], Optional[str], Optional[str]]:
    m = _PATH_RE.match(path)
    if not m:
        raise errors.NotFound(f"no route for {path}")
    plural = m.group("plural")
    group = m.group("group")
    if plural == "customresourcedefinitions":
        return "CRD", None, m.group("name"), None
    if group is None:
        kind = _CORE_PLURALS.get(plural)
    elif group == v1alpha1.GROUP_NAME and m.group("version") == v1alpha1.GROUP_VERSION:
        kind = _KF_PLURALS.get(plural) or _CORE_PLURALS.get(plural)
    elif group == "extensions" and m.group("version") == "v1beta1":
        kind = _EXT_PLURALS.get(plural)
    else:
        kind = None
    if kind is None:
        raise errors.NotFound(f"the server could not find the requested resource ({plural})")
    return kind, m.group("ns"), m.group("name"), m.group("sub")


class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    server: "APIServer"  # type: ignore[assignment]

    def log_message(self, fmt, *args):  # quiet
        pass

    # -------------------------------------------------------------- plumbing
    def _body(self):
        n = int(self.headers.get("Content-Length") or 0)
        if n == 0:
            return None
        return json.loads(self.rfile.read(n))

    def _send(self, code: int, payload) -> None:
        data = json.dumps(payload).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def _err(self, e: errors.StatusError) -> None:
        self._send(e.code, e.to_json())

    def _dispatch(self, verb: str) -> None:
        try:
            u = urlparse(self.path)
            q = {k: v[-1] for k, v in parse_qs(u.query).items()}
            if u.path in ("/healthz", "/readyz"):
                self._send(200, {"status": "ok"})
                return
            if u.path == "/version":
                from ..version import version_info
                self._send(200, version_info())
                return
            if u.path == "/metrics":  # Prometheus scrape (utils/metrics.py)
                from ..utils import metrics
                data = metrics.exposition()
                self.send_response(200)
                self.send_header("Content-Type", metrics.content_type())
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)
                return
            kind, ns, name, sub = _route(u.path)
            getattr(self, "_" + verb)(kind, ns, name, sub, q)
        except errors.StatusError as e:
            self._err(e)
        except (ValueError, TypeError, KeyError) as e:
            self._err(errors.BadRequest(str(e)))
        except (BrokenPipeError, ConnectionResetError):
            pass

    def do_GET(self):
        self._dispatch("get")

    def do_POST(self):
        self._dispatch("post")

    def do_PUT(self):
        self._dispatch("put")

    def do_PATCH(self):
        self._dispatch("patch")

    def do_DELETE(self):
        self._dispatch("delete")

    # -------------------------------------------------------------- verbs
    @property
    def store(self) -> ObjectStore:
        return self.server.store

    def _get(self, kind, ns, name, sub, q):
        if kind == "CRD":
            crds = self.store.crds()
            if name:
                if name not in crds:
                    raise errors.NotFound(f'customresourcedefinition "{name}" not found')
                self._send(200, crds[name])
            else:
                self._send(200, {"kind": "CustomResourceDefinitionList", "items": list(crds.values())})
            return
        sel = Selector.parse(q.get("labelSelector"))
        if q.get("watch") in ("true", "1"):
            self._watch(kind, ns, sel, q.get("resourceVersion"))
            return
        if name:
            self._send(200, self.store.get(kind, ns, name).to_json())
            return
        items, rv = self.store.list_and_rv(kind, ns, sel)
        self._send(200, {"kind": kind + "List", "apiVersion": "v1", "metadata": {"resourceVersion": rv},
                         "items": [o.to_json() for o in items]})

    def _watch(self, kind, ns, sel, rv):
        w = self.store.watch(kind, ns, sel, rv)
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Transfer-Encoding", "chunked")
        self.end_headers()
        try:
            while not self.server.stopping.is_set():
                item = w.next(timeout=1.0)
                if item is None:
                    if w.stopped:
                        break
                    line = json.dumps({"type": "BOOKMARK", "object": {"metadata": {
                        "resourceVersion": self.store.resource_version}}}) + "\n"
                else:
                    etype, obj = item
                    line = json.dumps({"type": etype, "object": obj.to_json()}) + "\n"
                data = line.encode()
                self.wfile.write(b"%x\r\n%s\r\n" % (len(data), data))
                self.wfile.flush()
            self.wfile.write(b"0\r\n\r\n")
        except (BrokenPipeError, ConnectionResetError, OSError):
            pass
        finally:
            w.stop()
            self.close_connection = True

    def _post(self, kind, ns, name, sub, q):
        body = self._body()
        if kind == "CRD":
            self.store.register_crd(body)
            self._send(201, body)
            return
        obj = serde.decode(body)
        if obj.kind != kind:
            raise errors.BadRequest(f"kind {obj.kind} posted to {kind} collection")
        self._send(201, self.store.create(obj, namespace=ns).to_json())

    def _put(self, kind, ns, name, sub, q):
        obj = serde.decode(self._body())
        if ns:
            obj.metadata.namespace = ns
        if name and obj.metadata.name != name:
            raise errors.BadRequest("name in body does not match URL")
        out = self.store.update_status(obj) if sub == "status" else self.store.update(obj)
        self._send(200, out.to_json())

    def _patch(self, kind, ns, name, sub, q):
        body = self._body() or {}
        uid = (body.get("metadata") or {}).get("uid")
        self._send(200, self.store.patch(kind, ns, name, body, expect_uid=uid).to_json())

    def _delete(self, kind, ns, name, sub, q):
        body = self._body() or {}
        prop = body.get("propagationPolicy") or q.get("propagationPolicy") or "Background"
        uid = (body.get("preconditions") or {}).get("uid")
        self.store.delete(kind, ns, name, propagation=prop, expect_uid=uid)
        self._send(200, {"kind": "Status", "apiVersion": "v1", "status": "Success"})


class APIServer(ThreadingHTTPServer):
    daemon_threads = True
    allow_reuse_address = True

    def __init__(self, store: ObjectStore, host: str = "127.0.0.1", port: int = 0):
        super().__init__((host, port), _Handler)
        self.store = store
        self.stopping = threading.Event()
        self._thread: Optional[threading.Thread] = None

    @property
    def url(self) -> str:
        host, port = self.server_address[:2]
        return f"http://{host}:{port}"

    def start(self) -> "APIServer":
        self._thread = threading.Thread(target=self.serve_forever, name="apiserver", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self.stopping.set()
        self.shutdown()
        self.server_close()
