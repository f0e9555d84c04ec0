"""REST client for ``store/apiserver.py`` with the ``ObjectStore`` interface.

``RESTStore(url)`` and ``ObjectStore()`` are interchangeable behind the
clientset (``client/clientset.py``), the way client-go's REST client and a fake
clientset are interchangeable behind ``kubernetes.Interface``.
"""
from __future__ import annotations

import http.client
import json
import queue
import threading
from typing import Dict, List, Optional, Tuple
from urllib.parse import quote, urlencode, urlparse

from ..api import serde, v1alpha1
from ..api.labels import Selector
from ..api.model import Model
from . import errors

_PLURAL = {v1alpha1.TFJOB_KIND: v1alpha1.TFJOB_PLURAL, "Pod": "pods", "Service": "services", "Event": "events",
           "ReplicaSet": "replicasets"}


def _path(kind: str, ns: Optional[str], name: Optional[str] = None, sub: Optional[str] = None) -> str:
    base = (f"/apis/{v1alpha1.GROUP_NAME}/{v1alpha1.GROUP_VERSION}" if kind == v1alpha1.TFJOB_KIND
            else "/apis/extensions/v1beta1" if kind == "ReplicaSet" else "/api/v1")
    p = base + (f"/namespaces/{quote(ns)}" if ns else "") + "/" + _PLURAL[kind]
    if name:
        p += "/" + quote(name)
    if sub:
        p += "/" + sub
    return p


class RESTWatch:
    def __init__(self, conn: http.client.HTTPConnection, resp: http.client.HTTPResponse):
        self._conn = conn
        self._resp = resp
        self._q: "queue.Queue" = queue.Queue()
        self._stopped = False
        self.last_rv: Optional[str] = None
        self._t = threading.Thread(target=self._pump, daemon=True, name="rest-watch")
        self._t.start()

    def _pump(self):
        try:
            while not self._stopped:
                line = self._resp.readline()
                if not line:
                    break
                ev = json.loads(line)
                if ev["type"] == "BOOKMARK":
                    self.last_rv = ev["object"]["metadata"]["resourceVersion"]
                    continue
                obj = serde.decode(ev["object"])
                self.last_rv = obj.metadata.resourceVersion
                self._q.put((ev["type"], obj))
        except Exception:  # connection closed
            pass
        finally:
            self._stopped = True
            self._q.put(None)

    @property
    def stopped(self) -> bool:
        return self._stopped and self._q.empty()

    def next(self, timeout: Optional[float] = None):
        try:
            return self._q.get(timeout=timeout)
        except queue.Empty:
            return None

    def stop(self):
        self._stopped = True
        try:
            self._conn.sock and self._conn.sock.shutdown(2)
        except OSError:
            pass
        self._conn.close()

    def __iter__(self):
        while True:
            item = self._q.get()
            if item is None:
                return
            yield item


class RESTStore:
    def __init__(self, url: str, timeout: float = 30.0):
        u = urlparse(url if "://" in url else "http://" + url)
        self.host = u.hostname or "127.0.0.1"
        self.port = u.port or 80
        self.timeout = timeout
        self._local = threading.local()

    # -------------------------------------------------------------- transport
    def _conn(self) -> http.client.HTTPConnection:
        c = getattr(self._local, "conn", None)
        if c is None:
            c = http.client.HTTPConnection(self.host, self.port, timeout=self.timeout)
            self._local.conn = c
        return c

    def _do(self, method: str, path: str, body=None, ctype="application/json"):
        data = None if body is None else json.dumps(body).encode()
        headers = {"Content-Type": ctype} if data is not None else {}
        for attempt in range(2):
            c = self._conn()
            try:
                c.request(method, path, body=data, headers=headers)
                resp = c.getresponse()
                raw = resp.read()
                break
            except (ConnectionError, http.client.HTTPException, OSError):
                c.close()
                self._local.conn = None
                if attempt:
                    raise
        payload = json.loads(raw) if raw else {}
        if resp.status >= 400:
            raise errors.from_status(payload)
        return payload

    # -------------------------------------------------------------- verbs
    def create(self, obj, namespace: Optional[str] = None):
        if isinstance(obj, dict):
            return self._do("POST", "/apis/apiextensions.k8s.io/v1beta1/customresourcedefinitions", obj)
        ns = namespace or obj.metadata.namespace or "default"
        return serde.decode(self._do("POST", _path(obj.kind, ns), obj.to_json()))

    def get(self, kind: str, namespace: str, name: str) -> Model:
        return serde.decode(self._do("GET", _path(kind, namespace or "default", name)))

    def list_and_rv(self, kind: str, namespace: Optional[str] = None,
                    selector: Optional[Selector] = None) -> Tuple[List[Model], str]:
        q = {"labelSelector": str(selector)} if selector is not None and not selector.empty() else {}
        p = _path(kind, namespace) + ("?" + urlencode(q) if q else "")
        d = self._do("GET", p)
        return [serde.decode(x) for x in d.get("items", [])], d.get("metadata", {}).get("resourceVersion", "")

    def list(self, kind: str, namespace: Optional[str] = None, selector: Optional[Selector] = None):
        return self.list_and_rv(kind, namespace, selector)[0]

    def update(self, obj: Model) -> Model:
        ns = obj.metadata.namespace or "default"
        return serde.decode(self._do("PUT", _path(obj.kind, ns, obj.metadata.name), obj.to_json()))

    def update_status(self, obj: Model) -> Model:
        ns = obj.metadata.namespace or "default"
        return serde.decode(self._do("PUT", _path(obj.kind, ns, obj.metadata.name, "status"), obj.to_json()))

    def patch(self, kind: str, namespace: str, name: str, patch: Dict, expect_uid: Optional[str] = None):
        body = dict(patch)
        if expect_uid is not None:
            body.setdefault("metadata", {})
            body["metadata"] = dict(body["metadata"], uid=expect_uid)
        return serde.decode(self._do("PATCH", _path(kind, namespace or "default", name), body,
                                     ctype="application/merge-patch+json"))

    def delete(self, kind: str, namespace: str, name: str, propagation: str = "Background",
               expect_uid: Optional[str] = None) -> None:
        body = {"propagationPolicy": propagation}
        if expect_uid is not None:
            body["preconditions"] = {"uid": expect_uid}
        self._do("DELETE", _path(kind, namespace or "default", name), body)

    def watch(self, kind: Optional[str] = None, namespace: Optional[str] = None,
              selector: Optional[Selector] = None, resource_version: Optional[str] = None) -> RESTWatch:
        q = {"watch": "true"}
        if resource_version:
            q["resourceVersion"] = resource_version
        if selector is not None and not selector.empty():
            q["labelSelector"] = str(selector)
        conn = http.client.HTTPConnection(self.host, self.port, timeout=None)
        conn.request("GET", _path(kind, namespace) + "?" + urlencode(q))
        resp = conn.getresponse()
        if resp.status >= 400:
            raise errors.from_status(json.loads(resp.read() or b"{}"))
        return RESTWatch(conn, resp)

    def crds(self) -> Dict[str, Dict]:
        d = self._do("GET", "/apis/apiextensions.k8s.io/v1beta1/customresourcedefinitions")
        return {c["metadata"]["name"]: c for c in d.get("items", [])}

    def register_crd(self, manifest: Dict) -> None:
        self.create(manifest)

    @property
    def resource_version(self) -> str:
        return self.list_and_rv("Event", None)[1]
