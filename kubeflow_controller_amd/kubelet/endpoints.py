"""Endpoint controller: the kube-proxy / kube-dns role on a single node.

Every Service gets ``clusterIP: 127.0.0.1`` and a host port
(``ports[0].nodePort``) from a port allocator, so the reference's fixed
service port 2222 (``pkg/tensorflow/distributed.go:28``) can appear in every
replica's cluster spec while each replica index still has its own TCP
endpoint.  ``resolve()`` maps ``<service-name>:<port>`` to ``127.0.0.1:<nodePort>``.
"""
from __future__ import annotations

import logging
import socket
import threading
from typing import Dict, Optional

from ..store import errors

log = logging.getLogger("kfa.endpoints")


class PortAllocator:
    def __init__(self, lo: int = 30000, hi: int = 32767, host: str = "127.0.0.1"):
        self.lo, self.hi, self.host = lo, hi, host
        self._used = set()
        self._next = lo
        self._lock = threading.Lock()

    def _free(self, port: int) -> bool:
        for fam, addr in ((socket.AF_INET, (self.host, port)),):
            s = socket.socket(fam, socket.SOCK_STREAM)
            try:
                s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
                s.bind(addr)
            except OSError:
                return False
            finally:
                s.close()
        return True

    def allocate(self) -> int:
        with self._lock:
            span = self.hi - self.lo + 1
            for _ in range(span):
                p = self._next
                self._next = self.lo + (self._next - self.lo + 1) % span
                if p not in self._used and self._free(p):
                    self._used.add(p)
                    return p
        raise RuntimeError("port range exhausted")

    def mark_used(self, port: int) -> None:
        with self._lock:
            self._used.add(port)

    def release(self, port: int) -> None:
        with self._lock:
            self._used.discard(port)


class EndpointController:
    def __init__(self, clientset, service_informer, allocator: Optional[PortAllocator] = None):
        self.client = clientset
        self.allocator = allocator or PortAllocator()
        self.lister = service_informer.lister()
        service_informer.add_event_handler(on_add=self._ensure, on_update=lambda o, n: self._ensure(n),
                                           on_delete=self._release)
        self._lock = threading.Lock()

    def _ensure(self, svc) -> None:
        if svc.spec.ports and svc.spec.ports[0].nodePort:
            self.allocator.mark_used(svc.spec.ports[0].nodePort)
            return
        with self._lock:
            try:
                cur = self.client.core_v1().services(svc.metadata.namespace).get(svc.metadata.name)
            except errors.NotFound:
                return
            if cur.spec.ports and cur.spec.ports[0].nodePort:
                return
            port = self.allocator.allocate()
            cur.spec.clusterIP = "127.0.0.1"
            if not cur.spec.ports:
                from ..api.core import ServicePort
                cur.spec.ports = [ServicePort(name="default", port=port)]
            for sp in cur.spec.ports:
                sp.nodePort = port if sp is cur.spec.ports[0] else (sp.nodePort or self.allocator.allocate())
                sp.targetPort = sp.nodePort
            try:
                self.client.core_v1().services(cur.metadata.namespace).update(cur)
            except (errors.NotFound, errors.Conflict):
                self.allocator.release(port)

    def _release(self, svc) -> None:
        for sp in svc.spec.ports:
            if sp.nodePort:
                self.allocator.release(sp.nodePort)


def service_host_map(services) -> Dict[str, str]:
    """``{"<svc>:<port>": "127.0.0.1:<nodePort>", "<svc>": "127.0.0.1"}`` for every ready service."""
    out: Dict[str, str] = {}
    for s in services:
        if not s.spec.ports or not s.spec.ports[0].nodePort:
            continue
        ip = s.spec.clusterIP or "127.0.0.1"
        out[s.metadata.name] = ip
        for sp in s.spec.ports:
            out[f"{s.metadata.name}:{sp.port}"] = f"{ip}:{sp.nodePort}"
    return out
