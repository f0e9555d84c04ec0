"""Shared informers and listers.

Reference: ``VCS/informers/externalversions/kubeflow/v1alpha1/tfjob.go:35-88``,
``VCS/listers/kubeflow/v1alpha1/tfjob.go:28-93``, the shared informer factory
(``factory.go:48-130``) and ``VCG/tools/cache/shared_informer.go``.

Behaviour:
* LIST then WATCH from the list's resourceVersion; on a broken watch, re-list
  and re-watch (emitting synthetic update/delete events for the diff).
* ``resync_period`` re-delivers every cached object to ``on_update(old, new)``
  with ``old is new`` content — the reference's UpdateFunc filters those by
  comparing resourceVersions (``controller.go:124-135``).
* Listers return DEEP COPIES.  The reference mutates the shared cache
  (SURVEY §3.3 quirk 5, §5.2 latent race); here a caller can never alias it.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Callable, Dict, List, Optional

from ..api.labels import Selector
from ..api.model import Model, deep_copy
from ..store import errors
from ..store.memory import ADDED, DELETED, MODIFIED

log = logging.getLogger("kfa.informer")


class Handler:
    def __init__(self, on_add: Optional[Callable] = None, on_update: Optional[Callable] = None,
                 on_delete: Optional[Callable] = None):
        self.on_add = on_add
        self.on_update = on_update
        self.on_delete = on_delete


class Lister:
    def __init__(self, informer: "SharedInformer"):
        self._inf = informer

    def get(self, namespace: str, name: str) -> Model:
        obj = self._inf._get(f"{namespace or 'default'}/{name}")
        if obj is None:
            raise errors.NotFound(f'{self._inf.kind} "{name}" not found')
        return deep_copy(obj)

    def list(self, namespace: Optional[str] = None, selector: Optional[Selector] = None) -> List[Model]:
        sel = selector or Selector.everything()
        return [deep_copy(o) for o in self._inf._items()
                if (not namespace or o.metadata.namespace == namespace) and sel.matches(o.metadata.labels)]


class SharedInformer:
    def __init__(self, store, kind: str, namespace: Optional[str] = None, resync_period: float = 30.0):
        self.store = store
        self.kind = kind
        self.namespace = namespace
        self.resync_period = resync_period
        self._cache: Dict[str, Model] = {}
        self._lock = threading.RLock()
        self._handlers: List[Handler] = []
        self._synced = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._stop: Optional[threading.Event] = None
        self._watch = None

    # ------------------------------------------------------------------ public
    def add_event_handler(self, on_add=None, on_update=None, on_delete=None) -> None:
        h = Handler(on_add, on_update, on_delete)
        with self._lock:
            self._handlers.append(h)
            existing = list(self._cache.values())
        if self._synced.is_set() and on_add:
            for o in existing:
                on_add(deep_copy(o))

    def lister(self) -> Lister:
        return Lister(self)

    def has_synced(self) -> bool:
        return self._synced.is_set()

    def run(self, stop: threading.Event) -> None:
        self._stop = stop
        self._thread = threading.Thread(target=self._loop, name=f"informer-{self.kind}", daemon=True)
        self._thread.start()

    def wait_for_sync(self, timeout: Optional[float] = None) -> bool:
        return self._synced.wait(timeout)

    # ------------------------------------------------------------------ internals
    @staticmethod
    def _key(o: Model) -> str:
        return f"{o.metadata.namespace}/{o.metadata.name}"

    def _get(self, key: str) -> Optional[Model]:
        with self._lock:
            return self._cache.get(key)

    def _items(self) -> List[Model]:
        with self._lock:
            return list(self._cache.values())

    def _dispatch(self, etype: str, old: Optional[Model], new: Optional[Model]) -> None:
        for h in list(self._handlers):
            try:
                if etype == ADDED and h.on_add:
                    h.on_add(deep_copy(new))
                elif etype == MODIFIED and h.on_update:
                    h.on_update(deep_copy(old), deep_copy(new))
                elif etype == DELETED and h.on_delete:
                    h.on_delete(deep_copy(old if new is None else new))
            except Exception:  # runtime.HandleCrash: log and keep the informer alive
                log.exception("informer %s handler failed", self.kind)

    def _relist(self) -> str:
        items, rv = self.store.list_and_rv(self.kind, self.namespace)
        fresh = {self._key(o): o for o in items}
        with self._lock:
            old = self._cache
            self._cache = fresh
        for k, o in fresh.items():
            if k not in old:
                self._dispatch(ADDED, None, o)
            elif old[k].metadata.resourceVersion != o.metadata.resourceVersion:
                self._dispatch(MODIFIED, old[k], o)
        for k, o in old.items():
            if k not in fresh:
                self._dispatch(DELETED, o, None)
        return rv

    def _apply(self, etype: str, obj: Model) -> None:
        k = self._key(obj)
        with self._lock:
            old = self._cache.get(k)
            if etype == DELETED:
                self._cache.pop(k, None)
            else:
                self._cache[k] = obj
        if etype == ADDED and old is not None:
            etype = MODIFIED
        if etype == MODIFIED and old is None:
            etype = ADDED
        self._dispatch(etype, old, obj)

    def _resync(self) -> None:
        for o in self._items():
            self._dispatch(MODIFIED, o, o)

    def _loop(self) -> None:
        stop = self._stop
        backoff = 0.1
        while not stop.is_set():
            try:
                rv = self._relist()
                self._synced.set()
                self._watch = self.store.watch(self.kind, self.namespace, None, rv)
                backoff = 0.1
                next_resync = time.monotonic() + self.resync_period if self.resync_period else None
                while not stop.is_set():
                    item = self._watch.next(timeout=0.2)
                    if item is not None:
                        self._apply(*item)
                    elif getattr(self._watch, "stopped", False):
                        break
                    if next_resync is not None and time.monotonic() >= next_resync:
                        self._resync()
                        next_resync = time.monotonic() + self.resync_period
            except Exception as e:  # broken watch / apiserver restart: relist
                log.debug("informer %s: %s; relisting", self.kind, e)
                stop.wait(backoff)
                backoff = min(backoff * 2, 5.0)
            finally:
                w, self._watch = self._watch, None
                if w is not None:
                    try:
                        w.stop()
                    except Exception:
                        pass


class SharedInformerFactory:
    """``NewSharedInformerFactory(client, resync)`` (``cmd/controller/main.go:46-47``)."""

    def __init__(self, store, resync_period: float = 30.0, namespace: Optional[str] = None):
        self.store = store
        self.resync_period = resync_period
        self.namespace = namespace
        self._informers: Dict[str, SharedInformer] = {}
        self._started = set()

    def informer_for(self, kind: str) -> SharedInformer:
        if kind not in self._informers:
            self._informers[kind] = SharedInformer(self.store, kind, self.namespace, self.resync_period)
        return self._informers[kind]

    def tfjobs(self) -> SharedInformer:
        return self.informer_for("TFJob")

    def pods(self) -> SharedInformer:
        return self.informer_for("Pod")

    def services(self) -> SharedInformer:
        return self.informer_for("Service")

    def start(self, stop: threading.Event) -> None:
        for k, inf in self._informers.items():
            if k not in self._started:
                inf.run(stop)
                self._started.add(k)

    def wait_for_cache_sync(self, timeout: Optional[float] = None) -> bool:
        deadline = None if timeout is None else time.monotonic() + timeout
        for inf in self._informers.values():
            rem = None if deadline is None else max(0.0, deadline - time.monotonic())
            if not inf.wait_for_sync(rem):
                return False
        return True
