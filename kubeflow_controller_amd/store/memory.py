"""In-process object store: the apiserver + etcd + garbage collector the
reference delegates to Kubernetes.

Semantics re-created:

* ``uid`` (uuid4), monotonically increasing ``resourceVersion`` shared by all
  kinds, ``creationTimestamp``; ``generateName`` + 5 random chars, retried on
  collision (``VKC/controller_utils.go:502-509``).
* ``update`` with a stale ``resourceVersion`` raises ``Conflict``; an update
  whose wire form is identical to the stored object is a **no-op** that keeps
  the resourceVersion and emits no watch event (the apiserver behaviour the
  reference's hot status loop depends on, SURVEY §3.2 notes).
* ``delete`` cascades to dependents through ``ownerReferences`` (background
  propagation, the k8s GC the reference relies on for cleanup);
  ``propagation="Orphan"`` strips the owner refs instead.
* ``watch`` fan-out with a bounded history so a watcher can resume from a
  resourceVersion (informer relist-free restart).
* TFJobs are defaulted and validated on create/update (``api/validation.py``).
* Optional ``data_dir`` persistence: a JSON snapshot written atomically after
  every mutation and reloaded on start (the etcd role), so a controller restart
  rebuilds its state from the store exactly as the reference rebuilds from
  informers.
"""
from __future__ import annotations

import collections
import json
import os
import queue
import threading
import uuid
from typing import Any, Callable, Dict, Iterable, List, Optional, Tuple

from ..api import serde, v1alpha1
from ..api.labels import Selector
from ..api.meta import generate_name, now_rfc3339
from ..api.model import Model, deep_copy
from ..api.validation import ValidationError, set_defaults, validate
from . import errors

ADDED = "ADDED"
MODIFIED = "MODIFIED"
DELETED = "DELETED"
BOOKMARK = "BOOKMARK"

_HISTORY = 4096


def merge_patch(target: Any, patch: Any) -> Any:
    """RFC 7386 JSON merge patch."""
    if not isinstance(patch, dict):
        return patch
    if not isinstance(target, dict):
        target = {}
    out = dict(target)
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


class Watch:
    """A stream of ``(type, object)`` events; iterate or call ``next(timeout)``."""

    def __init__(self, store: "ObjectStore", kind: Optional[str], namespace: Optional[str],
                 selector: Optional[Selector]):
        self._store = store
        self.kind = kind
        self.namespace = namespace or None
        self.selector = selector or Selector.everything()
        self._q: "queue.Queue[Optional[Tuple[str, Model]]]" = queue.Queue()
        self._stopped = False

    def _offer(self, etype: str, obj: Model) -> None:
        if self._stopped:
            return
        if self.kind and obj.kind != self.kind:
            return
        if self.namespace and obj.metadata.namespace != self.namespace:
            return
        if not self.selector.matches(obj.metadata.labels):
            return
        self._q.put((etype, deep_copy(obj)))

    def next(self, timeout: Optional[float] = None):
        try:
            item = self._q.get(timeout=timeout)
        except queue.Empty:
            return None
        return item

    def stop(self) -> None:
        if not self._stopped:
            self._stopped = True
            self._store._remove_watch(self)
            self._q.put(None)

    @property
    def stopped(self) -> bool:
        return self._stopped

    def __iter__(self):
        while True:
            item = self._q.get()
            if item is None:
                return
            yield item


class ObjectStore:
    """Thread-safe object store keyed by ``(kind, namespace, name)``."""

    def __init__(self, data_dir: Optional[str] = None):
        self._lock = threading.RLock()
        self._objs: Dict[Tuple[str, str, str], Model] = {}
        self._rv = 0
        self._watches: List[Watch] = []
        self._history: "collections.deque[Tuple[int, str, Model]]" = collections.deque(maxlen=_HISTORY)
        self._data_dir = data_dir
        self._crds: Dict[str, Dict] = {v1alpha1.CRD_NAME: v1alpha1.crd_manifest()}
        if data_dir:
            os.makedirs(data_dir, exist_ok=True)
            self._load()

    # ------------------------------------------------------------------ persistence
    def _snapshot_path(self) -> str:
        return os.path.join(self._data_dir, "store.json")  # type: ignore[arg-type]

    def _load(self) -> None:
        p = self._snapshot_path()
        if not os.path.exists(p):
            return
        with open(p) as f:
            data = json.load(f)
        self._rv = int(data.get("resourceVersion", 0))
        for d in data.get("objects", []):
            obj = serde.decode(d)
            self._objs[(obj.kind, obj.metadata.namespace, obj.metadata.name)] = obj
        self._crds.update(data.get("crds", {}))

    def _persist(self) -> None:
        if not self._data_dir:
            return
        p = self._snapshot_path()
        tmp = p + ".tmp"
        data = {"resourceVersion": self._rv, "crds": self._crds,
                "objects": [o.to_json() for o in self._objs.values()]}
        with open(tmp, "w") as f:
            json.dump(data, f)
        os.replace(tmp, p)

    # ------------------------------------------------------------------ helpers
    def _next_rv(self) -> str:
        self._rv += 1
        return str(self._rv)

    @property
    def resource_version(self) -> str:
        with self._lock:
            return str(self._rv)

    def _notify(self, etype: str, obj: Model) -> None:
        self._history.append((int(obj.metadata.resourceVersion or self._rv), etype, deep_copy(obj)))
        for w in list(self._watches):
            w._offer(etype, obj)

    def _remove_watch(self, w: Watch) -> None:
        with self._lock:
            if w in self._watches:
                self._watches.remove(w)

    @staticmethod
    def _wire_without_rv(obj: Model) -> Dict:
        d = obj.to_json()
        d.get("metadata", {}).pop("resourceVersion", None)
        return d

    def _admit(self, obj: Model) -> None:
        if obj.kind == "Pod" and not obj.status.phase:
            obj.status.phase = "Pending"  # apiserver default for a new pod
        if isinstance(obj, v1alpha1.TFJob):
            set_defaults(obj)
            try:
                validate(obj)
            except ValidationError as e:
                raise errors.Invalid(f"TFJob {obj.metadata.name!r} is invalid: {e}") from None

    # ------------------------------------------------------------------ CRD registry
    def register_crd(self, manifest: Dict) -> None:
        with self._lock:
            self._crds[manifest["metadata"]["name"]] = manifest
            self._persist()

    def crds(self) -> Dict[str, Dict]:
        with self._lock:
            return dict(self._crds)

    # ------------------------------------------------------------------ verbs
    def create(self, obj: Model, namespace: Optional[str] = None) -> Model:
        if isinstance(obj, dict):  # CRD registration through the same verb
            self.register_crd(obj)
            return obj
        obj = deep_copy(obj)
        meta = obj.metadata
        meta.namespace = namespace or meta.namespace or "default"
        self._admit(obj)
        with self._lock:
            if not meta.name:
                if not meta.generateName:
                    raise errors.Invalid("metadata.name or metadata.generateName is required")
                for _ in range(16):
                    cand = generate_name(meta.generateName)
                    if (obj.kind, meta.namespace, cand) not in self._objs:
                        meta.name = cand
                        break
                else:
                    raise errors.AlreadyExists(f"could not generate a unique name for {meta.generateName!r}")
            key = (obj.kind, meta.namespace, meta.name)
            if key in self._objs:
                raise errors.AlreadyExists(f'{obj.kind} "{meta.name}" already exists')
            for ref in meta.ownerReferences:
                # the GC would collect a dependent of a vanished owner at once; refuse it up front
                # (closes the stale-cache race of a sync that outlives its TFJob's deletion)
                if ref.controller and not any(o.metadata.uid == ref.uid for o in self._objs.values()):
                    raise errors.NotFound(f'owner {ref.kind} "{ref.name}" (uid {ref.uid}) not found')
            meta.uid = str(uuid.uuid4())
            meta.creationTimestamp = now_rfc3339()
            meta.resourceVersion = self._next_rv()
            meta.deletionTimestamp = None
            self._objs[key] = obj
            self._notify(ADDED, obj)
            self._persist()
            return deep_copy(obj)

    def get(self, kind: str, namespace: str, name: str) -> Model:
        with self._lock:
            obj = self._objs.get((kind, namespace or "default", name))
            if obj is None:
                raise errors.NotFound(f'{kind} "{name}" not found')
            return deep_copy(obj)

    def list(self, kind: str, namespace: Optional[str] = None,
             selector: Optional[Selector] = None) -> List[Model]:
        sel = selector or Selector.everything()
        with self._lock:
            out = [deep_copy(o) for (k, ns, _), o in self._objs.items()
                   if k == kind and (not namespace or ns == namespace) and sel.matches(o.metadata.labels)]
        out.sort(key=lambda o: (o.metadata.namespace, o.metadata.name))
        return out

    def update(self, obj: Model) -> Model:
        obj = deep_copy(obj)
        meta = obj.metadata
        meta.namespace = meta.namespace or "default"
        self._admit(obj)
        with self._lock:
            key = (obj.kind, meta.namespace, meta.name)
            cur = self._objs.get(key)
            if cur is None:
                raise errors.NotFound(f'{obj.kind} "{meta.name}" not found')
            if meta.resourceVersion and meta.resourceVersion != cur.metadata.resourceVersion:
                raise errors.Conflict(
                    f'Operation cannot be fulfilled on {obj.kind} "{meta.name}": the object has been '
                    f"modified; please apply your changes to the latest version and try again")
            # immutable metadata
            meta.uid = cur.metadata.uid
            meta.creationTimestamp = cur.metadata.creationTimestamp
            if cur.metadata.deletionTimestamp and not meta.deletionTimestamp:
                meta.deletionTimestamp = cur.metadata.deletionTimestamp
            if self._wire_without_rv(obj) == self._wire_without_rv(cur):
                return deep_copy(cur)  # identical update: no-op, RV unchanged, no event
            meta.resourceVersion = self._next_rv()
            if meta.deletionTimestamp and not meta.finalizers:
                del self._objs[key]
                self._notify(DELETED, obj)
                self._gc_dependents(meta.uid)
            else:
                self._objs[key] = obj
                self._notify(MODIFIED, obj)
            self._persist()
            return deep_copy(obj)

    def patch(self, kind: str, namespace: str, name: str, patch: Dict,
              expect_uid: Optional[str] = None) -> Model:
        """JSON merge patch; ``expect_uid`` is the uid precondition the ref
        manager embeds in its adopt/release patches (``ref/service.go:123-161``)."""
        with self._lock:
            cur = self.get(kind, namespace, name)
            if expect_uid is not None and cur.metadata.uid != expect_uid:
                raise errors.Conflict(f"uid precondition failed for {kind} {name}")
            merged = merge_patch(cur.to_json(), patch)
            merged.setdefault("metadata", {})["resourceVersion"] = cur.metadata.resourceVersion
            return self.update(type(cur).from_json(merged))

    def update_status(self, obj: Model) -> Model:
        """Status subresource write: only ``status`` of the stored object changes."""
        with self._lock:
            cur = self.get(obj.kind, obj.metadata.namespace, obj.metadata.name)
            cur.status = deep_copy(obj.status)
            return self.update(cur)

    def delete(self, kind: str, namespace: str, name: str, propagation: str = "Background",
               expect_uid: Optional[str] = None) -> None:
        with self._lock:
            key = (kind, namespace or "default", name)
            cur = self._objs.get(key)
            if cur is None:
                raise errors.NotFound(f'{kind} "{name}" not found')
            if expect_uid is not None and cur.metadata.uid != expect_uid:
                raise errors.Conflict(f"uid precondition failed for {kind} {name}")
            if cur.metadata.finalizers:
                if not cur.metadata.deletionTimestamp:
                    cur = deep_copy(cur)
                    cur.metadata.deletionTimestamp = now_rfc3339()
                    cur.metadata.resourceVersion = self._next_rv()
                    self._objs[key] = cur
                    self._notify(MODIFIED, cur)
                    self._persist()
                return
            del self._objs[key]
            gone = deep_copy(cur)
            gone.metadata.deletionTimestamp = gone.metadata.deletionTimestamp or now_rfc3339()
            gone.metadata.resourceVersion = self._next_rv()
            self._notify(DELETED, gone)
            if propagation == "Orphan":
                self._orphan_dependents(cur.metadata.uid)
            else:
                self._gc_dependents(cur.metadata.uid)
            self._persist()

    def _dependents(self, uid: str) -> List[Model]:
        return [o for o in self._objs.values() if any(r.uid == uid for r in o.metadata.ownerReferences)]

    def _gc_dependents(self, uid: str) -> None:
        for dep in self._dependents(uid):
            try:
                self.delete(dep.kind, dep.metadata.namespace, dep.metadata.name)
            except errors.NotFound:
                pass

    def _orphan_dependents(self, uid: str) -> None:
        for dep in self._dependents(uid):
            d = deep_copy(dep)
            d.metadata.ownerReferences = [r for r in d.metadata.ownerReferences if r.uid != uid]
            d.metadata.resourceVersion = ""
            self.update(d)

    def watch(self, kind: Optional[str] = None, namespace: Optional[str] = None,
              selector: Optional[Selector] = None, resource_version: Optional[str] = None) -> Watch:
        w = Watch(self, kind, namespace, selector)
        with self._lock:
            if resource_version:
                since = int(resource_version)
                oldest = self._history[0][0] if self._history else self._rv + 1
                if since < self._rv and since + 1 < oldest:
                    raise errors.StatusError(f"too old resource version: {since} ({oldest})")
                for rv, etype, obj in self._history:
                    if rv > since:
                        w._offer(etype, obj)
            self._watches.append(w)
        return w

    def list_and_rv(self, kind: str, namespace: Optional[str] = None,
                    selector: Optional[Selector] = None) -> Tuple[List[Model], str]:
        with self._lock:
            return self.list(kind, namespace, selector), str(self._rv)

    def dump(self) -> Iterable[Model]:
        with self._lock:
            return [deep_copy(o) for o in self._objs.values()]
