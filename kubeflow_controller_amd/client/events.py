"""Event recorder / broadcaster (``VCG/tools/record/event.go``) and a fake recorder.

* ``EventBroadcaster``: a non-blocking fan-out with a 1000-deep queue that
  drops when full (``event.go:39,43,98-100``); sinks are "log" (the
  ``StartLogging(glog.Infof)`` of ``controller.go:91``) and "store" (write a
  ``v1.Event`` through the clientset, retried up to 12 times, ``event.go:246-300``).
  Identical events (same object, type, reason, message) are aggregated into one
  Event object with an increasing ``count`` — the apiserver-side correlator.
* ``EventRecorder.event(obj, type, reason, message)`` with the source component
  (``kubeflow-controller``, ``controller.go:36``).
* ``FakeRecorder`` collects ``"<type> <reason> <message>"`` strings
  (``VCG/tools/record/fake.go:29-54``).
"""
from __future__ import annotations

import logging
import queue
import threading
import time
import uuid
from typing import Callable, Dict, List, Optional, Tuple

from ..api.core import Event, EventSource, ObjectReference
from ..api.meta import ObjectMeta, now_rfc3339
from ..store import errors

NORMAL = "Normal"
WARNING = "Warning"

_QUEUE_LEN = 1000
_MAX_TRIES = 12

log = logging.getLogger("kfa.events")


def _ref(obj) -> ObjectReference:
    return ObjectReference(kind=obj.kind, namespace=obj.metadata.namespace or "default", name=obj.metadata.name,
                           uid=obj.metadata.uid, apiVersion=getattr(obj, "apiVersion", ""),
                           resourceVersion=obj.metadata.resourceVersion)


class EventBroadcaster:
    def __init__(self):
        self._q: "queue.Queue[Optional[Event]]" = queue.Queue(maxsize=_QUEUE_LEN)
        self._sinks: List[Callable[[Event], None]] = []
        self._thread = threading.Thread(target=self._loop, name="event-broadcaster", daemon=True)
        self._thread.start()
        self.dropped = 0

    def _loop(self):
        while True:
            ev = self._q.get()
            if ev is None:
                return
            for s in list(self._sinks):
                try:
                    s(ev)
                except Exception:
                    log.exception("event sink failed")

    def action(self, ev: Event) -> None:
        try:
            self._q.put_nowait(ev)
        except queue.Full:  # drop, never block the controller
            self.dropped += 1

    def start_logging(self, logf: Callable[[str], None] = None) -> None:
        logf = logf or log.info

        def sink(ev: Event):
            io = ev.involvedObject
            logf(f'Event(v1.ObjectReference{{Kind:"{io.kind}", Namespace:"{io.namespace}", Name:"{io.name}", '
                 f'UID:"{io.uid}"}}): type: \'{ev.type}\' reason: \'{ev.reason}\' {ev.message}')
        self._sinks.append(sink)

    def start_recording_to_sink(self, clientset, sleep: float = 0.01) -> None:
        seen: Dict[Tuple[str, str, str, str], str] = {}
        lock = threading.Lock()

        def sink(ev: Event):
            key = (ev.involvedObject.uid, ev.type, ev.reason, ev.message)
            events = clientset.core_v1().events(ev.metadata.namespace)
            for attempt in range(_MAX_TRIES):
                try:
                    with lock:
                        name = seen.get(key)
                    if name:
                        try:
                            cur = events.get(name)
                            cur.count += 1
                            cur.lastTimestamp = ev.lastTimestamp
                            cur.metadata.resourceVersion = ""
                            events.update(cur)
                            return
                        except errors.NotFound:
                            with lock:
                                seen.pop(key, None)
                    created = events.create(ev)
                    with lock:
                        seen[key] = created.metadata.name
                    return
                except errors.AlreadyExists:
                    return
                except Exception:
                    time.sleep(sleep * (attempt + 1))
            log.error("unable to write event %s/%s after %d tries", ev.reason, ev.message, _MAX_TRIES)
        self._sinks.append(sink)

    def new_recorder(self, component: str) -> "EventRecorder":
        return EventRecorder(self, component)

    def shutdown(self) -> None:
        self._q.put(None)


class EventRecorder:
    def __init__(self, broadcaster: EventBroadcaster, component: str, host: str = ""):
        self.b = broadcaster
        self.source = EventSource(component=component, host=host)

    def event(self, obj, etype: str, reason: str, message: str) -> None:
        ts = now_rfc3339()
        ns = obj.metadata.namespace or "default"
        ev = Event(metadata=ObjectMeta(name=f"{obj.metadata.name}.{uuid.uuid4().hex[:16]}", namespace=ns),
                   involvedObject=_ref(obj), reason=reason, message=message, source=self.source,
                   firstTimestamp=ts, lastTimestamp=ts, count=1, type=etype)
        self.b.action(ev)

    def eventf(self, obj, etype: str, reason: str, fmt: str, *args) -> None:
        self.event(obj, etype, reason, fmt % args if args else fmt)


class FakeRecorder:
    """Test double: records ``"<type> <reason> <message>"``."""

    def __init__(self):
        self.events: List[str] = []
        self._lock = threading.Lock()

    def event(self, obj, etype: str, reason: str, message: str) -> None:
        with self._lock:
            self.events.append(f"{etype} {reason} {message}")

    def eventf(self, obj, etype: str, reason: str, fmt: str, *args) -> None:
        self.event(obj, etype, reason, fmt % args if args else fmt)
