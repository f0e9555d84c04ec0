"""Controller-ref managers: claim / adopt / release children.

Reference: ``pkg/controller/ref/base.go:26-112`` (generic ``claimObject``),
``ref/service.go:33-161`` (Services) and the upstream Pod manager
``VKC/controller_ref_manager.go:67-240`` (``ClaimPods``), with the
``RecheckDeletionTimestamp`` ``canAdopt`` guard (``:373-386``) memoised once
per manager (the ``sync.Once`` of ``base.go:35-42``).

Rules of ``claim_object``:

* owned by another controller      -> ignore
* owned by us, selector matches     -> keep
* owned by us, mismatch             -> release (unless we are being deleted)
* orphan, matches, neither deleting -> adopt (patch in our controller ref,
  guarded by a uid precondition and by ``can_adopt``)

Adopt/release are JSON merge patches of ``metadata.ownerReferences`` carrying
the child's uid as precondition (the reference uses strategic-merge patches
with ``$patch: delete``; merge patches need the full list, which we send).
"""
from __future__ import annotations

import threading
from typing import Callable, List, Optional

from ..api.labels import Selector
from ..api.meta import OwnerReference, get_controller_of
from ..api.model import to_json
from ..store import errors


class _Base:
    def __init__(self, controller, selector: Selector, controller_kind: str, api_version: str,
                 can_adopt: Optional[Callable[[], None]] = None):
        self.controller = controller
        self.selector = selector
        self.controller_kind = controller_kind
        self.api_version = api_version
        self._can_adopt_fn = can_adopt
        self._once = threading.Lock()
        self._done = False
        self._err: Optional[Exception] = None

    def can_adopt(self) -> None:
        with self._once:
            if not self._done:
                self._done = True
                if self._can_adopt_fn is not None:
                    try:
                        self._can_adopt_fn()
                    except Exception as e:  # noqa: BLE001
                        self._err = e
        if self._err is not None:
            raise self._err

    def claim_object(self, obj, match: Callable, adopt: Callable, release: Callable) -> bool:
        ref = get_controller_of(obj)
        if ref is not None:
            if ref.uid != self.controller.metadata.uid:
                return False
            if match(obj):
                return True
            if self.controller.metadata.deletionTimestamp is not None:
                return False
            try:
                release(obj)
            except errors.NotFound:
                return False
            return False
        if self.controller.metadata.deletionTimestamp is not None or not match(obj):
            return False
        if obj.metadata.deletionTimestamp is not None:
            return False
        try:
            adopt(obj)
        except errors.NotFound:
            return False
        return True

    def _controller_ref(self) -> OwnerReference:
        return OwnerReference(apiVersion=self.api_version, kind=self.controller_kind,
                              name=self.controller.metadata.name, uid=self.controller.metadata.uid,
                              controller=True, blockOwnerDeletion=True)

    def _adopt_patch(self, obj):
        refs = [to_json(r) for r in obj.metadata.ownerReferences] + [to_json(self._controller_ref())]
        return {"metadata": {"ownerReferences": refs}}

    def _release_patch(self, obj):
        refs = [to_json(r) for r in obj.metadata.ownerReferences if r.uid != self.controller.metadata.uid]
        return {"metadata": {"ownerReferences": refs}}


class PodControllerRefManager(_Base):
    def __init__(self, pod_control, controller, selector, controller_kind, api_version, can_adopt=None):
        super().__init__(controller, selector, controller_kind, api_version, can_adopt)
        self.pod_control = pod_control

    def claim_pods(self, pods: List, *filters: Callable) -> List:
        claimed, errs = [], []

        def match(p):
            return self.selector.matches(p.metadata.labels) and all(f(p) for f in filters)

        for p in pods:
            try:
                if self.claim_object(p, match, self.adopt_pod, self.release_pod):
                    claimed.append(p)
            except Exception as e:  # aggregate like utilerrors.NewAggregate
                errs.append(e)
        if errs:
            raise errs[0]
        return claimed

    def adopt_pod(self, pod) -> None:
        self.can_adopt()
        self.pod_control.patch_pod(pod.metadata.namespace, pod.metadata.name, self._adopt_patch(pod),
                                   expect_uid=pod.metadata.uid)

    def release_pod(self, pod) -> None:
        try:
            self.pod_control.patch_pod(pod.metadata.namespace, pod.metadata.name, self._release_patch(pod),
                                       expect_uid=pod.metadata.uid)
        except (errors.NotFound, errors.Conflict):
            # already gone, or re-created with a new uid: nothing to release
            pass


class ServiceControllerRefManager(_Base):
    def __init__(self, service_control, controller, selector, controller_kind, api_version, can_adopt=None):
        super().__init__(controller, selector, controller_kind, api_version, can_adopt)
        self.service_control = service_control

    def claim_services(self, services: List, *filters: Callable) -> List:
        claimed, errs = [], []

        def match(s):
            return self.selector.matches(s.metadata.labels) and all(f(s) for f in filters)

        for s in services:
            try:
                if self.claim_object(s, match, self.adopt_service, self.release_service):
                    claimed.append(s)
            except Exception as e:
                errs.append(e)
        if errs:
            raise errs[0]
        return claimed

    def adopt_service(self, svc) -> None:
        self.can_adopt()
        self.service_control.patch_service(svc.metadata.namespace, svc.metadata.name, self._adopt_patch(svc),
                                           expect_uid=svc.metadata.uid)

    def release_service(self, svc) -> None:
        try:
            self.service_control.patch_service(svc.metadata.namespace, svc.metadata.name,
                                               self._release_patch(svc), expect_uid=svc.metadata.uid)
        except (errors.NotFound, errors.Conflict):
            pass


def recheck_deletion_timestamp(get_object: Callable):
    """``RecheckDeletionTimestamp``: a fresh (quorum) read must not be deleting."""
    def fn():
        obj = get_object()
        if obj.metadata.deletionTimestamp is not None:
            raise RuntimeError(f"{obj.metadata.namespace}/{obj.metadata.name} has just been deleted at "
                               f"{obj.metadata.deletionTimestamp}")
    return fn
