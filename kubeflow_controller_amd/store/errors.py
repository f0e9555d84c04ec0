"""API status errors (``k8s.io/apimachinery/pkg/api/errors`` equivalents)."""
from __future__ import annotations


class StatusError(Exception):
    code = 500
    reason = "InternalError"

    def __init__(self, message: str = ""):
        super().__init__(message or self.reason)
        self.message = message or self.reason

    def to_json(self):
        return {"kind": "Status", "apiVersion": "v1", "status": "Failure",
                "message": self.message, "reason": self.reason, "code": self.code}


class NotFound(StatusError):
    code = 404
    reason = "NotFound"


class AlreadyExists(StatusError):
    code = 409
    reason = "AlreadyExists"


class Conflict(StatusError):
    code = 409
    reason = "Conflict"


class Invalid(StatusError):
    code = 422
    reason = "Invalid"


class BadRequest(StatusError):
    code = 400
    reason = "BadRequest"


class Timeout(StatusError):
    code = 504
    reason = "Timeout"


_BY_REASON = {c.reason: c for c in (NotFound, AlreadyExists, Conflict, Invalid, BadRequest, Timeout)}


def from_status(d) -> StatusError:
    cls = _BY_REASON.get(d.get("reason"), StatusError)
    return cls(d.get("message", ""))


def is_not_found(e) -> bool:
    return isinstance(e, NotFound)


def is_already_exists(e) -> bool:
    return isinstance(e, AlreadyExists)


def is_conflict(e) -> bool:
    return isinstance(e, Conflict)


def is_timeout(e) -> bool:
    return isinstance(e, Timeout)
