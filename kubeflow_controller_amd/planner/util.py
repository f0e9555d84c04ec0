"""Name / runtime-ID generation (reference ``pkg/tensorflow/util.go:19-26``)."""
from ..api.meta import generate_name as _gen


def generate_runtime_id(uid: str = "") -> str:
    """5 alphanumerics, like ``SimpleNameGenerator.GenerateName("")``.

    Derived deterministically from the TFJob's UID when there is one: a sync
    that reads a TFJob from a cache that has not yet seen the controller's own
    write (runtimeID still empty) then mints the SAME id, instead of a new one
    that would orphan every replica."""
    if not uid:
        return _gen("")
    import hashlib
    from ..api.meta import _ALPHANUMS
    h = int(hashlib.sha256(uid.encode()).hexdigest(), 16)
    out = []
    for _ in range(5):
        h, r = divmod(h, len(_ALPHANUMS))
        out.append(_ALPHANUMS[r])
    return "".join(out)


def generate_name(base: str) -> str:
    return _gen(base)
