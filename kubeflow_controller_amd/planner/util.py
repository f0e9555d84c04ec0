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


# TFJob spec directories the reference accepted but never used (types.go:44-51);
# here they reach every replica as environment variables (checkpoint / resume).
JOB_DIR_ENV = (("modelDir", "KFA_MODEL_DIR"), ("logDir", "KFA_LOG_DIR"), ("dataDir", "KFA_DATA_DIR"),
               ("exportDir", "KFA_EXPORT_DIR"))


def with_job_dirs(tmpl, tfjob):
    """Copy of a pod template whose first container also gets the job's dir env vars."""
    from ..api.core import EnvVar
    from ..api.model import deep_copy
    pairs = [(env, getattr(tfjob.spec, key, "")) for key, env in JOB_DIR_ENV]
    pairs = [(e, v) for e, v in pairs if v]
    if not pairs or not tmpl.spec.containers:
        return tmpl
    out = deep_copy(tmpl)
    c0 = out.spec.containers[0]
    names = {e for e, _ in pairs}
    c0.env = [e for e in c0.env if e.name not in names] + [EnvVar(name=e, value=v) for e, v in pairs]
    return out
