"""Name / runtime-ID generation (reference ``pkg/tensorflow/util.go:19-26``)."""
from ..api.meta import generate_name as _gen


def generate_runtime_id() -> str:
    """``SimpleNameGenerator.GenerateName("")``: 5 random alphanumerics."""
    return _gen("")


def generate_name(base: str) -> str:
    return _gen(base)
