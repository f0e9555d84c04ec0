"""Loader for the native control-plane runtime (``csrc/runtime/runtime.cpp``).

The module is built in-tree on first use (g++, ~5 s) when the ``.so`` is
missing or stale, so a fresh checkout works without a separate build step.
There is deliberately no pure-Python fallback: the workqueue, expectations and
process launcher ARE this native module.
"""
from __future__ import annotations

import importlib

_mod = None


def load():
    global _mod
    if _mod is None:
        from .. import _build
        _build.build_runtime()
        _mod = importlib.import_module("kubeflow_controller_amd._native_runtime")
    return _mod


def __getattr__(name):
    return getattr(load(), name)
