"""Graceful-shutdown signal handling (reference ``pkg/util/signals/signals.go:26-40``).

The first SIGINT/SIGTERM sets the returned stop event; a second one exits
the process with status 1.  Setting the handler up twice is a programming
error (the reference panics).
"""
from __future__ import annotations

import os
import signal
import threading

SHUTDOWN_SIGNALS = (signal.SIGINT, signal.SIGTERM)
_only_once = threading.Lock()
_installed = False


def setup_signal_handler() -> threading.Event:
    global _installed
    with _only_once:
        if _installed:
            raise RuntimeError("setup_signal_handler called twice")
        _installed = True
    stop = threading.Event()

    def handler(signum, frame):
        if stop.is_set():
            os._exit(1)  # second signal: exit directly
        stop.set()

    for s in SHUTDOWN_SIGNALS:
        signal.signal(s, handler)
    return stop


def _reset_for_tests() -> None:
    global _installed
    with _only_once:
        _installed = False
