"""Side stream for weight-gradient kernels.

Weight gradients (the BERT encoder's dense wgrads) depend on the
layer's input and output gradient but nothing downstream of the backward pass
waits for them except the gradient buckets and the optimizer.  They are
launched on a per-device side stream, concurrently with the data-gradient
chain on the main stream (dgrad GEMMs, BatchNorm / LayerNorm / attention
backward), and filled into the CUs those kernels leave idle.

Ordering contract:

* ``run_on_side`` makes the side stream wait for everything already queued on
  the current stream, and records the operand tensors on the side stream so
  the caching allocator does not hand their memory to the main stream early;
* ``join`` makes the current stream wait for the side stream — called by the
  gradient-bucket launcher (``parallel/ddp.py``) before a collective reads a
  bucket, and automatically at the end of every backward pass that used the
  side stream (an autograd engine callback), so ``loss.backward()`` returns
  with the main stream ordered after every weight gradient.

Off by default since round 3 (env ``KFA_SIDE_STREAM=1`` turns it on): with the
projections on the persistent GEMM (one 128 KB-LDS block per CU, ``gemm_ppp``) a
co-running wgrad holds CUs the persistent grid expects to own, and one stream
measured faster — BERT-base 8,444-8,466 vs 8,410-8,442 seq/s (same box, 3
rounds).  (Round 1, hipBLASLt projections: +1.5 % with the side stream.)
ResNet-50 conv wgrads never used it (9223 -> 9200 img/s: the dgrad convs
already fill the CUs).
"""
from __future__ import annotations

import os
from typing import Callable, Dict, Iterable

import torch

ENABLED = os.environ.get("KFA_SIDE_STREAM", "0") == "1"
_side: Dict[int, torch.cuda.Stream] = {}


def enabled(t: torch.Tensor) -> bool:
    return ENABLED and t.is_cuda


def side_stream(dev: torch.device) -> torch.cuda.Stream:
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _side.get(idx)
    if s is None:
        s = _side[idx] = torch.cuda.Stream(torch.device("cuda", idx))
    return s


def join(dev=None) -> None:
    """Current stream waits for the side stream(s) (of ``dev``, or all)."""
    if dev is not None and not isinstance(dev, torch.device):
        dev = torch.device(dev)
    for idx, s in _side.items():
        if dev is None or dev.type != "cuda" or dev.index in (None, idx):
            torch.cuda.current_stream(torch.device("cuda", idx)).wait_stream(s)


def _end_of_backward() -> None:
    join()


def run_on_side(fn: Callable, device: torch.device, tensors: Iterable[torch.Tensor] = ()):
    """``fn()`` on the side stream of ``device``, after the current stream's queued work."""
    main = torch.cuda.current_stream(device)
    side = side_stream(device)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        out = fn()
    for t in tensors:
        if t is not None and t.is_cuda:
            t.record_stream(side)
    # One join per side-stream launch, queued on THIS backward's graph task: no
    # process-wide "already queued" flag that a backward which raised (and so
    # never ran its callbacks) could leave set for the next one.  A join is an
    # event record + wait, so the extra ones cost nothing measurable.
    try:
        torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
    except RuntimeError:  # not inside a backward pass: join right away
        main.wait_stream(side)
    return out
