"""Work queue, rate limiters and controller expectations — thin re-exports of
the native C++ runtime (``csrc/runtime/runtime.cpp``).

* ``RateLimitingQueue(rate_limiter=None, name="")``: dedup FIFO; an item is
  never processed by two workers at once (``VCG/util/workqueue/queue.go:33-60``);
  ``add_rate_limited`` = ``add_after(when(item))``.
* ``default_controller_rate_limiter()`` = max(5 ms * 2^n capped at 1000 s per
  item, 10 qps / burst 100 token bucket) (``default_rate_limiters.go:39-45``).
* ``ControllerExpectations(ttl=300)``: ``expect_creations`` OVERWRITES (the
  reference's ``SetExpectations``), ``raise_expectations`` accumulates;
  satisfied when fulfilled, expired (5 min) or absent
  (``VKC/controller_utils.go:136-288``).
* ``set_fake_clock / advance_fake_clock / use_real_clock``: injectable clock
  for TTL / backoff tests (the fake-clock expectations tests of
  ``VKC/controller_utils_test.go:53-60``).
"""
from __future__ import annotations

from ..native import load as _load

_rt = _load()

RateLimitingQueue = _rt.RateLimitingQueue
ItemExponentialFailureRateLimiter = _rt.ItemExponentialFailureRateLimiter
BucketRateLimiter = _rt.BucketRateLimiter
MaxOfRateLimiter = _rt.MaxOfRateLimiter
default_controller_rate_limiter = _rt.default_controller_rate_limiter
ControllerExpectations = _rt.ControllerExpectations
set_fake_clock = _rt.set_fake_clock
advance_fake_clock = _rt.advance_fake_clock
use_real_clock = _rt.use_real_clock
now = _rt.now

EXPECTATIONS_TIMEOUT = 5 * 60.0

__all__ = ["RateLimitingQueue", "ItemExponentialFailureRateLimiter", "BucketRateLimiter", "MaxOfRateLimiter",
           "default_controller_rate_limiter", "ControllerExpectations", "EXPECTATIONS_TIMEOUT",
           "set_fake_clock", "advance_fake_clock", "use_real_clock", "now"]
